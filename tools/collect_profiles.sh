#!/bin/bash
# rocprofv3 evidence for the bench kernels, per round: kernel-trace stats of the bench
# command (both workloads + the LR-TS update), then separate PMC passes (MI355X_MICROARCH.md:
# FETCH_SIZE costs 3 TCC slots, WRITE_SIZE 2 -> not in one pass) for the headline kernel
# (SP_Oracle-shaped) and for the SP_Truthful_TS kernel, plus the SQ instruction mix.
# Usage (on the GPU box): bash tools/collect_profiles.sh <round tag>
set -u
TAG=${1:-r01}
OUT=gpurun_out/prof_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
HEAD="python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-ts --no-populations"
TS="python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-update --no-populations"
HK='k_simulate<2, 6, true, 1, false>'
TK='k_simulate<2, 6, true, 1, true>'
step() { local name=$1; shift; echo "== $name"; timeout -k 10 400 "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "rc=$rc"; if [ $rc -ge 124 ]; then exit $rc; fi; }
step fetch rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$HK" --output-format csv -d "$OUT/fetch" -o run -- $HEAD
step write rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$HK" --output-format csv -d "$OUT/write" -o run -- $HEAD
step ts_fetch rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$TK" --output-format csv -d "$OUT/ts_fetch" -o run -- $TS
step ts_write rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$TK" --output-format csv -d "$OUT/ts_write" -o run -- $TS
step sq rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_FMA_F64 --kernel-include-regex "$HK" --output-format csv -d "$OUT/sq" -o run -- $HEAD
step sq2 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE --kernel-include-regex "$HK" --output-format csv -d "$OUT/sq2" -o run -- $HEAD
# last: the whole bench command incl. the cooperative LR-TS training launch (rocprofv3 has
# crashed in its exit handler after writing the results of this command)
step stats rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/stats" -o run -- python bench.py --no-cpu-baseline
echo "== done"
