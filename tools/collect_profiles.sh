#!/bin/bash
# rocprofv3 evidence for the bench kernel, per round: kernel-trace stats of the bench
# command, then separate PMC passes for FETCH_SIZE and WRITE_SIZE (MI355X_MICROARCH.md:
# FETCH_SIZE costs 3 TCC slots, WRITE_SIZE 2 -> not in one pass) and SQ instruction mix.
# Usage (on the GPU box): bash tools/collect_profiles.sh <round tag>
set -u
TAG=${1:-r01}
OUT=gpurun_out/prof_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
CMD="python bench.py --steps 10 --warmup 2 --no-cpu-baseline"
step() { local name=$1; shift; echo "== $name"; timeout -k 10 400 "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "rc=$rc"; if [ $rc -ge 124 ]; then exit $rc; fi; }
step stats rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/stats" -o run -- $CMD
step fetch rocprofv3 --pmc FETCH_SIZE --kernel-include-regex k_simulate --output-format csv -d "$OUT/fetch" -o run -- $CMD
step write rocprofv3 --pmc WRITE_SIZE --kernel-include-regex k_simulate --output-format csv -d "$OUT/write" -o run -- $CMD
step sq rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_FMA_F64 --kernel-include-regex k_simulate --output-format csv -d "$OUT/sq" -o run -- $CMD
step sq2 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE --kernel-include-regex k_simulate --output-format csv -d "$OUT/sq2" -o run -- $CMD
echo "== done"
