#!/bin/bash
# PMC passes for k_oracle on the headline workload (2^24 auctions, 10 launches after warm-up).
set -u
TAG=${1:-pmc}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
CMD="python bench.py --steps 10 --warmup 60 --no-cpu-baseline --no-ts --no-populations --no-generate --batch 16777216"
K='k_oracle<2, 6, false>'
step() { local name=$1; shift; timeout -s KILL 120 "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi; }
step sq rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_FMA_F64 --kernel-include-regex "$K" --output-format csv -d "$OUT/sq" -o run -- $CMD
step sq2 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE --kernel-include-regex "$K" --output-format csv -d "$OUT/sq2" -o run -- $CMD
step fetch rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$K" --output-format csv -d "$OUT/fetch" -o run -- $CMD
step write rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$K" --output-format csv -d "$OUT/write" -o run -- $CMD
python tools/summarize_pmc.py "$OUT" > "$OUT/summary.txt" 2>&1; cat "$OUT/summary.txt"
