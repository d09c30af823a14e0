#!/bin/bash
# r03d: per-kernel times (rocprofv3 kernel trace) of every population line with the split
# pass, and SQ counters of k_ts_choice / k_pop on configs_1 and configs_4.
set -u
TAG=${1:-r03d}
OUT=gpurun_out/prof_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
pop() { echo "python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-ts --no-update --no-generate --batch 1048576 --populations $1"; }
TS="python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-update --no-populations --no-generate --batch 1048576"
step() { local name=$1 secs=$2; shift 2; echo "== $name"; timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "rc=$rc"; tail -n 2 "$OUT/$name.log" | cut -c1-300; if [ $rc -ne 0 ]; then exit $rc; fi; }
SQA="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_FMA_F64"
SQB="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE"
step c1_trace 150 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/c1_trace" -o run -- $TS
for c in 2 3 4; do step c${c}_trace 150 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/c${c}_trace" -o run -- $(pop configs_$c); done
for p in A B; do
  eval "CTR=\$SQ$p"
  step c1_sq$p 150 rocprofv3 --pmc $CTR --kernel-include-regex "k_ts_choice|k_pop" --output-format csv -d "$OUT/c1_sq$p" -o run -- $TS
  step c4_sq$p 150 rocprofv3 --pmc $CTR --kernel-include-regex "k_ts_choice|k_pop" --output-format csv -d "$OUT/c4_sq$p" -o run -- $(pop configs_4)
done
echo "== done"
