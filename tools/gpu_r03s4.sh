#!/bin/bash
# r03s4: driver-shaped bench, SQ counters of the general simulate kernel on configs_1..3,
# then (last: rocprofv3 faults in its exit path after a cooperative launch) one trainer PMC pass.
# Usage: bash tools/gpu_r03s4.sh <trainer counter set: T1|T2|T3>
set -u
TS=${1:-T1}
OUT=gpurun_out/prof_r03s4
mkdir -p "$OUT"
export TMPDIR=/tmp
pop() { echo "python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-ts --no-update --no-generate --no-p8 --batch 1048576 --populations $1"; }
TSL="python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-update --no-populations --no-generate --no-p8 --batch 1048576"
UPD="python bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-ts --no-generate --no-p8 --batch 1048576 --populations configs_2"
step() { local name=$1 secs=$2; shift 2; echo "== $name"; timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "rc=$rc"; tail -n 2 "$OUT/$name.log" | cut -c1-300; if [ $rc -ne 0 ]; then exit $rc; fi; }
SQA="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_FMA_F64"
SQB="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE"
T1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64"
T2="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE"
T3="SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_VALU_FMA_F32"
if [ "${SKIP_BENCH:-0}" = 0 ]; then
step bench_driver 300 python bench.py --steps 20 --warmup 5
for c in 1 2 3; do
  if [ $c = 1 ]; then CMD=$TSL; else CMD=$(pop configs_$c); fi
  for p in A B; do
    eval "CTR=\$SQ$p"
    step c${c}_sq$p 150 rocprofv3 --pmc $CTR --kernel-include-regex "k_simulate" --output-format csv -d "$OUT/c${c}_sq$p" -o run -- $CMD
  done
done
fi
eval "CTR=\$$TS"
echo "== trainer_$TS (last: the profiler's exit path faults after cooperative launches, results written first)"
timeout -k 10 200 rocprofv3 --pmc $CTR --kernel-include-regex "k_bidder_train|k_lrts_train" --output-format csv -d "$OUT/trainer_$TS" -o run -- $UPD > "$OUT/trainer_$TS.log" 2>&1
echo "rc=$?"
ls "$OUT/trainer_$TS"
echo "== done"
