#!/bin/bash
# r03a: driver-shaped bench on this round's first box, then the SQ counter passes of the
# general simulate kernel for every population line (configs_1..4): instruction mix, wave
# cycles / waits / LDS conflicts, scalar + F64 mix. Usage: bash tools/gpu_r03a.sh <tag>
set -u
TAG=${1:-r03a}
OUT=gpurun_out/prof_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
pop() { echo "python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-ts --no-update --no-generate --batch 1048576 --populations $1"; }
TS="python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-update --no-populations --no-generate --batch 1048576"
GK='k_simulate'
step() { local name=$1 secs=$2; shift 2; echo "== $name"; timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "rc=$rc"; tail -n 2 "$OUT/$name.log" | cut -c1-300; if [ $rc -ne 0 ]; then exit $rc; fi; }
SQA="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_FMA_F64"
SQB="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE"
SQC="SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_WAIT_INST_LDS SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64"
SQD="SQ_ACTIVE_INST_ANY SQ_INSTS_VALU_CVT SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VMEM"
step bench_driver 300 python bench.py --steps 20 --warmup 5
for c in 1 2 3 4; do
  if [ $c = 1 ]; then CMD=$TS; else CMD=$(pop configs_$c); fi
  for p in A B C D; do
    eval "CTR=\$SQ$p"
    step c${c}_sq$p 150 rocprofv3 --pmc $CTR --kernel-include-regex "$GK" --output-format csv -d "$OUT/c${c}_sq$p" -o run -- $CMD
  done
done
echo "== done"
