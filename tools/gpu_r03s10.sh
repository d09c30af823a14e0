#!/bin/bash
# r03s10: PMC traffic (FETCH_SIZE, WRITE_SIZE) and SQ cycle counters of this build's general
# kernel on configs_1..4 (P = 2), for profiles/pmc_traffic.json and the round-3 PMC summary.
set -u
OUT=gpurun_out/prof_r03s10
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { local name=$1 secs=$2; shift 2; echo "== $name"; timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "rc=$rc"; if [ $rc -ne 0 ]; then tail -3 "$OUT/$name.log"; exit $rc; fi; }
pop() { echo "python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-ts --no-update --no-generate --no-p8 --batch 1048576 --populations $1"; }
TSL="python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-update --no-populations --no-generate --no-p8 --batch 1048576"
SQA="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_FMA_F64"
SQB="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE"
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
step bench_driver 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-update --no-p8
for c in 1 2 3 4; do
  if [ $c = 1 ]; then CMD=$TSL; else CMD=$(pop configs_$c); fi
  step c${c}_fetch 150 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "k_simulate" --output-format csv -d "$OUT/c${c}_fetch" -o run -- $CMD
  step c${c}_write 150 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "k_simulate" --output-format csv -d "$OUT/c${c}_write" -o run -- $CMD
  step c${c}_sqA 150 rocprofv3 --pmc $SQA --kernel-include-regex "k_simulate" --output-format csv -d "$OUT/c${c}_sqA" -o run -- $CMD
  step c${c}_sqB 150 rocprofv3 --pmc $SQB --kernel-include-regex "k_simulate" --output-format csv -d "$OUT/c${c}_sqB" -o run -- $CMD
done
echo "== done"
