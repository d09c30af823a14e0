#!/bin/bash
# r03s8: GPU suite (per-agent item counts), the driver-shaped bench of this build, PMC traffic of the P = 8 lines (configs_1_p8:
# k_ts_choice + k_pop; configs_4_p8: k_simulate), then a trainer PMC pass last.
set -u
TS=${1:-T2}
OUT=gpurun_out/prof_r03s8
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { local name=$1 secs=$2; shift 2; echo "== $name"; timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "rc=$rc"; tail -n 1 "$OUT/$name.log" | cut -c1-200; if [ $rc -ne 0 ]; then exit $rc; fi; }
C1="python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-update --no-populations --no-generate --batch 1048576"
C4="python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-update --no-ts --populations configs_4 --no-generate --batch 1048576"
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
step bench_driver 300 python bench.py --steps 20 --warmup 5
for ctr in FETCH_SIZE WRITE_SIZE; do
  step c1p8_$ctr 150 rocprofv3 --pmc $ctr --kernel-include-regex "k_ts_choice<8|k_pop<8" --output-format csv -d "$OUT/c1p8_$ctr" -o run -- $C1
  step c4p8_$ctr 150 rocprofv3 --pmc $ctr --kernel-include-regex "k_simulate<8" --output-format csv -d "$OUT/c4p8_$ctr" -o run -- $C4
done
T2="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE"
UPD="python bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-ts --no-generate --no-p8 --batch 1048576 --populations configs_2"
eval "CTR=\$$TS"
echo "== trainer_$TS (last)"
timeout -k 10 200 rocprofv3 --pmc $CTR --kernel-include-regex "k_bidder_train|k_lrts_train" --output-format csv -d "$OUT/trainer_$TS" -o run -- $UPD > "$OUT/trainer_$TS.log" 2>&1
echo "rc=$?"
echo "== done"
