#!/bin/bash
# r03s7: GPU suite; the shipped-shape k_simulate build (KSH = 12) against the runtime-shape
# build on every population line; trainer A/B (biased fixed-point sums) against round 2; the
# drop-in rates with threaded transforms; a trainer PMC pass last (the profiler's exit fault).
set -u
TS=${1:-T1}
OUT=gpurun_out/prof_r03s7
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { local name=$1 secs=$2; shift 2; echo "== $name"; timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "rc=$rc"; grep -E "passed|failed|rror|^\{|min update|median" "$OUT/$name.log" | cut -c1-400 | tail -8; if [ $rc -ne 0 ]; then exit $rc; fi; }
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
for c in 1 2 3 4; do step ab_c$c 200 python tools/ab_pop.py configs_$c noship; done
step ab_c1_p8 200 python tools/ab_pop.py configs_1:8 noship generic
step ab_trainer_c2 300 python tools/ab_trainer.py configs_2 r02
step replay_sp_ts 200 python tools/replay_rate.py SP_Truthful_TS 1048576
step replay_fp_dr_policy 300 python tools/replay_rate.py FP_DR_TS_policy 1048576
T1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64"
T2="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE"
UPD="python bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-ts --no-generate --no-p8 --batch 1048576 --populations configs_2"
eval "CTR=\$$TS"
echo "== trainer_$TS (last)"
timeout -k 10 200 rocprofv3 --pmc $CTR --kernel-include-regex "k_bidder_train|k_lrts_train" --output-format csv -d "$OUT/trainer_$TS" -o run -- $UPD > "$OUT/trainer_$TS.log" 2>&1
echo "rc=$?"
echo "== done"
