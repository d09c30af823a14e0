#!/bin/bash
# r03s5: GPU suite (drop-in driver tests now draw through ag_replay_draw_population), drop-in
# replay rates of SP_Oracle / SP_Truthful_TS / FP_DR_TS (Gaussian and fitted-policy bids),
# configs_1 P=8 A/B, then one trainer PMC pass last (the profiler's exit fault).
set -u
TS=${1:-T2}
OUT=gpurun_out/prof_r03s5
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { local name=$1 secs=$2; shift 2; echo "== $name"; timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "rc=$rc"; grep -E "passed|failed|rror|^\{|median" "$OUT/$name.log" | cut -c1-400 | tail -8; if [ $rc -ne 0 ]; then exit $rc; fi; }
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
step replay_sp_oracle 200 python tools/replay_rate.py SP_Oracle 1048576
step replay_sp_ts 200 python tools/replay_rate.py SP_Truthful_TS 65536
step replay_sp_ts_big 200 python tools/replay_rate.py SP_Truthful_TS 1048576
step replay_fp_dr 200 python tools/replay_rate.py FP_DR_TS 1048576
step replay_fp_dr_policy 300 python tools/replay_rate.py FP_DR_TS_policy 1048576
T1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64"
T2="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE"
UPD="python bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-ts --no-generate --no-p8 --batch 1048576 --populations configs_2"
eval "CTR=\$$TS"
echo "== trainer_$TS (last)"
timeout -k 10 200 rocprofv3 --pmc $CTR --kernel-include-regex "k_bidder_train|k_lrts_train" --output-format csv -d "$OUT/trainer_$TS" -o run -- $UPD > "$OUT/trainer_$TS.log" 2>&1
echo "rc=$?"
echo "== done"
