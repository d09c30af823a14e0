#!/bin/bash
# r03s6: GPU suite (biased fixed-point trainer sums, AUTO split pass at P >= 8, threaded
# Thompson draws), trainer A/B against the round-2 build, drop-in rates, then a trainer PMC
# pass last (the profiler's exit fault after cooperative launches).
set -u
TS=${1:-T3}
OUT=gpurun_out/prof_r03s6
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { local name=$1 secs=$2; shift 2; echo "== $name"; timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "rc=$rc"; grep -E "passed|failed|rror|^\{|min update|median" "$OUT/$name.log" | cut -c1-400 | tail -8; if [ $rc -ne 0 ]; then exit $rc; fi; }
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
step ab_trainer_c2 300 python tools/ab_trainer.py configs_2 r02
step ab_trainer_c3 300 python tools/ab_trainer.py configs_3 r02
step replay_sp_ts 200 python tools/replay_rate.py SP_Truthful_TS 1048576
step replay_fp_dr_policy 300 python tools/replay_rate.py FP_DR_TS_policy 1048576
step ab_c1_p8 200 python tools/ab_pop.py configs_1:8 generic split
T3="SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_VALU_FMA_F32"
T1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64"
UPD="python bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-ts --no-generate --no-p8 --batch 1048576 --populations configs_2"
eval "CTR=\$$TS"
echo "== trainer_$TS (last)"
timeout -k 10 200 rocprofv3 --pmc $CTR --kernel-include-regex "k_bidder_train|k_lrts_train" --output-format csv -d "$OUT/trainer_$TS" -o run -- $UPD > "$OUT/trainer_$TS.log" 2>&1
echo "rc=$?"
echo "== done"
