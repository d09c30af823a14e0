#!/bin/bash
# PMC passes of the general simulate kernel on configs_1 (SP_Truthful_TS) and configs_4 (mix).
set -u
OUT=gpurun_out/pmc_ts
mkdir -p $OUT
export TMPDIR=/tmp
TS="python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-update --no-populations --no-generate --batch 1048576"
MIX="python bench.py --steps 10 --warmup 5 --no-cpu-baseline --no-ts --no-update --populations configs_4 --no-generate --batch 1048576"
K='k_simulate'
step() { local name=$1; shift; timeout -k 10 120 "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; if [ $rc -ge 124 ]; then exit $rc; fi; }
step ts_sq rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_FMA_F64 --kernel-include-regex "$K" --output-format csv -d $OUT/ts_sq -o run -- $TS
step ts_sq2 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE SQ_ACTIVE_INST_LDS --kernel-include-regex "$K" --output-format csv -d $OUT/ts_sq2 -o run -- $TS
step ts_sq3 rocprofv3 --pmc SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_WAIT_INST_LDS SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 --kernel-include-regex "$K" --output-format csv -d $OUT/ts_sq3 -o run -- $TS
step mix_sq rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_FMA_F64 --kernel-include-regex "$K" --output-format csv -d $OUT/mix_sq -o run -- $MIX
step mix_sq2 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE SQ_ACTIVE_INST_LDS --kernel-include-regex "$K" --output-format csv -d $OUT/mix_sq2 -o run -- $MIX
step mix_sq3 rocprofv3 --pmc SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_WAIT_INST_LDS SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 --kernel-include-regex "$K" --output-format csv -d $OUT/mix_sq3 -o run -- $MIX
python tools/summarize_pmc.py $OUT $((1<<20)) > $OUT/summary.json 2>&1
