#!/bin/bash
# Round-2 evidence: driver-shaped bench line, kernel-trace stats, and PMC passes of the
# headline kernel (k_oracle) and of the general kernel on configs_1 / configs_4.
# Usage (on the GPU box): bash tools/prof_r02.sh <tag>
set -u
TAG=${1:-r02}
OUT=gpurun_out/prof_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
HEAD="python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-ts --no-populations --no-generate"
MIX="python bench.py --steps 10 --warmup 5 --no-cpu-baseline --no-ts --no-update --populations configs_4 --no-generate --batch 1048576"
HK='k_oracle<2, 6, false>'
GK='k_simulate'
step() { local name=$1 secs=$2; shift 2; echo "== $name"; timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "rc=$rc"; tail -3 "$OUT/$name.log"; if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then exit $rc; fi; }
step bench_driver 300 python bench.py --steps 20 --warmup 5
step fetch 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$HK" --output-format csv -d "$OUT/fetch" -o run -- $HEAD
step write 120 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$HK" --output-format csv -d "$OUT/write" -o run -- $HEAD
step sq 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_FMA_F64 --kernel-include-regex "$HK" --output-format csv -d "$OUT/sq" -o run -- $HEAD
step sq2 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE --kernel-include-regex "$HK" --output-format csv -d "$OUT/sq2" -o run -- $HEAD
step mix_fetch 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$GK" --output-format csv -d "$OUT/mix_fetch" -o run -- $MIX
step mix_write 120 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$GK" --output-format csv -d "$OUT/mix_write" -o run -- $MIX
step mix_sq 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_FMA_F64 --kernel-include-regex "$GK" --output-format csv -d "$OUT/mix_sq" -o run -- $MIX
step mix_sq2 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE --kernel-include-regex "$GK" --output-format csv -d "$OUT/mix_sq2" -o run -- $MIX
step stats_head 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/stats_head" -o run -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-ts --no-populations
step stats 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/stats" -o run -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline
echo "== done"
