#!/bin/bash
# Round-2 final evidence: driver-shaped bench line, kernel-trace stats, and HBM traffic
# (FETCH_SIZE / WRITE_SIZE passes) of the headline kernel and of the general kernel on
# every population line (configs_1..4), plus the SQ passes of the headline and the mix.
# Usage (on the GPU box): bash tools/prof_r02e.sh <tag>; then
# python tools/make_pmc_traffic.py gpurun_out/prof_<tag> (here) -> profiles/pmc_traffic.json
set -u
TAG=${1:-r02e}
OUT=gpurun_out/prof_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
HEAD="python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-ts --no-populations --no-generate"
TS="python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-update --no-populations --no-generate --batch 1048576"
pop() { echo "python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-ts --no-update --no-generate --batch 1048576 --populations $1"; }
HK='k_oracle<2, 6, false>'
GK='k_simulate'
step() { local name=$1 secs=$2; shift 2; echo "== $name"; timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "rc=$rc"; tail -2 "$OUT/$name.log"; if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then exit $rc; fi; }
step bench_driver 300 python bench.py --steps 20 --warmup 5
step fetch 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$HK" --output-format csv -d "$OUT/fetch" -o run -- $HEAD
step write 120 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$HK" --output-format csv -d "$OUT/write" -o run -- $HEAD
step sq 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_FMA_F64 --kernel-include-regex "$HK" --output-format csv -d "$OUT/sq" -o run -- $HEAD
step sq2 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE --kernel-include-regex "$HK" --output-format csv -d "$OUT/sq2" -o run -- $HEAD
step c1_fetch 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$GK" --output-format csv -d "$OUT/c1_fetch" -o run -- $TS
step c1_write 120 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$GK" --output-format csv -d "$OUT/c1_write" -o run -- $TS
for c in 2 3 4; do
  step c${c}_fetch 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$GK" --output-format csv -d "$OUT/c${c}_fetch" -o run -- $(pop configs_$c)
  step c${c}_write 120 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$GK" --output-format csv -d "$OUT/c${c}_write" -o run -- $(pop configs_$c)
done
step mix_sq 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_FMA_F64 --kernel-include-regex "$GK" --output-format csv -d "$OUT/mix_sq" -o run -- $(pop configs_4)
step mix_sq2 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE --kernel-include-regex "$GK" --output-format csv -d "$OUT/mix_sq2" -o run -- $(pop configs_4)
step stats_head 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/stats_head" -o run -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-ts --no-populations
step stats 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/stats" -o run -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline
echo "== done"
