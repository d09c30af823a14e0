#!/bin/bash
# Ablations + PMC passes for the simulate kernel (diagnostics). Usage: bash tools/gpu_ablate.sh <tag>
set -u
TAG=${1:-abl}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { local name=$1 secs=$2; shift 2; echo "== $name"; timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "rc=$rc"; tail -12 "$OUT/$name.log"; if [ $rc -ge 124 ]; then exit $rc; fi; }
step ablate 300 python tools/ablate.py
step pmc_fetch 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex k_simulate --output-format csv -d "$OUT/pmc_fetch" -o p -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline
step pmc_write 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex k_simulate --output-format csv -d "$OUT/pmc_write" -o p -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline
step pmc_sq 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY --kernel-include-regex k_simulate --output-format csv -d "$OUT/pmc_sq" -o p -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline
step pmc_sq2 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU GRBM_GUI_ACTIVE SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU_FMA_F64 --kernel-include-regex k_simulate --output-format csv -d "$OUT/pmc_sq2" -o p -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline
