#!/bin/bash
# quick loop: GPU tests then ablation timings. Usage: bash tools/gpu_quick.sh <tag>
set -u
TAG=${1:-q}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -q -m gpu -x > "$OUT/pytest_gpu.log" 2>&1
rc=$?; tail -15 "$OUT/pytest_gpu.log"; echo "pytest rc=$rc"
if [ $rc -ge 124 ]; then exit $rc; fi
timeout -k 10 300 python tools/ablate.py > "$OUT/ablate.log" 2>&1
rc=$?; cat "$OUT/ablate.log" | grep -v amdgpu.ids; echo "ablate rc=$rc"
