#!/bin/bash
# Driver-shaped GPU run: smoke(), the GPU suite (optional), bench.py as the driver runs it.
# Usage (on the GPU box): bash tools/gpu_bench.sh <tag> [tests]
set -u
TAG=${1:-b}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
rc=$?; tail -2 "$OUT/smoke.log"; echo "smoke rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi
if [ "${2:-}" = "tests" ]; then
  timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1
  rc=$?; tail -3 "$OUT/pytest.log"; echo "pytest rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi
fi
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/bench.log" 2>&1
rc=$?; echo "bench rc=$rc"; grep -v amdgpu.ids "$OUT/bench.log" | tail -1 | cut -c1-3000
