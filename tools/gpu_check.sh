#!/bin/bash
# GPU check of a build: the -m gpu suite, the kernel A/B, and the driver-shaped bench at
# several batch sizes (fresh process each, --warmup 5 --steps 20 as the driver runs it).
# Usage (on the GPU box): bash tools/gpu_check.sh <tag> [pytest -k expr]
set -u
TAG=${1:-chk}
KEXPR=${2:-}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
if [ -n "$KEXPR" ]; then
  timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread -k "$KEXPR" > "$OUT/pytest.log" 2>&1
else
  timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1
fi
rc=$?; tail -4 "$OUT/pytest.log"; echo "pytest rc=$rc"
if [ $rc -ge 124 ]; then exit $rc; fi
timeout -k 10 300 python tools/ab_oracle.py > "$OUT/ab.log" 2>&1
rc=$?; grep -v amdgpu.ids "$OUT/ab.log"; echo "ab rc=$rc"
if [ $rc -ge 124 ]; then exit $rc; fi
for b in 16777216 67108864 134217728; do
  timeout -k 10 300 python bench.py --warmup 5 --steps 20 --no-cpu-baseline --no-ts --no-populations --batch $b > "$OUT/bench_$b.log" 2>&1
  rc=$?; echo "bench B=$b rc=$rc"; if [ $rc -ge 124 ]; then exit $rc; fi
  python -c "import json,sys; d=json.loads(open('$OUT/bench_$b.log').read().strip().splitlines()[-1]); print(' value %.4g ms/step %.4f kernel %.4f frac %.4f' % (d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frac']))"
done
