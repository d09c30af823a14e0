#!/bin/bash
# r03s12: the round's final build -- smoke, GPU suite, the driver-shaped bench line.
set -u
OUT=gpurun_out/prof_${TAG:-r03s12}
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { local name=$1 secs=$2; shift 2; echo "== $name"; timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "rc=$rc"; tail -n 2 "$OUT/$name.log" | cut -c1-200; if [ $rc -ne 0 ]; then exit $rc; fi; }
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
step bench_driver 300 python bench.py --steps 20 --warmup 5
echo "== done"
