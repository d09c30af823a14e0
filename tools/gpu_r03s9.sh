#!/bin/bash
# r03s9: the kernel trace of the driver-shaped bench (last:
# the profiler's exit path faults after the learners' cooperative launches, results written first).
set -u
OUT=gpurun_out/prof_r03s9
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { local name=$1 secs=$2; shift 2; echo "== $name"; timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "rc=$rc"; grep -E "median|rror" "$OUT/$name.log" | cut -c1-200 | tail -6; if [ $rc -ne 0 ]; then exit $rc; fi; }
echo "== stats (last)"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/stats" -o run -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline > "$OUT/stats.log" 2>&1
echo "rc=$?"
echo "== done"
