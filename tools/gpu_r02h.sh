#!/bin/bash
# r02h: full GPU suite, smoke, driver-shaped bench, HBM traffic of the mix (compact noise
# layout, early per-slot counters), kernel stats. Usage: bash tools/gpu_r02h.sh <tag>
set -u
TAG=${1:-r02h}
OUT=gpurun_out/prof_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
pop() { echo "python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-ts --no-update --no-generate --batch 1048576 --populations $1"; }
TS="python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-update --no-populations --no-generate --batch 1048576"
GK='k_simulate'
step() { local name=$1 secs=$2; shift 2; echo "== $name"; timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "rc=$rc"; tail -n 3 "$OUT/$name.log" | cut -c1-400; if [ $rc -ne 0 ]; then exit $rc; fi; }
step pytest_gpu 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread
step smoke 200 python -c "import __graft_entry__ as g; g.smoke()"
step bench_driver 300 python bench.py --steps 20 --warmup 5
step ab_c4 200 python tools/ab_pop.py configs_4
step ab_c2 200 python tools/ab_pop.py configs_2
for c in 2 3 4; do
  step c${c}_fetch 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$GK" --output-format csv -d "$OUT/c${c}_fetch" -o run -- $(pop configs_$c)
  step c${c}_write 120 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$GK" --output-format csv -d "$OUT/c${c}_write" -o run -- $(pop configs_$c)
done
step c1_fetch 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$GK" --output-format csv -d "$OUT/c1_fetch" -o run -- $TS
step c1_write 120 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$GK" --output-format csv -d "$OUT/c1_write" -o run -- $TS
step stats 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/stats" -o run -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline
echo "== done"
