#!/bin/bash
set -u
TAG=${1:-r03f}
OUT=gpurun_out/prof_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { local name=$1 secs=$2; shift 2; echo "== $name"; timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "rc=$rc"; grep -E "configs_|passed|failed|Error" "$OUT/$name.log" | cut -c1-200 | tail -12; if [ $rc -ne 0 ]; then exit $rc; fi; }
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
step sweep_c1 150 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/c1" -o run -- python tools/size_sweep.py configs_1
step sweep_c2 150 python tools/size_sweep.py configs_2
step sweep_c4 150 python tools/size_sweep.py configs_4
step ab_c1 200 python tools/ab_pop.py configs_1 generic fused
step ab_c2 200 python tools/ab_pop.py configs_2 generic split
step ab_c3 200 python tools/ab_pop.py configs_3 generic split
step ab_c4 200 python tools/ab_pop.py configs_4 generic split
step bench_small 600 python bench.py --steps 10 --warmup 3 --batch 16777216 --cpu-sample 1048576
echo "== done"
