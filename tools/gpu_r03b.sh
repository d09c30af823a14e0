#!/bin/bash
# r03b: k_pop (the general-population kernel of the shipped shape) -- parity against
# k_simulate and the oracle, then one-process A/B timings on every population line.
set -u
TAG=${1:-r03b}
OUT=gpurun_out/prof_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { local name=$1 secs=$2; shift 2; echo "== $name"; timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "rc=$rc"; tail -n 4 "$OUT/$name.log" | cut -c1-300; if [ $rc -ne 0 ]; then exit $rc; fi; }
step pytest_pop 400 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread -k "pop_kernel or mixed_population or fitted_policy or compact_ts or population_replay or search_bids"
step ab_c1 200 python tools/ab_pop.py configs_1 generic fused bt1024
step ab_c2 200 python tools/ab_pop.py configs_2 generic fused bt1024
step ab_c3 200 python tools/ab_pop.py configs_3 generic fused
step ab_c4 200 python tools/ab_pop.py configs_4 generic fused bt256
echo "== done"
