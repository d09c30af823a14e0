#!/bin/bash
set -u
OUT=gpurun_out/prof_r03k
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { local name=$1 secs=$2; shift 2; echo "== $name"; timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "rc=$rc"; grep -E "configs_|passed|failed|rror" "$OUT/$name.log" | cut -c1-200 | tail -12; if [ $rc -ne 0 ]; then exit $rc; fi; }
step pytest_pop 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "pop_kernel or mixed_population or fitted_policy or compact_ts or population_replay or driver or integration"
for c in 1 2 3 4; do step ab_c$c 200 python tools/ab_pop.py configs_$c nocnt bt256 generic; done
echo "== done"
