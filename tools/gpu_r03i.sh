#!/bin/bash
set -u
OUT=gpurun_out/prof_r03i
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { local name=$1 secs=$2; shift 2; echo "== $name"; timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "rc=$rc"; grep -E "configs_" "$OUT/$name.log" | cut -c1-200 | tail -12; if [ $rc -ne 0 ]; then exit $rc; fi; }
step ab_c1 200 python tools/ab_pop.py configs_1 pf1 w5
step ab_c2 200 python tools/ab_pop.py configs_2 pf1 w5 split
step ab_c3 200 python tools/ab_pop.py configs_3 pf1 w5 split
step ab_c4 200 python tools/ab_pop.py configs_4 pf1 split
echo "== done"
