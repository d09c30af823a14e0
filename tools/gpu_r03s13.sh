#!/bin/bash
# r03s13: the TruthfulBidder-only general build at a 5-wave cap (variant t5: 96 VGPRs, 22 spilled)
# against the 4-wave default (115 VGPRs) on configs_1, twice.
set -u
OUT=gpurun_out/prof_r03s13
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { local name=$1 secs=$2; shift 2; echo "== $name"; timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "rc=$rc"; grep -E "median|rror" "$OUT/$name.log" | cut -c1-200 | tail -6; if [ $rc -ne 0 ]; then exit $rc; fi; }
step ab_c1 200 python tools/ab_pop.py configs_1 t5
step ab_c1_again 200 python tools/ab_pop.py configs_1 t5
echo "== done"
