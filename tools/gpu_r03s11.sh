#!/bin/bash
# r03s11: the full general build with the LR-TS width compile-time at a 4-wave cap (variant w4:
# 128 VGPRs, 3 spilled) against the 3-wave default (140 VGPRs) on configs_2 / configs_3.
set -u
OUT=gpurun_out/prof_r03s11
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { local name=$1 secs=$2; shift 2; echo "== $name"; timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "rc=$rc"; grep -E "median|rror" "$OUT/$name.log" | cut -c1-200 | tail -6; if [ $rc -ne 0 ]; then exit $rc; fi; }
step ab_c2 200 python tools/ab_pop.py configs_2 w4
step ab_c3 200 python tools/ab_pop.py configs_3 w4
step ab_c2_again 200 python tools/ab_pop.py configs_2 w4
echo "== done"
