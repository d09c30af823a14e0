#!/bin/bash
# r03s2: one-process A/B of the round-2 library (variant r02, built from commit d03704c) against
# this build's kernel choices on every population line and on the headline.
set -u
OUT=gpurun_out/prof_r03s2
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { local name=$1 secs=$2; shift 2; echo "== $name"; timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "rc=$rc"; grep -E "configs_|median|rror" "$OUT/$name.log" | cut -c1-200 | tail -12; if [ $rc -ne 0 ]; then exit $rc; fi; }
for c in 1 2 3 4; do step ab_c$c 200 python tools/ab_pop.py configs_$c r02 generic fused split; done
step ab_head 200 python tools/ab_libs.py r02
echo "== done"
