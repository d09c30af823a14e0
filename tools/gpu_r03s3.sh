#!/bin/bash
# r03s3: k_pop at 256-lane workgroups against k_simulate (generic) on every population line.
set -u
OUT=gpurun_out/prof_r03s3
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { local name=$1 secs=$2; shift 2; echo "== $name"; timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "rc=$rc"; grep -E "configs_|median|rror" "$OUT/$name.log" | cut -c1-200 | tail -12; if [ $rc -ne 0 ]; then exit $rc; fi; }
for c in 1 2 3 4; do step ab_c$c 200 python tools/ab_pop.py configs_$c generic bt256 bt1024; done
echo "== done"
