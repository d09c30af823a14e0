#!/bin/bash
# r03s15: the runtime-P general kernel (wide: slot results not kept in registers) against AUTO
# at P = 8 on the mix (1024-lane DOS build, 880 B/lane scratch) and on configs_1 (split k_pop).
set -u
OUT=gpurun_out/prof_r03s15
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { local name=$1 secs=$2; shift 2; echo "== $name"; timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "rc=$rc"; grep -E "median|rror" "$OUT/$name.log" | cut -c1-200 | tail -6; if [ $rc -ne 0 ]; then exit $rc; fi; }
step ab_c4_p8 200 python tools/ab_pop.py configs_4:8 wide
step ab_c1_p8 200 python tools/ab_pop.py configs_1:8 wide
step ab_c4_p2 200 python tools/ab_pop.py configs_4 wide
echo "== done"
