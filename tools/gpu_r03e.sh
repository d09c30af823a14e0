#!/bin/bash
set -u
OUT=gpurun_out/prof_r03e
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { local name=$1 secs=$2; shift 2; echo "== $name"; timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "rc=$rc"; grep -E "configs_" "$OUT/$name.log" | cut -c1-200; if [ $rc -ne 0 ]; then exit $rc; fi; }
step sweep_c1 150 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/c1" -o run -- python tools/size_sweep.py configs_1
step sweep_c2 150 python tools/size_sweep.py configs_2 fused
step sweep_c4 150 python tools/size_sweep.py configs_4 fused
echo "== done"
