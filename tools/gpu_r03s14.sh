#!/bin/bash
# r03s14: drop-in driver / surface tests and the drop-in rates after the chunking change.
set -u
OUT=gpurun_out/prof_r03s14
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { local name=$1 secs=$2; shift 2; echo "== $name"; timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "rc=$rc"; grep -E "passed|failed|rror|^\{" "$OUT/$name.log" | cut -c1-300 | tail -4; if [ $rc -ne 0 ]; then exit $rc; fi; }
step pytest_dropin 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "dropin or driver or integration or notebook"
step replay_sp_ts 200 python tools/replay_rate.py SP_Truthful_TS 1048576
step replay_sp_oracle 200 python tools/replay_rate.py SP_Oracle 1048576
echo "== done"
