#!/bin/bash
# rocprofv3 kernel trace of tools/archive/exit_probe.py, plain launch first, cooperative second.
set -u
OUT=gpurun_out/exit_probe
mkdir -p $OUT
export TMPDIR=/tmp
for m in plain coop; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$m -o run -- python tools/archive/exit_probe.py $m $OUT > $OUT/$m.log 2>&1
  echo "$m rc=$?"
done
grep -h "^    @\|SIGSEGV\|PC:" $OUT/*.log | head -40
# the same cooperative launch without torch (only /opt/rocm's HIP and HSA in the process)
timeout -k 10 60 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c -o run -- build/coop_exit > $OUT/coop_c.log 2>&1
echo "coop_c (no torch) rc=$?"
