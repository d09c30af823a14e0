#!/bin/bash
# One GPU-box session: smoke, GPU tests, bench, rocprofv3 kernel trace. Every GPU step
# has its own time limit; a crash / timeout / signal ends the session (no retries).
# Usage: bash tools/gpu_session.sh <tag>
set -u
TAG=${1:-r01}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {  # name, seconds, command...
  local name=$1 secs=$2; shift 2
  echo "== $name: $*" | tee -a "$OUT/session.log"
  local t0=$(date +%s)
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc ($(( $(date +%s) - t0 )) s)" | tee -a "$OUT/session.log"
  tail -5 "$OUT/$name.log"
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then
    echo "== fatal rc=$rc in $name: stopping" | tee -a "$OUT/session.log"; exit $rc
  fi
  return $rc
}
rocm-smi --showproductname > "$OUT/gpu.txt" 2>&1 || true
nproc > "$OUT/host.txt"; lscpu | grep "Model name" >> "$OUT/host.txt"
run smoke 400 python -c "import __graft_entry__ as g; g.smoke()"
run pytest_gpu 900 python -u -m pytest tests -v -m gpu -x --timeout 300 --timeout-method thread
run bench 600 python bench.py
# last: rocprofv3 7.2 crashes in its exit handler after a cooperative launch (the learner
# updates), after writing its results -- tools/gpu_round.sh skips this and profiles in
# tools/collect_profiles.sh instead (PMC passes first, that command last)
if [ -z "${NO_ROCPROF:-}" ]; then
  run rocprof 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o bench -- python bench.py --steps 10 --warmup 2 --no-cpu-baseline
fi
echo "== done" | tee -a "$OUT/session.log"
