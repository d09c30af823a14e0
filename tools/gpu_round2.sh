#!/bin/bash
# Round-2 end-of-milestone session: smoke, the full GPU suite, the driver-shaped bench, then
# the profile passes (tools/prof_r02.sh). Usage: bash tools/gpu_round2.sh <tag>
set -u
TAG=${1:-r02}
NO_ROCPROF=1 bash tools/gpu_session.sh "$TAG" || exit $?
bash tools/prof_r02.sh "$TAG"
