#!/bin/bash
# End-of-milestone GPU session: smoke, GPU tests, bench, profiles. Usage: bash tools/gpu_round.sh <tag>
set -u
TAG=${1:-r01}
NO_ROCPROF=1 bash tools/gpu_session.sh "$TAG" || exit $?
bash tools/collect_profiles.sh "$TAG"
