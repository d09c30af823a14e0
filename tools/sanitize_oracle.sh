#!/bin/bash
# The oracle's C restatement under AddressSanitizer + UBSan: builds
# oracle/libag_oracle_san.so and runs the oracle's CPU tests against it (python loads the
# instrumented library, so the ASan runtime is preloaded; leak checks off -- the
# interpreter's own allocations are not ours). Usage: bash tools/sanitize_oracle.sh
set -eu
cd "$(dirname "$0")/.."
make -s -C oracle sanitize
export AG_ORACLE_LIB=$PWD/oracle/libag_oracle_san.so
export ASAN_OPTIONS=detect_leaks=0:abort_on_error=1
export UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1
LD_PRELOAD="$(gcc -print-file-name=libasan.so):$(gcc -print-file-name=libubsan.so)" \
  python -m pytest tests/test_oracle_golden.py tests/test_exp_restatement.py -x -q -p no:cacheprovider "$@"
