#!/bin/bash
# Exhaustive check of ag_replay.cpp's restatement of torch's float normal kernel block
# (normal_fill_16_AVX2: avx_mathfun.h's Cephes log256_ps / sincos256_ps, multiply-adds
# contracted as the x86-64 GCC build does) against torch's own header compiled the same way,
# on every 24-bit uniform in both the radius and the angle position. Host only (test tool).
set -eu
cd "$(dirname "$0")/torch_normal_probe"
T=$(python -c "import torch, os; print(os.path.dirname(torch.__file__))")
g++ -O2 -mavx2 -mfma -DCPU_CAPABILITY_AVX2 -shared -fPIC -I"$T/include" -o /tmp/probe.so probe.cpp
gcc -O2 -o /tmp/exhaustive exhaustive.c -ldl
/tmp/exhaustive "$(cd ../.. && pwd)/auction-gym_amd/auctiongym_amd/libauctiongym_hip.so"
