#!/bin/bash
# configs_4 at P = 8 (the streamed 768-lane build): timing A/B of P = 8 variant builds in one
# process (tools/ab_pop.py, outputs checked equal), then FETCH_SIZE / WRITE_SIZE of each build's
# simulate kernel (each copied over the library in the GPU box's scratch tree, one rocprofv3
# pass per counter). Variants: make variant-p VP=8 NAME=<v> VFLAGS=...
#   TAG=r05z VARIANTS="base8 pk8" PMC="base8 pk8 abl2" bash tools/archive/ab_p8.sh
# KEY / POPARGS select another line, e.g. KEY=configs_4 POPARGS="--populations configs_4 --no-p8" (P = 2)
set -u
TAG=${TAG:-r05z}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
LIB=auction-gym_amd/auctiongym_amd/libauctiongym_hip.so
KEY=${KEY:-configs_4:8}
POP="python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-ts --no-update --no-generate --batch 1048576 ${POPARGS:---populations configs_4 --p8-only}"
if [ -n "${VARIANTS-base8 pk8}" ]; then
  timeout -k 10 400 python -u tools/ab_pop.py $KEY ${VARIANTS-base8 pk8} > "$OUT/ab_${KEY/:/_}.log" 2>&1 || { echo "ab rc=$?"; exit 1; }
  tail -n 8 "$OUT/ab_${KEY/:/_}.log"
fi
ORIG=$(mktemp /tmp/lib_orig.XXXXXX)
cp "$LIB" "$ORIG"
for v in ${PMC-base8 pk8}; do
  if [ "$v" = base ]; then cp "$ORIG" "$LIB"; else cp auction-gym_amd/build/variants/libauctiongym_hip_$v.so "$LIB"; fi
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 150 rocprofv3 --pmc $c --kernel-include-regex k_simulate --output-format csv -d "$OUT/${KEY/:/_}_${v}_$c" -o run -- $POP > "$OUT/${KEY/:/_}_${v}_$c.log" 2>&1 || { echo "$v $c rc=$?"; exit 1; }
  done
  tail -n 1 "$OUT/${KEY/:/_}_${v}_FETCH_SIZE.log" | cut -c1-200
done
cp "$ORIG" "$LIB"
rm -f "$ORIG"
echo done
