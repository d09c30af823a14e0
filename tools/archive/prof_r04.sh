#!/bin/bash
# Round-4 evidence passes (on the GPU box): HBM traffic (FETCH_SIZE / WRITE_SIZE, separate
# passes) of the headline kernel and of the general kernel on every population line incl.
# the P = 8 lines, the SQ passes (instruction mix, LDS bank conflicts, SALU) of the headline
# and of configs_2 / configs_4, the driver-shaped bench line and the kernel-trace stats.
# Usage: TAG=r04x bash tools/archive/prof_r04.sh; then (here)
#   python tools/make_pmc_traffic.py gpurun_out/prof_<tag> <tag> > profiles/pmc_traffic.json
#   python tools/summarize_pmc.py gpurun_out/prof_<tag> > profiles/<tag>_pmc_summary.json
set -u
TAG=${TAG:-r04p}
OUT=gpurun_out/prof_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
HEAD="python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-ts --no-populations --no-generate"
ts() { echo "python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-update --no-populations --no-generate --batch 1048576 ${1:---no-p8}"; }
pop() { echo "python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-ts --no-update --no-generate --batch 1048576 --populations $1 ${2:---no-p8}"; }
HK='k_oracle<2, 6, false>'
GK='k_simulate'
SQA="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM"
SQB="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE"
step() { local name=$1 secs=$2; shift 2; echo "== $name"; timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "rc=$rc"; tail -n 2 "$OUT/$name.log" | cut -c1-300; if [ $rc -ne 0 ]; then exit $rc; fi; }
pmc() { local name=$1 k=$2; shift 2; local ctr=$1; shift; step "$name" 150 rocprofv3 --pmc $ctr --kernel-include-regex "$k" --output-format csv -d "$OUT/$name" -o run -- "$@"; }
for s in ${STEPS:-bench head pops sq stats}; do
  case $s in
    bench) step bench_driver 400 python bench.py --steps 20 --warmup 5 ;;
    head)
      pmc fetch "$HK" FETCH_SIZE $HEAD && pmc write "$HK" WRITE_SIZE $HEAD &&
      pmc sqA "$HK" "$SQA" $HEAD && pmc sqB "$HK" "$SQB" $HEAD ;;
    pops)
      pmc c1_fetch "$GK" FETCH_SIZE $(ts) && pmc c1_write "$GK" WRITE_SIZE $(ts) &&
      pmc c1p8_fetch "$GK" FETCH_SIZE $(ts "--p8-only") && pmc c1p8_write "$GK" WRITE_SIZE $(ts "--p8-only") &&
      for c in 2 3 4; do
        pmc c${c}_fetch "$GK" FETCH_SIZE $(pop configs_$c) && pmc c${c}_write "$GK" WRITE_SIZE $(pop configs_$c) || exit 1
      done &&
      pmc c4p8_fetch "$GK" FETCH_SIZE $(pop configs_4 --p8-only) && pmc c4p8_write "$GK" WRITE_SIZE $(pop configs_4 --p8-only) ;;
    p8)
      pmc c1p8_fetch "$GK" FETCH_SIZE $(ts "--p8-only") && pmc c1p8_write "$GK" WRITE_SIZE $(ts "--p8-only") &&
      pmc c4p8_fetch "$GK" FETCH_SIZE $(pop configs_4 --p8-only) && pmc c4p8_write "$GK" WRITE_SIZE $(pop configs_4 --p8-only) &&
      pmc c4p8_sqA "$GK" "$SQA" $(pop configs_4 --p8-only) && pmc c4p8_sqB "$GK" "$SQB" $(pop configs_4 --p8-only) ;;
    c4) pmc c4_fetch "$GK" FETCH_SIZE $(pop configs_4) && pmc c4_write "$GK" WRITE_SIZE $(pop configs_4) ;;
    sq)
      pmc c1_sqA "$GK" "$SQA" $(ts) && pmc c1_sqB "$GK" "$SQB" $(ts) &&
      for c in 2 4; do
        pmc c${c}_sqA "$GK" "$SQA" $(pop configs_$c) && pmc c${c}_sqB "$GK" "$SQB" $(pop configs_$c) || exit 1
      done ;;
    trainer*)  # the learners' update kernels (configs_2); LAST in a call: rocprofv3 has faulted at
      # exit after cooperative kernels (r03s7), so its rc is reported, not acted on, and nothing follows
      T1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64"
      T2="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE"
      eval "CTR=\$${s#trainer_}"
      UPD="python bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-ts --no-generate --no-p8 --batch 1048576 --populations configs_2"
      echo "== $s"
      timeout -k 10 300 rocprofv3 --pmc $CTR --kernel-include-regex "k_bidder_train|k_lrts_train" --output-format csv -d "$OUT/$s" -o run -- $UPD > "$OUT/$s.log" 2>&1
      echo "rc=$?"
      break ;;
    sizes)  # the L2's memory-side read / write requests by size: calibrates FETCH_SIZE x 2 on the
      # headline (16 B per lane, known bytes) against the general kernel's 4-B-per-lane noise reads
      rocprofv3 --list-avail > "$OUT/avail.txt" 2>&1 || true
      CS=$(grep -o 'TCC_EA0_\(RD\|WR\)REQ[A-Z0-9_]*' "$OUT/avail.txt" | sed 's/_*$//' | sort -u | tr '\n' ' ')
      echo "tcc request counters: $CS"
      for c in $CS; do
        pmc "hd_$c" "$HK" "${c}_sum" $HEAD && pmc "c4p8_$c" "$GK" "${c}_sum" $(pop configs_4 --p8-only) &&
        pmc "c1_$c" "$GK" "${c}_sum" $(ts) || exit 1
      done ;;
    stats) step kernel_stats 500 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/stats" -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline ;;
  esac
done
echo "== done"
