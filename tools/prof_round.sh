#!/bin/bash
# A round's evidence passes (on the GPU box): for every bench line, its own rocprofv3 kernel
# trace (one run per workload, so two lines whose kernels share a name -- configs_2 and
# configs_3 run the same k_simulate instantiation -- never fold into one row), HBM traffic
# (FETCH_SIZE / WRITE_SIZE in separate passes, MI355X_MICROARCH.md), the SQ passes, and the
# driver-shaped bench line.
# Usage: TAG=r06x [STEPS="bench trace head pops sq"] bash tools/prof_round.sh; then (here)
#   python tools/summarize_traces.py gpurun_out/prof_<tag> > profiles/<tag>_kernel_stats_by_workload.csv
#   python tools/summarize_pmc.py gpurun_out/prof_<tag> > profiles/<tag>_pmc_summary.json
#   python tools/make_pmc_traffic.py profiles/<tag>_pmc_summary.json > profiles/pmc_traffic.json
set -u
TAG=${TAG:-r06x}
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
# one kernel trace per bench line: the line's JSON (HIP-event kernel_ms) lands in the same log
trace() { local wl=$1; shift; step "tr_$wl" 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/tr_$wl" -o run -- "$@"; }
for s in ${STEPS:-bench trace head pops sq}; do
  case $s in
    bench) step bench_driver 400 python bench.py --steps 20 --warmup 5 ;;
    trace)
      # the headline and its generate mode at the driver's shape; each population line with its
      # generate-mode line, no learner update (the update's cooperative launches are traced in
      # the `update` step, last: rocprofv3 has faulted at exit after them)
      trace hd python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-ts --no-populations --no-p8 &&
      trace c1 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-update --no-populations --no-p8 --batch 1048576 &&
      trace c1p8 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-update --no-populations --p8-only --batch 1048576 &&
      for c in 2 3 4; do
        trace c$c python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-ts --no-update --no-p8 --batch 1048576 --populations configs_$c || exit 1
      done &&
      trace c4p8 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-ts --no-update --p8-only --batch 1048576 --populations configs_4 ;;
    head)
      pmc hd_fetch "$HK" FETCH_SIZE $HEAD && pmc hd_write "$HK" WRITE_SIZE $HEAD &&
      pmc hd_sqA "$HK" "$SQA" $HEAD && pmc hd_sqB "$HK" "$SQB" $HEAD ;;
    pops)
      pmc c1_fetch "$GK" FETCH_SIZE $(ts) && pmc c1_write "$GK" WRITE_SIZE $(ts) &&
      pmc c1p8_fetch "$GK" FETCH_SIZE $(ts "--p8-only") && pmc c1p8_write "$GK" WRITE_SIZE $(ts "--p8-only") &&
      for c in 2 3 4; do
        pmc c${c}_fetch "$GK" FETCH_SIZE $(pop configs_$c) && pmc c${c}_write "$GK" WRITE_SIZE $(pop configs_$c) || exit 1
      done &&
      pmc c4p8_fetch "$GK" FETCH_SIZE $(pop configs_4 --p8-only) && pmc c4p8_write "$GK" WRITE_SIZE $(pop configs_4 --p8-only) ;;
    sq)
      pmc c1_sqA "$GK" "$SQA" $(ts) && pmc c1_sqB "$GK" "$SQB" $(ts) &&
      for c in 2 4; do
        pmc c${c}_sqA "$GK" "$SQA" $(pop configs_$c) && pmc c${c}_sqB "$GK" "$SQB" $(pop configs_$c) || exit 1
      done ;;
    gen)  # the generate-mode kernels' instruction mix (VALU-bound: Philox)
      GEN1="python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-update --no-populations --no-p8 --batch 1048576"
      pmc c1g_sqA "k_simulate.*true>" "$SQA" $GEN1 && pmc c1g_sqB "k_simulate.*true>" "$SQB" $GEN1 ;;
    update)  # LAST in a call (see above): the learners' update of configs_2 under the trace
      echo "== update"
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/tr_update" -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-ts --no-generate --no-p8 --batch 1048576 --populations configs_2 > "$OUT/tr_update.log" 2>&1
      echo "rc=$?"
      break ;;
  esac
done
echo "== done"
