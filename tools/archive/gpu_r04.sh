#!/bin/bash
# Round-4 GPU session: smoke, the per-config full-size oracle tests (first), the whole GPU
# suite, the driver-shaped bench line. TAG names the output directory; STEPS picks the steps.
set -u
OUT=gpurun_out/prof_${TAG:-r04}
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { local name=$1 secs=$2; shift 2; echo "== $name"; timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "rc=$rc"; tail -n 3 "$OUT/$name.log" | cut -c1-300; if [ $rc -ne 0 ]; then exit $rc; fi; }
for s in ${STEPS:-smoke configs suite bench}; do
  case $s in
    smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    configs) step pytest_configs 600 python -u -m pytest tests/test_00_configs_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread ;;
    rp) step pytest_rp 900 python -u -m pytest tests/test_gpu_rp.py tests/test_gpu_parity.py tests/test_gpu_distributed.py -m gpu -v --timeout 300 --timeout-method thread -k "rp_ or pipe or driver_ or dropin_ or record_parallel or interleaved or memory or empirical or lrts" ;;
    upd)
      U="python bench.py --steps 5 --warmup 2 --no-ts --no-p8 --no-generate --no-cpu-baseline --populations configs_2,configs_3,configs_4"
      step upd_train 600 env AG_BIDDER_PIPE=0 $U &&
      step upd_pipe 600 $U &&
      step upd_pipe128 600 env AG_PIPE_RECS=128 $U &&
      step upd_pipe2048 600 env AG_PIPE_RECS=2048 $U ;;
    dropin) step dropin_dr 600 python tools/archive/dropin_update_time.py dr 2 && step dropin_dm 600 python tools/archive/dropin_update_time.py dm 2 ;;
    suite) step pytest_gpu 1200 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread ;;
    bench) step bench_driver 400 python bench.py --steps 20 --warmup 5 ;;
    bench_default) step bench_default 600 python bench.py ;;
    ab_stream)
      step ab_c4p8 300 python tools/ab_pop.py configs_4:8 nostream stream1 &&
      step ab_c1p8 300 python tools/ab_pop.py configs_1:8 generic &&
      step ab_c4 300 python tools/ab_pop.py configs_4 stream1 nostream &&
      step ab_c3 300 python tools/ab_pop.py configs_3 stream1 &&
      step ab_c2 300 python tools/ab_pop.py configs_2 stream1 &&
      step ab_c1 300 python tools/ab_pop.py configs_1 stream1 ;;
    ab_p8)
      step ab_c4p8 300 python tools/ab_pop.py configs_4:8 bt768 bt768s streamall &&
      step ab_c4 300 python tools/ab_pop.py configs_4 bt768 streamall ;;
    stats) step kernel_stats 500 rocprofv3 --kernel-trace --stats -d "$OUT/rocprof" -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline ;;
  esac
done
echo "== done"
