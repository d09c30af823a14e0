#!/bin/bash
# r02g: compact Thompson-noise layout -- parity test, population bench lines, the mix's HBM
# traffic (FETCH_SIZE / WRITE_SIZE passes of the general kernel).
set -u
TAG=${1:-r02g}
OUT=gpurun_out/prof_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
pop() { echo "python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-ts --no-update --no-generate --batch 2097152 --populations $1"; }
GK='k_simulate'
step() { local name=$1 secs=$2; shift 2; echo "== $name"; timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "rc=$rc"; tail -3 "$OUT/$name.log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
step pytest_compact 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "compact_ts_noise or mixed_population or wide_participants"
step pop 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-ts --no-generate --batch 1048576
step c4_fetch 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$GK" --output-format csv -d "$OUT/c4_fetch" -o run -- $(pop configs_4)
step c4_write 120 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$GK" --output-format csv -d "$OUT/c4_write" -o run -- $(pop configs_4)
step mix_sq 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_FMA_F64 --kernel-include-regex "$GK" --output-format csv -d "$OUT/mix_sq" -o run -- $(pop configs_4)
step mix_sq2 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE --kernel-include-regex "$GK" --output-format csv -d "$OUT/mix_sq2" -o run -- $(pop configs_4)
echo "== done"
