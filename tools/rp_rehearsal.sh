#!/bin/bash
# Record-parallel update costs on one GPU box: 2 ranks sharing the GPU over gloo (record- and
# agent-parallel), the per-epoch launch path alone at N = 1, and the drop-in update times.
set -u
OUT=gpurun_out/prof_r04q; mkdir -p $OUT
B="bench.py --steps 2 --warmup 1 --no-ts --no-p8 --no-generate --no-cpu-baseline --batch 1048576 --populations configs_3"
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 $B --gpus 2 --rehearse-on-one-gpu --learner-parallel record > $OUT/rehearse_record.log 2>&1 || exit 1
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29534 $B --gpus 2 --rehearse-on-one-gpu --learner-parallel agent > $OUT/rehearse_agent.log 2>&1 || exit 2
timeout -k 10 300 python $B --learner-parallel record > $OUT/single_record.log 2>&1 || exit 3
timeout -k 10 300 python tools/archive/dropin_update_time.py dr 2 > $OUT/dropin_dr.log 2>&1 || exit 4
timeout -k 10 300 python tools/archive/dropin_update_time.py dm 2 > $OUT/dropin_dm.log 2>&1 || exit 5
echo done
