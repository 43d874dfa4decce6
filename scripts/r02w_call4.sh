#!/bin/bash
# Multi-rank rehearsal of bench.py on one GPU (2 ranks, gloo, host-staged collectives), then
# the C3 / C4 bench lines and profiles.
set -e
mkdir -p gpurun_out
MPCG_BENCH_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 5 --warmup 1 > gpurun_out/r02w_rehearsal_n2.log 2>&1
bash scripts/r02w_profiles.sh r02w C3 C4
echo all-done
