#!/bin/bash
# A/B of library variants: bash scripts/ab.sh <tag> <lib-suffix>...  ("" = libmpcg.so)
# per variant: GPU parity tests, then C2 / C4 / C5 bench lines (no CPU baseline)
set -e
mkdir -p gpurun_out
tag=$1; shift
P=oscar_mpc_planner_mr_modification_amd
for v in "$@"; do
  lib=$P/libmpcg${v:+_$v}.so
  MPCG_LIB=$lib timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scenario.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${tag}_${v:-base}_gpu.log 2>&1 || echo "tests failed for $v"
  for c in C2 C4 C5; do
    MPCG_LIB=$lib timeout -k 10 300 python bench.py --config $c --no-cpu --steps 5 --warmup 1 > gpurun_out/${tag}_${v:-base}_$c.log 2>&1
  done
done
echo ab-done
