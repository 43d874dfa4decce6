#!/bin/bash
# A/B of library variants on C3: bash scripts/ab_c3.sh <tag> <lib-suffix>...  ("" = libmpcg.so)
set -e
mkdir -p gpurun_out
tag=$1; shift
P=oscar_mpc_planner_mr_modification_amd
for v in "$@"; do
  lib=$P/libmpcg${v:+_$v}.so
  MPCG_LIB=$lib timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k "C3 or c3 or bicycle" --timeout 120 --timeout-method thread > gpurun_out/${tag}_${v:-base}_gpu.log 2>&1 || echo "tests failed for $v"
  MPCG_LIB=$lib timeout -k 10 300 python bench.py --config C3 --no-cpu --steps 5 --warmup 1 > gpurun_out/${tag}_${v:-base}_C3.log 2>&1
done
echo ab-done
