#!/bin/bash
# session-3 GPU call 1: C2 bench line with the analytic fp64 roofline; C4 A/B of the constant
# [B A] rows (libmpcg_fca.so) against the production library
set -e
mkdir -p gpurun_out
P=oscar_mpc_planner_mr_modification_amd
timeout -k 10 300 python bench.py > gpurun_out/s3_bench_c2.json 2> gpurun_out/s3_bench_c2.err
MPCG_LIB=$P/libmpcg_fca.so timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -x -q -k "c4 or C4" --timeout 120 --timeout-method thread > gpurun_out/s3_fca_c4_tests.log 2>&1
for v in base fca; do
  lib=$P/libmpcg.so; [ $v = fca ] && lib=$P/libmpcg_fca.so
  MPCG_LIB=$lib timeout -k 10 300 python bench.py --config C4 --no-cpu --steps 5 --warmup 1 > gpurun_out/s3_${v}_C4.json 2>/dev/null
  MPCG_LIB=$lib timeout -k 10 300 python bench.py --config JS --no-cpu --steps 5 --warmup 1 > gpurun_out/s3_${v}_JS.json 2>/dev/null
done
echo call1-done
