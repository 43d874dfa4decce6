#!/bin/bash
# r03b: the GPU suite on ABI 6 (full-size parity of every config against the default oracle,
# solver_type SQP parity, the rounding-decided C5 copy, JD), the stored-1/t and three-part
# bicycle variants once, the default bench line, and bench.py --gpus 2 spawning its ranks.
set -e
mkdir -p gpurun_out
timeout -k 10 1200 python -u -m pytest tests -m gpu -x -v --timeout 900 --timeout-method thread > gpurun_out/r03b_gpu_tests.log 2>&1
timeout -k 10 300 python -u scripts/variant_parity.py --run storeit > gpurun_out/r03b_variant_storeit.jsonl 2> gpurun_out/r03b_variant_storeit.err
timeout -k 10 300 python -u scripts/variant_parity.py --run bike3 > gpurun_out/r03b_variant_bike3.jsonl 2> gpurun_out/r03b_variant_bike3.err
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r03b_bench_c2.json 2> gpurun_out/r03b_bench_c2.err
MPCG_BENCH_BACKEND=gloo timeout -k 10 400 python bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu > gpurun_out/r03b_spawn_gloo.json 2> gpurun_out/r03b_spawn_gloo.err
echo all-done
