#!/bin/bash
# Quick GPU check: parity tests, C2 / C4 / C5 bench lines (one call, steps chained).
set -e
mkdir -p gpurun_out
tag=${1:-q}
timeout -k 10 300 python -m pytest tests/test_gpu_parity.py tests/test_gpu_scenario.py -x -q > gpurun_out/${tag}_tests.log 2>&1
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu > gpurun_out/${tag}_c2.log 2>&1
timeout -k 10 300 python bench.py --config C4 --scenes 2048 --steps 5 --warmup 1 --no-cpu > gpurun_out/${tag}_c4.log 2>&1
timeout -k 10 600 python bench.py --config C5 --steps 5 --warmup 1 --no-cpu > gpurun_out/${tag}_c5.log 2>&1
echo all-done
