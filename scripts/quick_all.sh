#!/bin/bash
# GPU check after a kernel change: parity tests, then C2 / C3 / C4 / C5 bench lines
# (no CPU baseline).  bash scripts/quick_all.sh <tag> [skip-tests]
set -e
mkdir -p gpurun_out
tag=${1:-q}
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${tag}_gpu.log 2>&1
fi
timeout -k 10 300 python bench.py --no-cpu > gpurun_out/${tag}_c2.log 2>&1
timeout -k 10 300 python bench.py --config C3 --no-cpu --steps 5 --warmup 1 > gpurun_out/${tag}_c3.log 2>&1
timeout -k 10 300 python bench.py --config C4 --no-cpu --steps 5 --warmup 1 > gpurun_out/${tag}_c4.log 2>&1
timeout -k 10 300 python bench.py --config C5 --no-cpu --steps 5 --warmup 1 > gpurun_out/${tag}_c5.log 2>&1
echo all-done
