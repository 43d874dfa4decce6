#!/bin/bash
# Round check on the GPU box: every -m gpu test, smoke(), the default bench line
# (C2 with the CPU baseline).  bash scripts/round_check.sh <tag>
set -e
mkdir -p gpurun_out
tag=${1:-rc}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 900 --timeout-method thread > gpurun_out/${tag}_gpu.log 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${tag}_smoke.log 2>&1
timeout -k 10 400 python bench.py > gpurun_out/${tag}_bench.log 2>&1
echo all-done
