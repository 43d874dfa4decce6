#!/bin/bash
# r03l: checkpoint on the padded-stride sources: every -m gpu test, smoke, C2 bench line
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > gpurun_out/r03l_gpu_tests.log 2>&1 || { tail -30 gpurun_out/r03l_gpu_tests.log; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03l_smoke.log 2>&1 || exit 1
timeout -k 10 400 python bench.py --config C2 --steps 20 --warmup 5 > gpurun_out/r03l_bench_c2.json 2> gpurun_out/r03l_bench_c2.err || exit 1
tail -3 gpurun_out/r03l_gpu_tests.log
echo all-done
