#!/bin/bash
# r03a: C5 copy 7799 side-by-side IPM trace (GPU diagnostic build vs oracle), the GPU test
# suite on the current tree, the CPU share of the box, and bench.py --gpus 2 spawning its own
# ranks (gloo rehearsal on the one GPU).
set -e
mkdir -p gpurun_out
{ nproc; cat /sys/fs/cgroup/cpu.max 2>/dev/null || true; python -c "import bench, json; print(json.dumps(bench.cpu_share()))"; } > gpurun_out/r03a_cpu_share.txt 2>&1
timeout -k 10 300 python -u scripts/trace_solve.py --config C5 --scene 1949 --solve 3 > gpurun_out/r03a_trace_7799.log 2>&1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r03a_gpu_tests.log 2>&1
MPCG_BENCH_BACKEND=gloo timeout -k 10 400 python bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu > gpurun_out/r03a_spawn_gloo.json 2> gpurun_out/r03a_spawn_gloo.err
echo all-done
