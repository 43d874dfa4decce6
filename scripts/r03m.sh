#!/bin/bash
# r03m: constant [B A] rows hoisted out of the Riccati recursion -- A/B, then every -m gpu test,
# smoke and the C2 bench line on these sources
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 700 python scripts/ab_bench.py --run base,hoist --configs JS,C4,JD,C2 --reps 2 > gpurun_out/r03m_ab.jsonl 2> gpurun_out/r03m_ab.err || { echo ab-failed; exit 1; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > gpurun_out/r03m_gpu_tests.log 2>&1 || { tail -30 gpurun_out/r03m_gpu_tests.log; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03m_smoke.log 2>&1 || exit 1
timeout -k 10 400 python bench.py --config C2 --steps 20 --warmup 5 > gpurun_out/r03m_bench_c2.json 2> gpurun_out/r03m_bench_c2.err || exit 1
tail -3 gpurun_out/r03m_gpu_tests.log
echo all-done
