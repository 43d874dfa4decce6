#!/bin/bash
# r03r: the residual / barrier stage algebra split over the parts (split) vs the fused barrier
# pass alone (fuse) -- A/B; then every -m gpu test and smoke on the production build (split)
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 600 python scripts/ab_bench.py --run fuse,split --configs C2,C1,C5,JS,C4,JD --reps 2 > gpurun_out/r03r_ab.jsonl 2> gpurun_out/r03r_ab.err || { echo ab-failed; exit 1; }
echo ab-done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > gpurun_out/r03r_gpu_tests.log 2>&1 || { tail -30 gpurun_out/r03r_gpu_tests.log; exit 1; }
tail -3 gpurun_out/r03r_gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03r_smoke.log 2>&1 || exit 1
echo all-done
