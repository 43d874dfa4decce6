#!/bin/bash
# r03s: feedback multipliers split over the parts (base) vs not (nopin); the fused barrier pass on
# C3 (base vs nofuse); every -m gpu test, smoke, the C2 bench line on the production build
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 400 python scripts/ab_bench.py --run nopin,base --configs C2,C1,C5 --reps 2 > gpurun_out/r03s_ab.jsonl 2> gpurun_out/r03s_ab.err || { echo ab-failed; exit 1; }
timeout -k 10 300 python scripts/ab_bench.py --run nofuse,base --configs C3 --reps 2 >> gpurun_out/r03s_ab.jsonl 2>> gpurun_out/r03s_ab.err || { echo ab-failed; exit 1; }
echo ab-done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > gpurun_out/r03s_gpu_tests.log 2>&1 || { tail -30 gpurun_out/r03s_gpu_tests.log; exit 1; }
tail -3 gpurun_out/r03s_gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03s_smoke.log 2>&1 || exit 1
timeout -k 10 400 python bench.py --config C2 --steps 20 --warmup 5 > gpurun_out/r03s_bench_c2.json 2> gpurun_out/r03s_bench_c2.err || exit 1
echo all-done
