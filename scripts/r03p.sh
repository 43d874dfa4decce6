#!/bin/bash
# r03p: one reduction for the three IPM residual maxima A/B
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 800 python scripts/ab_bench.py --run c3h2,redmax --configs C2,C4,JS,C5 --reps 2 > gpurun_out/r03p_ab.jsonl 2> gpurun_out/r03p_ab.err || { echo ab-failed; exit 1; }
echo all-done
