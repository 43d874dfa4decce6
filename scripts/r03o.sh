#!/bin/bash
# r03o: C3 with its constant [B A] rows hoisted (odd cost-to-go stride); branch-free Y / Cholesky
# stores on the three-part instances (C1, C2)
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 700 python scripts/ab_bench.py --run hoist,c3h2 --configs C3 --reps 2 > gpurun_out/r03o_ab.jsonl 2> gpurun_out/r03o_ab.err || { echo ab-failed; exit 1; }
timeout -k 10 700 python scripts/ab_bench.py --run hoist,flatyl --configs C2,C1 --reps 2 >> gpurun_out/r03o_ab.jsonl 2>> gpurun_out/r03o_ab.err || { echo ab-failed; exit 1; }
echo all-done
