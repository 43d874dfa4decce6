#!/bin/bash
# r03k: stored 1/t up to 12 slots (JD and C5 scratch-free) A/B; per-phase cycle stamps of C2 / C4 / JS
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 600 python scripts/ab_bench.py --run cur,jd12,bsel4 --configs JD,C5,C4 --reps 2 > gpurun_out/r03k_ab.jsonl 2> gpurun_out/r03k_ab.err || { echo ab-failed; exit 1; }
export MPCG_LIB=oscar_mpc_planner_mr_modification_amd/build/ab/stamps/libmpcg.so
for c in C2 C4 JS; do
  timeout -k 10 300 python scripts/stamp_phases.py $c 1024 > gpurun_out/r03k_stamps_$(echo $c | tr A-Z a-z).txt 2>&1 || { echo stamps-failed-$c; exit 1; }
done
echo all-done
