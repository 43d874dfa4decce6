#!/bin/bash
# r03i: even-stride gradient rows (JS, JD, C4) A/B; what the parameter reads' misses cost C4
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 600 python scripts/ab_bench.py --run nopad,pad2 --configs JS,C4,JD --reps 2 > gpurun_out/r03i_ab.jsonl 2> gpurun_out/r03i_ab.err || { echo ab-failed; exit 1; }
for cfg in C4 JS; do
  timeout -k 10 300 python scripts/param_locality.py --config $cfg --natural >> gpurun_out/r03i_locality.jsonl 2>> gpurun_out/r03i_locality.err || exit 1
  timeout -k 10 300 python scripts/param_locality.py --config $cfg >> gpurun_out/r03i_locality.jsonl 2>> gpurun_out/r03i_locality.err || exit 1
  MPCG_LIB=oscar_mpc_planner_mr_modification_amd/build/ab/p0/libmpcg.so timeout -k 10 300 python scripts/param_locality.py --config $cfg >> gpurun_out/r03i_locality.jsonl 2>> gpurun_out/r03i_locality.err || exit 1
done
echo all-done
