#!/bin/bash
# r03z: per-phase cycle stamps (diagnostic build) of C2 / C4 / JS on the final sources
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
export MPCG_LIB=oscar_mpc_planner_mr_modification_amd/build/ab/stamps/libmpcg.so
for c in C2 C4 JS; do
  timeout -k 10 300 python scripts/stamp_phases.py $c 1024 > gpurun_out/r03z_stamps_$(echo $c | tr A-Z a-z).txt 2>&1 || { echo stamps-failed-$c; exit 1; }
done
echo all-done
