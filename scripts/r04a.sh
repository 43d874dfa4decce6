#!/bin/bash
# r04a: interior-point traces of the determined full-SQP divergences
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
T="timeout -k 10 300 python -u scripts/trace_solve.py"
$T --config C2 --scenes 1024 --solve 7414 --lib-solve 7414 --solver-type SQP --variant full > gpurun_out/r04a_c2_7414_sqp_full.log 2>&1 || exit 1
$T --config C2 --scenes 1024 --solve 7414 --lib-solve 7414 --solver-type SQP_RTI --variant full > gpurun_out/r04a_c2_7414_rti_full.log 2>&1 || exit 1
$T --config C2 --scenes 1024 --solve 7414 --lib-solve 7414 --solver-type SQP_RTI --variant lean > gpurun_out/r04a_c2_7414_rti_lean.log 2>&1 || exit 1
$T --config C4 --scenes 2048 --solve 6290 --lib-solve 6290 --solver-type SQP --variant full > gpurun_out/r04a_c4_6290_sqp_full.log 2>&1 || exit 1
echo all-done
