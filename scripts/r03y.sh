#!/bin/bash
# r03y: full-size parity records of every config on the final sources (the reference's QP start;
# C5B = C5 from the braking plan) and of solver_type SQP
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u scripts/parity_full.py --configs C2,C1,C3,C4,C5,C5B,JS,JD --ws 2 --warm-first 0 > gpurun_out/r03y_fullsize_parity.jsonl 2> gpurun_out/r03y_fullsize_parity.err || exit 1
timeout -k 10 600 python -u scripts/parity_full.py --configs C2,C1,C4 --ws 2 --warm-first 0 --solver-type SQP > gpurun_out/r03y_sqp_parity.jsonl 2> gpurun_out/r03y_sqp_parity.err || exit 1
echo all-done
