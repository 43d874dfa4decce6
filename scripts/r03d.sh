#!/bin/bash
# r03d: A/B of stored 1/t on the two-part (JS, JD) and the 14-slot (C5) instances; full-size
# parity records of every config (cold / reference QP start), the restated warm start and
# solver_type SQP with the capped-QP statistics.
mkdir -p gpurun_out
timeout -k 10 900 python -u scripts/ab_bench.py --run base,storeit --configs JS,JD --reps 2 > gpurun_out/r03d_ab_storeit.jsonl 2> gpurun_out/r03d_ab_storeit.err || exit 1
timeout -k 10 600 python -u scripts/ab_bench.py --run base,sit14 --configs C5 --reps 2 > gpurun_out/r03d_ab_sit14.jsonl 2> gpurun_out/r03d_ab_sit14.err || exit 1
timeout -k 10 900 python -u scripts/parity_full.py --configs C1,C2,C3,C4,C5,C5B,JS,JD --ws 2 --warm-first 0 > gpurun_out/r03d_fullsize_parity.jsonl 2> gpurun_out/r03d_fullsize_parity.err || exit 1
timeout -k 10 600 python -u scripts/parity_full.py --configs C2,C4,C5 --ws 2 --warm-first 1 > gpurun_out/r03d_ws_parity.jsonl 2> gpurun_out/r03d_ws_parity.err || exit 1
timeout -k 10 600 python -u scripts/parity_full.py --configs C2,C1,C4 --ws 2 --warm-first 0 --solver-type SQP > gpurun_out/r03d_sqp_parity.jsonl 2> gpurun_out/r03d_sqp_parity.err || exit 1
echo all-done
