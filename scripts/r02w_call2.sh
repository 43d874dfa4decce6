#!/bin/bash
# Full-size cold/warm QP-start parity (C2/C4/C5) and the C2 profile on the current sources.
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u scripts/parity_full.py --configs C2,C4,C5 --ws 0,2 > gpurun_out/r02w_ws_parity.jsonl 2> gpurun_out/r02w_ws_parity.err
bash scripts/profile_kernels.sh r02w_c2 --config C2
echo all-done
