#!/bin/bash
# Final check of the round's tree: every -m gpu test, smoke, the default bench line (C2, counters
# from the profile keyed to these sources), and the cold/warm QP-start parity of the C5 workload.
set -e
mkdir -p gpurun_out
bash scripts/round_check.sh r02y
timeout -k 10 600 python -u scripts/parity_full.py --configs C5 --ws 0,2 > gpurun_out/r02y_c5_ws_parity.jsonl 2> gpurun_out/r02y_c5_ws_parity.err
echo all-done
