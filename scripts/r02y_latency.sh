#!/bin/bash
set -e
mkdir -p gpurun_out
timeout -k 10 300 python scripts/latency.py --config JS --guesses 5 --reps 200 > gpurun_out/r02y_latency_js.json 2> gpurun_out/r02y_latency_js.err
timeout -k 10 300 python scripts/latency.py --config C2 --guesses 8 --reps 200 > gpurun_out/r02y_latency_c2.json 2> gpurun_out/r02y_latency_c2.err
echo all-done
