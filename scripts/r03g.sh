#!/bin/bash
# r03g: profiles of C3, C4, JD on the final sources, and the drop-in latency of the shipped solvers
mkdir -p gpurun_out
bash scripts/r03f.sh C3 C4 JD || exit 1
timeout -k 10 300 python scripts/latency.py --config JD --guesses 5 > gpurun_out/r03g_latency_jd.json 2> gpurun_out/r03g_latency_jd.err || exit 1
timeout -k 10 300 python scripts/latency.py --config JS --guesses 5 > gpurun_out/r03g_latency_js.json 2> gpurun_out/r03g_latency_js.err || exit 1
timeout -k 10 300 python scripts/latency.py --config C2 --guesses 8 --solver-type SQP > gpurun_out/r03g_latency_c2_sqp.json 2> gpurun_out/r03g_latency_c2_sqp.err || exit 1
echo all-done
