#!/bin/bash
# r03n: even conflict-free cost-to-go stride on the long horizons (C4 15 -> 18, C3 21 -> 22) A/B
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 700 python scripts/ab_bench.py --run hoist,palign,c3hoist --configs C4,C3 --reps 2 > gpurun_out/r03n_ab.jsonl 2> gpurun_out/r03n_ab.err || { echo ab-failed; exit 1; }
echo all-done
