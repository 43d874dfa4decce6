#!/bin/bash
# r03x: final sources -- the bench lines of C5, JS, JD, C3, C4 (with their CPU baselines)
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for c in C5 JS JD C3 C4; do
  t=$(echo "$c" | tr 'A-Z' 'a-z')
  timeout -k 10 400 python bench.py --config $c --steps 20 --warmup 5 > gpurun_out/r03x_bench_$t.json 2> gpurun_out/r03x_bench_$t.err || exit 1
  echo "bench $c done"
done
echo all-done
timeout -k 10 300 python scripts/latency.py --config JS --guesses 5 > gpurun_out/r03x_latency_js.json 2> gpurun_out/r03x_latency_js.err || exit 1
timeout -k 10 300 python scripts/latency.py --config C2 --guesses 8 > gpurun_out/r03x_latency_c2.json 2> gpurun_out/r03x_latency_c2.err || exit 1
echo latency-done
