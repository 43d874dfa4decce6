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
