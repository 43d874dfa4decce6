#!/bin/bash
# r03w: final sources -- C5 profile, every -m gpu test, smoke, the C2 and C1 bench lines
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
bash scripts/r03u.sh r03w C5 || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > gpurun_out/r03w_gpu_tests.log 2>&1 || { tail -30 gpurun_out/r03w_gpu_tests.log; exit 1; }
tail -2 gpurun_out/r03w_gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03w_smoke.log 2>&1 || exit 1
for c in C2 C1; do
  t=$(echo "$c" | tr 'A-Z' 'a-z')
  timeout -k 10 400 python bench.py --config $c --steps 20 --warmup 5 > gpurun_out/r03w_bench_$t.json 2> gpurun_out/r03w_bench_$t.err || exit 1
  echo "bench $c done"
done
echo all-done
