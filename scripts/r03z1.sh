#!/bin/bash
# r03z1: final sources -- every -m gpu test, smoke, the bench line of every config
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > gpurun_out/r03z_gpu_tests.log 2>&1 || { tail -30 gpurun_out/r03z_gpu_tests.log; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03z_smoke.log 2>&1 || exit 1
for c in C2 C1 C3 C4 C5 JS JD; do
  t=$(echo "$c" | tr 'A-Z' 'a-z')
  timeout -k 10 400 python bench.py --config $c --steps 20 --warmup 5 > gpurun_out/r03z_bench_$t.json 2> gpurun_out/r03z_bench_$t.err || exit 1
  echo "bench $c done"
done
tail -3 gpurun_out/r03z_gpu_tests.log
echo all-done
