#!/bin/bash
# r03e: final-sources check: every -m gpu test, smoke, the bench line of every config (with the
# CPU baseline and parity legs) and the rocprofv3 passes of the north-star config C2.
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > gpurun_out/r03e_gpu_tests.log 2>&1 || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03e_smoke.log 2>&1 || exit 1
for c in C2 C1 C3 C4 C5 JS JD; do
  t=$(echo "$c" | tr 'A-Z' 'a-z')
  timeout -k 10 400 python bench.py --config $c --steps 20 --warmup 5 > gpurun_out/r03e_bench_$t.json 2> gpurun_out/r03e_bench_$t.err || exit 1
done
bash scripts/profile_kernels.sh r03e_c2 --config C2 > gpurun_out/r03e_prof_c2.log 2>&1 || exit 1
echo all-done
