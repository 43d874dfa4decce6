#!/bin/bash
# r03t: MIRROR's eigenvector rows split over the parts (base) vs one lane per stage (nomsplit):
# A/B, and a bit-for-bit comparison of the two builds' outputs on the bench batches
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 700 python scripts/ab_bench.py --run nomsplit,base --configs C2,C1,C5,C4,JS,JD --reps 2 > gpurun_out/r03t_ab.jsonl 2> gpurun_out/r03t_ab.err || { echo ab-failed; exit 1; }
echo ab-done
AB=oscar_mpc_planner_mr_modification_amd/build/ab
for c in C2 C5 C4 JS; do
  for v in base nomsplit; do
    MPCG_LIB=$PWD/$AB/$v/libmpcg.so timeout -k 10 120 python scripts/bitcmp.py dump gpurun_out/r03t_${c}_$v.npz --config $c --scenes 512 >> gpurun_out/r03t_bitcmp.log 2>&1 || { echo dump-failed; exit 1; }
  done
  echo "== $c" >> gpurun_out/r03t_bitcmp.log
  python scripts/bitcmp.py cmp gpurun_out/r03t_${c}_base.npz gpurun_out/r03t_${c}_nomsplit.npz >> gpurun_out/r03t_bitcmp.log 2>&1
done
rm -f gpurun_out/r03t_*.npz
cat gpurun_out/r03t_bitcmp.log | grep -v "^gpurun_out"
echo all-done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > gpurun_out/r03t_gpu_tests.log 2>&1 || { tail -30 gpurun_out/r03t_gpu_tests.log; exit 1; }
tail -2 gpurun_out/r03t_gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03t_smoke.log 2>&1 || exit 1
for c in C2 C5; do
  t=$(echo "$c" | tr 'A-Z' 'a-z')
  timeout -k 10 400 python bench.py --config $c --steps 20 --warmup 5 --no-cpu > gpurun_out/r03t_bench_$t.json 2> gpurun_out/r03t_bench_$t.err || exit 1
done
echo all-done2
