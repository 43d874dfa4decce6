set -e
mkdir -p gpurun_out
P=oscar_mpc_planner_mr_modification_amd
for v in v5a v5b; do
  MPCG_LIB=$P/libmpcg_stamps_$v.so timeout -k 10 200 python scripts/stamp_phases.py > gpurun_out/stamps_$v.log 2>&1
  MPCG_LIB=$P/libmpcg_$v.so timeout -k 10 200 python bench.py --no-cpu > gpurun_out/bench_$v.log 2>&1
done
