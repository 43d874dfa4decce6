#!/bin/bash
# r03zz: C3 traffic attribution (diagnostic builds only): three solves per CU instead of four
# (pad3: LDS padded over the quarter-CU line) -- time and HBM traffic; the parameter reads' misses
# (p0: every solve reads copy 0's parameters)
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
AB=$PWD/oscar_mpc_planner_mr_modification_amd/build/ab
timeout -k 10 300 python scripts/ab_bench.py --run base,pad3 --configs C3 --reps 2 > gpurun_out/r03zz_ab.jsonl 2> gpurun_out/r03zz_ab.err || { echo ab-failed; exit 1; }
timeout -k 10 300 python scripts/param_locality.py --config C3 --scenes 4096 --natural >> gpurun_out/r03zz_locality.jsonl 2>> gpurun_out/r03zz_locality.err || exit 1
timeout -k 10 300 python scripts/param_locality.py --config C3 --scenes 4096 >> gpurun_out/r03zz_locality.jsonl 2>> gpurun_out/r03zz_locality.err || exit 1
MPCG_LIB=$AB/p0/libmpcg.so timeout -k 10 300 python scripts/param_locality.py --config C3 --scenes 4096 >> gpurun_out/r03zz_locality.jsonl 2>> gpurun_out/r03zz_locality.err || exit 1
echo locality-done
cd /tmp && export TMPDIR=/tmp && cd "$OLDPWD"
for v in base pad3 p0; do
  export MPCG_LIB=$AB/$v/libmpcg.so
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d gpurun_out/prof_r03zz_${v}_fetch -o run --output-format csv \
    -- python3 bench.py --config C3 --no-cpu --steps 3 --warmup 1 > gpurun_out/prof_r03zz_${v}_fetch.log 2>&1 || { echo prof-failed; exit 1; }
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d gpurun_out/prof_r03zz_${v}_write -o run --output-format csv \
    -- python3 bench.py --config C3 --no-cpu --steps 3 --warmup 1 > gpurun_out/prof_r03zz_${v}_write.log 2>&1 || { echo prof-failed; exit 1; }
  echo "profiled $v"
done
echo all-done
