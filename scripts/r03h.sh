#!/bin/bash
# r03h: conflict-minimal LDS strides -- parity on the padded build, A/B timing, bank-conflict counters
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_instances.py > gpurun_out/r03h_tests.log 2>&1 || { echo tests-failed; tail -20 gpurun_out/r03h_tests.log; exit 1; }
timeout -k 10 900 python scripts/ab_bench.py --run nopad,pad --configs C2,C1,C4,JS,JD --reps 2 > gpurun_out/r03h_ab.jsonl 2> gpurun_out/r03h_ab.err || { echo ab-failed; exit 1; }
for v in nopad pad; do
  MPCG_LIB=oscar_mpc_planner_mr_modification_amd/build/ab/$v/libmpcg.so timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAVE_CYCLES -d gpurun_out/r03h_pmc_$v -o pmc --output-format csv -- python bench.py --config C2 --no-cpu --steps 3 --warmup 1 > gpurun_out/r03h_pmc_$v.log 2>&1 || { echo pmc-failed-$v; exit 1; }
done
echo all-done
