#!/bin/bash
# r03q: predictor barrier pass fused into the residual pass (fuse), + FCONST on N 20 (fusefc),
# + round-robin MIRROR (rr) -- A/B; full-size parity of the rr build; every -m gpu test on the
# production build (fuse)
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 900 python scripts/ab_bench.py --run nofuse,fuse,fusefc,rr --configs C2,C1,C5,JS,C4 --reps 2 > gpurun_out/r03q_ab.jsonl 2> gpurun_out/r03q_ab.err || { echo ab-failed; exit 1; }
echo ab-done
MPCG_LIB=$PWD/oscar_mpc_planner_mr_modification_amd/build/ab/rr/libmpcg.so timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r03q_rr_fullsize.log 2>&1 || { tail -30 gpurun_out/r03q_rr_fullsize.log; exit 1; }
echo rr-fullsize-done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > gpurun_out/r03q_gpu_tests.log 2>&1 || { tail -30 gpurun_out/r03q_gpu_tests.log; exit 1; }
tail -3 gpurun_out/r03q_gpu_tests.log
echo all-done
