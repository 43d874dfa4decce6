#!/bin/bash
# C5 workload with the previous-plan warm start: GPU tests touching C5, full-size parity,
# bench line and profile.
set -e
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_scenario.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_cpp_solver.py -m gpu -x -v --timeout 900 --timeout-method thread > gpurun_out/r02x_gpu.log 2>&1
timeout -k 10 600 python -u scripts/parity_full.py --configs C5 --ws 0 > gpurun_out/r02x_c5_parity.jsonl 2> gpurun_out/r02x_c5_parity.err
bash scripts/r02w_profiles.sh r02x C5
echo all-done
