#!/bin/bash
set -e
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_fullsize.py -m gpu -v -s --timeout 900 --timeout-method thread > gpurun_out/r02y_fullsize.log 2>&1
echo all-done
