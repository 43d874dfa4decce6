set -e
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -m pytest tests/test_gpu_parity.py tests/test_gpu_scenario.py -x -q > gpurun_out/a_tests.log 2>&1
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu > gpurun_out/a_c2.log 2>&1
timeout -k 10 600 python bench.py --config C5 --steps 5 --warmup 1 > gpurun_out/a_c5.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d gpurun_out/prof_a_fetch -o run --output-format csv -- python3 bench.py --no-cpu --steps 3 --warmup 1 > gpurun_out/a_fetch.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d gpurun_out/prof_a_write -o run --output-format csv -- python3 bench.py --no-cpu --steps 3 --warmup 1 > gpurun_out/a_write.log 2>&1
echo all-done
