#!/bin/bash
# r03c: the whole GPU suite (no -x: every result), the variants once, the default bench line,
# bench.py --gpus 2 spawning its own ranks, a trace of a rounding-decided braking-plan copy,
# A/B of the bounds-select switch, the restated warm start and solver_type SQP at full size.
mkdir -p gpurun_out
timeout -k 10 1500 python -u -m pytest tests -m gpu -v --timeout 900 --timeout-method thread > gpurun_out/r03c_gpu_tests.log 2>&1
echo "pytest rc=$?"
timeout -k 10 300 python -u scripts/variant_parity.py --run storeit > gpurun_out/r03c_variant_storeit.jsonl 2> gpurun_out/r03c_variant_storeit.err || exit 1
timeout -k 10 300 python -u scripts/variant_parity.py --run bike3 > gpurun_out/r03c_variant_bike3.jsonl 2> gpurun_out/r03c_variant_bike3.err || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r03c_bench_c2.json 2> gpurun_out/r03c_bench_c2.err || exit 1
MPCG_BENCH_BACKEND=gloo timeout -k 10 400 python bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu > gpurun_out/r03c_spawn_gloo.json 2> gpurun_out/r03c_spawn_gloo.err || exit 1
timeout -k 10 300 python -u scripts/trace_solve.py --config C5 --braking --scene 1633 --solve 1 > gpurun_out/r03c_trace_c5b_6533.log 2>&1 || exit 1
timeout -k 10 600 python -u scripts/ab_bench.py --run base,bsel --configs C2,C3,C4 > gpurun_out/r03c_ab_bsel.jsonl 2> gpurun_out/r03c_ab_bsel.err || exit 1
timeout -k 10 600 python -u scripts/parity_full.py --configs C2,C4,C5 --ws 2 --warm-first 1 > gpurun_out/r03c_ws_parity.jsonl 2> gpurun_out/r03c_ws_parity.err || exit 1
timeout -k 10 600 python -u scripts/parity_full.py --configs C2,C1,C4 --ws 2 --warm-first 0 --solver-type SQP > gpurun_out/r03c_sqp_parity.jsonl 2> gpurun_out/r03c_sqp_parity.err || exit 1
echo all-done
