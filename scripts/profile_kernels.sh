#!/bin/bash
# Kernel-trace statistics and HBM-traffic counters of the bench workload.
# Run on the GPU box:  bash scripts/profile_kernels.sh <tag>
# Outputs under gpurun_out/prof_<tag>_{trace,fetch,write,sq}/.  Every pass is a
# separate process (PMC passes never combined with trace domains).
set -e
tag=${1:-latest}
shift || true
extra="$@"   # extra bench.py arguments, e.g. --config C5
cd /tmp && export TMPDIR=/tmp && cd "$OLDPWD"
o=gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $o/prof_${tag}_trace -o run --output-format csv \
  -- python3 bench.py --no-cpu --alt-steps 0 --steps 5 --warmup 1 $extra > $o/prof_${tag}_trace.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $o/prof_${tag}_fetch -o run --output-format csv \
  -- python3 bench.py --no-cpu --alt-steps 0 --steps 3 --warmup 1 $extra > $o/prof_${tag}_fetch.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $o/prof_${tag}_write -o run --output-format csv \
  -- python3 bench.py --no-cpu --alt-steps 0 --steps 3 --warmup 1 $extra > $o/prof_${tag}_write.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS \
  -d $o/prof_${tag}_sq -o run --output-format csv \
  -- python3 bench.py --no-cpu --alt-steps 0 --steps 3 --warmup 1 $extra > $o/prof_${tag}_sq.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES \
  -d $o/prof_${tag}_f64 -o run --output-format csv \
  -- python3 bench.py --no-cpu --alt-steps 0 --steps 3 --warmup 1 $extra > $o/prof_${tag}_f64.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES \
  -d $o/prof_${tag}_lanes -o run --output-format csv \
  -- python3 bench.py --no-cpu --alt-steps 0 --steps 3 --warmup 1 $extra > $o/prof_${tag}_lanes.log 2>&1
# the effective clock under load (GRBM_GUI_ACTIVE / 8 XCDs / kernel time) and wave cycles: how much
# of the launch the SIMDs are busy (the tail)
timeout -k 10 300 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
  -d $o/prof_${tag}_clk -o run --output-format csv \
  -- python3 bench.py --no-cpu --alt-steps 0 --steps 3 --warmup 1 $extra > $o/prof_${tag}_clk.log 2>&1
echo profile-done
