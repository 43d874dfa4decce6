#!/bin/bash
# Instruction-cache counters of the solve kernel (one PMC pass of 8 SQ-block counters; gfx950 counts the
# SQC instruction-cache events in the SQ block).  GPU box:  bash scripts/icache_pass.sh <tag> [bench args]
set -e
tag=${1:-latest}
shift || true
cd /tmp && export TMPDIR=/tmp && cd "$OLDPWD"
o=gpurun_out
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
  -d $o/prof_${tag}_icache -o run --output-format csv \
  -- python3 bench.py --no-cpu --alt-steps 0 --steps 3 --warmup 1 "$@" > $o/prof_${tag}_icache.log 2>&1
echo icache-done
