#!/bin/bash
# r03u / r03v: rocprofv3 passes (kernel stats, HBM traffic, wave-cycle shares, fp64 and lane counters)
# of the final sources:  bash scripts/r03u.sh <tag-prefix> C2 C1 C5
mkdir -p gpurun_out
pfx=$1; shift
for c in "$@"; do
  t=${pfx}_$(echo "$c" | tr 'A-Z' 'a-z')
  bash scripts/profile_kernels.sh "$t" --config "$c" > gpurun_out/${t}_prof.log 2>&1 || { echo "profile $c failed"; tail -5 gpurun_out/${t}_prof.log; exit 1; }
  echo "profiled $c"
done
echo all-done
