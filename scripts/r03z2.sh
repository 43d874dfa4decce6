#!/bin/bash
# r03z2 / r03z3: rocprofv3 passes (kernel stats, HBM traffic, fp64 / lane counters) per config on
# the final sources:  bash scripts/r03z2.sh C2 C1 C5 JS
mkdir -p gpurun_out
for c in "$@"; do
  t=r03z_$(echo "$c" | tr 'A-Z' 'a-z')
  bash scripts/profile_kernels.sh "$t" --config "$c" > gpurun_out/${t}_prof.log 2>&1 || exit 1
  echo "profiled $c"
done
echo all-done
