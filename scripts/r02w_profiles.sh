#!/bin/bash
# Bench line (with the CPU baseline) and the rocprofv3 passes of each named config on the
# current sources:  bash scripts/r02w_profiles.sh <tag-prefix> C5 C1 JS
set -e
mkdir -p gpurun_out
prefix=$1
shift
for c in "$@"; do
  t=${prefix}_$(echo "$c" | tr 'A-Z' 'a-z')
  timeout -k 10 400 python bench.py --config "$c" > gpurun_out/${t}_bench.log 2>&1
  bash scripts/profile_kernels.sh "$t" --config "$c"
  echo "done $c"
done
echo all-done
