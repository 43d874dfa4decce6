#!/bin/bash
# Profile several bench configurations in one GPU call:
#   bash scripts/profile_configs.sh <tag-prefix> C2 C3 JS
# runs scripts/profile_kernels.sh <prefix>_<cfg> --config <cfg> for each; stops at the first failure.
set -e
prefix=$1
shift
for c in "$@"; do
  t=${prefix}_$(echo "$c" | tr 'A-Z' 'a-z')
  bash scripts/profile_kernels.sh "$t" --config "$c"
  echo "profiled $c"
done
