#!/bin/bash
# diagnostic build with per-phase s_memtime stamps (never the measured library)
cd "$(dirname "$0")/.."
hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -DMPCG_STAMPS -Iinclude \
  -Ioscar_mpc_planner_mr_modification_amd/csrc oscar_mpc_planner_mr_modification_amd/csrc/mpcg_kernels.hip \
  -o oscar_mpc_planner_mr_modification_amd/libmpcg_stamps.so
