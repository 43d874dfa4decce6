#!/bin/bash
# diagnostic build with per-phase s_memtime stamps (never the measured library)
cd "$(dirname "$0")/.."
python3 -c "
from oscar_mpc_planner_mr_modification_amd import _build
_build.build_lib(force=True, extra_flags=['-DMPCG_STAMPS'], out=_build.os.path.join(_build.PKG, 'libmpcg_stamps.so'))"
