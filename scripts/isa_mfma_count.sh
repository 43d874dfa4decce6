#!/bin/bash
# MFMA instructions in every sqp_kernel instance's gfx950 ISA (CPU only; the evidence behind the
# bench line's roofline.mfma).  One line per kernel: instructions, v_mfma_*, fp64 VALU (v_*_f64).
#   bash scripts/isa_mfma_count.sh > profiles/r04_isa_mfma.txt
C=oscar_mpc_planner_mr_modification_amd/csrc
for f in mpcg_inst_tmpc20 mpcg_inst_tmpc30 mpcg_inst_shmpc mpcg_inst_bicycle mpcg_kernels mpcg_prepare; do
  hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Iinclude -I$C --cuda-device-only -S $C/$f.hip -o /tmp/isa_$f.s || exit 1
  awk -v file=$f '
    /^_Z[_A-Za-z0-9]+:/ && /kernel/ {name=$1; sub(/:$/,"",name); sub(/PyPd$|Pd$/,"",name); n=0; m=0; d=0; inside=1; next}
    inside && /^[ \t]+s_endpgm/ {n++; printf "%-22s %-60.60s insts %6d mfma %d f64_valu %d\n", file, name, n, m, d; inside=0; next}
    inside && /^[ \t]+[sv]_|^[ \t]+ds_|^[ \t]+global_|^[ \t]+buffer_|^[ \t]+scratch_|^[ \t]+flat_/ {n++; if ($1 ~ /^v_mfma/) m++; if ($1 ~ /^v_.*_f64/) d++}
  ' /tmp/isa_$f.s
done
