#!/bin/bash
# Register budget of the solve kernel (CPU only): VGPR, AGPR and
# scratch of the lean kernels at one wave per SIMD (production) and under a two-wave budget
# (MPCG_WAVES_PER_EU=2 with a 128-lane launch bound so the 40 KB LDS block does not clamp it), with
# the linearisation left out (MPCG_DIAG_NO_LIN: what the interior point alone keeps live) and with
# six lane parts per stage instead of three (MPCG_PARTS_OVERRIDE=6 on an N 9, 8 + 8 rows shape: the
# row state and the chain rows of a lane halved).  The two diagnostic switches are patched into a
# temporary copy of the sources (compiled, never run); the shipped sources stay as they are.
#   bash scripts/register_budget.sh > profiles/r04_register_budget.txt
C=/tmp/rb_csrc
rm -rf $C && cp -r oscar_mpc_planner_mr_modification_amd/csrc $C
python3 - $C/mpcg_sqp.h <<'PY'
import sys
p = sys.argv[1]
s = open(p).read()
old = "    static constexpr int PARTS_MAX = (64 / (N + 1)) >= 3 ? 3 : 2;"
assert s.count(old) == 1
s = s.replace(old, "#ifdef MPCG_PARTS_OVERRIDE\n    static constexpr int PARTS_MAX = MPCG_PARTS_OVERRIDE;\n#else\n" + old + "\n#endif")
old = "            if (stage_lane && k < N) {\n                double g[NZ], xn[NX], pi[NX];"
assert s.count(old) == 1
s = s.replace(old, "#ifdef MPCG_DIAG_NO_LIN\n            if (false) {\n#else\n            if (stage_lane && k < N) {\n#endif\n"
              "                double g[NZ], xn[NX], pi[NX];")
open(p, "w").write(s)
PY
res() {  # res <label> <source> <kernel-name filter> <flags...>
  local label=$1 src=$2 filt=$3; shift 3
  hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Iinclude -I$C "$@" --cuda-device-only -c $src -o /tmp/rb.o \
      -Rpass-analysis=kernel-resource-usage 2>&1 |
    awk -v l="$label" -v f="$filt" '/Function Name:/ {show = ($0 ~ f) && ($0 ~ /Lb0E/)}
         function num() { match($0, /: [0-9]+/); return substr($0, RSTART + 2, RLENGTH - 2) }
         show && /VGPRs:/ {v=num()} show && /AGPRs:/ {a=num()} show && /ScratchSize/ {s=num()}
         show && /Occupancy/ {printf "%-58s VGPR %3s AGPR %3s scratch %4s B/lane  waves/SIMD %s\n", l, v, a, s, num(); show=0}'
}
W2="-DMPCG_WAVES_PER_EU=2 -DMPCG_WG_LANES=128"
res "C2 lean, production (1 wave/SIMD)" $C/mpcg_inst_tmpc20.hip "ILi20ELi8ELi8E"
res "C2 lean, two-wave budget" $C/mpcg_inst_tmpc20.hip "ILi20ELi8ELi8E" $W2
res "C2 lean, interior point only" $C/mpcg_inst_tmpc20.hip "ILi20ELi8ELi8E" -DMPCG_DIAG_NO_LIN
res "C2 lean, interior point only, two-wave budget" $C/mpcg_inst_tmpc20.hip "ILi20ELi8ELi8E" -DMPCG_DIAG_NO_LIN $W2
printf '#include "mpcg_instance.h"\nMPCG_DEFINE_INSTANCE(9, 8, 8, 0, 5, 0)\n' > /tmp/rb_n9.hip
for p in 3 6; do
  res "N 9, 8+8 rows, $p parts" /tmp/rb_n9.hip "ILi9ELi8ELi8E" -DMPCG_PARTS_OVERRIDE=$p
  res "N 9, 8+8 rows, $p parts, interior point only" /tmp/rb_n9.hip "ILi9ELi8ELi8E" -DMPCG_PARTS_OVERRIDE=$p -DMPCG_DIAG_NO_LIN
done
