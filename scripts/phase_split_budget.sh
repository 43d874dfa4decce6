#!/bin/bash
# Scratch of the lean HPIPM-profile kernel of every instance with the SQP body whole, with the interior
# point compiled out (MPCG_DIAG_LIN_ONLY: the linearisation alone -- what a linearisation kernel of its
# own would allocate) and with the linearisation compiled out (MPCG_DIAG_NO_LIN: what an interior-point
# kernel of its own would allocate).  VERDICT r05 item 2: the case for splitting the SQP loop into two
# kernels per RTI iteration.  Both switches are patched into a temporary copy of the sources (compiled,
# never run); the shipped sources stay as they are.  CPU only.
#   bash scripts/phase_split_budget.sh > profiles/r06f_phase_split_budget.txt
C=/tmp/psb_csrc
rm -rf $C && cp -r oscar_mpc_planner_mr_modification_amd/csrc $C
python3 - $C/mpcg_sqp_body.inc <<'PY'
import sys
p = sys.argv[1]
s = open(p).read()
old = "            if (stage_lane && k < N) {\n                double g[NZ], xn[NX], pi[NX];"
assert s.count(old) == 1
s = s.replace(old, "#ifdef MPCG_DIAG_NO_LIN\n            if (false) {\n#else\n            if (stage_lane && k < N) {\n#endif\n"
              "                double g[NZ], xn[NX], pi[NX];")
old = "        for (;; ++qit) {"
assert s.count(old) == 1
s = s.replace(old, "#ifdef MPCG_DIAG_LIN_ONLY\n        qstat = AC_SUCCESS;\n        if (lane < 1000) goto lin_only_skip;\n#endif\n" + old)
old = "        wave_sync();\n        qp_status = qstat;"
assert s.count(old) == 1
s = s.replace(old, "#ifdef MPCG_DIAG_LIN_ONLY\n        lin_only_skip:\n#endif\n" + old)
open(p, "w").write(s)
PY
run() {  # run <label> <flags...>
  local label=$1; shift
  for f in mpcg_inst_tmpc20 mpcg_inst_tmpc30 mpcg_inst_shmpc mpcg_inst_bicycle; do
    hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Iinclude -I$C "$@" --cuda-device-only -c $C/$f.hip -o /tmp/psb_$f.o \
        -Rpass-analysis=kernel-resource-usage 2>&1 |
      awk -v l="$label" '/Function Name: .*sqp_kernel/ {n=$0; sub(/.*CfgIL/,"",n); t=n; sub(/EEE.*/,"",n);
                                           gsub(/ELi/,",",n); sub(/^i/,"",n); show=(t ~ /Lb0ELi1E/) && (n !~ /^10,/); next}
           /Function Name:/ {show=0}
           function num() { match($0, /: [0-9]+/); return substr($0, RSTART + 2, RLENGTH - 2) }
           show && /VGPRs:/ {v=num()} show && /AGPRs:/ {a=num()} show && /ScratchSize/ {s=num()}
           show && /LDS Size/ {printf "%-24s Cfg<%s> lean-hpipm  VGPR %s AGPR %s scratch %s B/lane\n", l, n, v, a, s; show=0}' &
  done
  wait
}
run "whole SQP body"
run "linearisation only" -DMPCG_DIAG_LIN_ONLY
run "interior point only" -DMPCG_DIAG_NO_LIN
