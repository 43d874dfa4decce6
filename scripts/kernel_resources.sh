#!/bin/bash
# Register, scratch and LDS use of every sqp_kernel instance (compiler remarks; CPU only).
#   bash scripts/kernel_resources.sh [extra hipcc flags...]
# one line per kernel: Cfg<N,NL,NE,NS,NX,MODEL> variant | VGPR AGPR scratch(B/lane) LDS(B)
# variant: full (run-time profile switches), lean-hpipm / lean-robust (the profile compiled in);
# -lin / -qp: the split launch's linearisation and interior-point kernels (-DMPCG_SPLIT=1)
C=oscar_mpc_planner_mr_modification_amd/csrc
for f in mpcg_inst_tmpc20 mpcg_inst_tmpc30 mpcg_inst_shmpc mpcg_inst_bicycle; do
  hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Iinclude -I$C "$@" --cuda-device-only -c $C/$f.hip -o /tmp/kr_$f.o \
      -Rpass-analysis=kernel-resource-usage 2>&1 |
    awk '/Function Name: .*sqp_kernel/ {n=$0; sub(/.*CfgIL/,"",n); t=n; sub(/EEE.*/,"",n);
                                         f=(t ~ /Lb1ELi0E/)?"full":((t ~ /Lb0ELi1E/)?"lean-hpipm":((t ~ /Lb0ELi2E/)?"lean-robust":"lean"));
                                         if (t ~ /ELi[0-9]ELi1EEEv/) f=f "-lin"; else if (t ~ /ELi[0-9]ELi2EEEv/) f=f "-qp";
                                         gsub(/ELi/,",",n); sub(/^i/,"",n); name="Cfg<" n "> " f; show=1; next}
         /Function Name:/ {show=0}
         function num() { match($0, /: [0-9]+/); return substr($0, RSTART + 2, RLENGTH - 2) }
         show && /VGPRs:/ {v=num()} show && /AGPRs:/ {a=num()} show && /ScratchSize/ {s=num()}
         show && /LDS Size/ {printf "%-34s VGPR %s AGPR %s scratch %s LDS %s\n", name, v, a, s, num(); show=0}' &
done
wait
