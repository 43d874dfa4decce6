#!/bin/bash
# r03j: PC sampling (host trap) of the C2 solve kernel, line-table build
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$OLDPWD"
export MPCG_LIB=oscar_mpc_planner_mr_modification_amd/build/ab/dbg/libmpcg.so
timeout -k 10 240 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method host_trap --pc-sampling-unit time \
  --pc-sampling-interval 1 -d /tmp/r03j_pcs -o pcs --output-format csv \
  -- python3 bench.py --config C2 --no-cpu --steps 2 --warmup 1 > gpurun_out/r03j_pcs.log 2>&1 || { echo pcs-failed; tail -20 gpurun_out/r03j_pcs.log; exit 1; }
find /tmp/r03j_pcs -name "*.csv" -exec ls -la {} \; > gpurun_out/r03j_files.txt
f=$(find /tmp/r03j_pcs -name "*pc_sampling*.csv" | head -1)
[ -n "$f" ] || { echo no-pcs-csv; cat gpurun_out/r03j_files.txt; exit 1; }
python3 scripts/pcs_summary.py "$f" gpurun_out/r03j_c2 > gpurun_out/r03j_summary.txt 2>&1 || exit 1
cat gpurun_out/r03j_summary.txt
echo all-done
