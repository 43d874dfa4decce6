#!/bin/bash
# Round-6 GPU recipes, one named step per argument (each step under its own time limit; the
# first failing step ends the call):
#   bash scripts/r06.sh trace parity sqp tests smoke bench profile
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
tag=${R06_TAG:-r06}
step() {  # step <name> <seconds> <output file> <command...>
  local name=$1 secs=$2 out=$3; shift 3
  echo "[$(date +%T)] $name -> $out"
  timeout -k 10 $secs "$@" > "$out" 2> "$out.err" || { echo "step $name failed ($?)"; tail -n 20 "$out" "$out.err"; exit 1; }
}
for s in "$@"; do
  case $s in
    trace)  # interior-point trace of the C5B copy 299 divergence, robust profile
      step trace1 300 gpurun_out/${tag}_trace_c5b_299.log python -u scripts/trace_solve.py --config C5B --scenes 2048 --solve 299 --lib-solve 299 --qp-profile robust ;;
    parity)  # full-size parity of every config, product (lean) and FULL launches (R06_PROFILE: hpipm | robust)
      step parity 1500 gpurun_out/${tag}_fullsize_parity_${R06_PROFILE:-hpipm}.jsonl python -u scripts/parity_full.py --configs ${R06_PARITY:-C2,C1,C3,C4,C5,C5B,JS,JD} --ws 2 --warm-first 0 --qp-profile ${R06_PROFILE:-hpipm} ;;
    qtests)  # the quick GPU tests: queue, small-size parity
      step qtests 900 gpurun_out/${tag}_qtests.log python -u -m pytest tests/test_queue.py tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread ;;
    ws)  # the restated warm start on every QP (qp_warm_first 1), full size
      step ws 900 gpurun_out/${tag}_ws_parity.jsonl python -u scripts/parity_full.py --configs C2,C4,C5 --ws 2 --warm-first 1 ;;
    sqp)
      step sqp 900 gpurun_out/${tag}_sqp_parity.jsonl python -u scripts/parity_full.py --configs C2,C1,C4 --ws 2 --warm-first 0 --solver-type SQP ;;
    tests)
      step tests 1500 gpurun_out/${tag}_gpu_tests.log python -u -m pytest tests -m gpu -v --timeout 900 --timeout-method thread ;;
    smoke)
      step smoke 300 gpurun_out/${tag}_smoke.log python -u -c "import __graft_entry__ as g; g.smoke()" ;;
    bench)
      for c in ${R06_BENCH:-C2}; do
        step bench_$c 600 gpurun_out/${tag}_bench_$(echo $c | tr A-Z a-z).json python -u bench.py --config $c --steps 20 --warmup 5
      done ;;
    latency)  # one Solver::solve() / one GuidanceConstraints::optimize through the drop-in's context
      step latency_js 300 gpurun_out/${tag}_latency_js.json python -u scripts/latency.py --config JS --guesses 5
      step latency_c2 300 gpurun_out/${tag}_latency_c2.json python -u scripts/latency.py --config C2 --guesses 8 ;;
    profile)  # rocprofv3 kernel trace + PMC passes of the bench workloads (R06_PROF="C2 C1 ...")
      for c in ${R06_PROF:-C2}; do
        lc=$(echo $c | tr A-Z a-z)
        step prof_$c 600 gpurun_out/${tag}_${lc}_prof.log bash scripts/profile_kernels.sh ${tag}_${lc} --config $c
      done ;;
    ab)  # A/B of kernel variants (scripts/ab_bench.py; R06_AB="variants:configs ...")
      for spec in ${R06_AB:-prod,fpair:C2,C1}; do
        v=${spec%%:*}; c=${spec##*:}
        step ab_${v//,/_}_${c//,/_} 1100 gpurun_out/${tag}_ab_${v//,/_}_${c//,/_}.jsonl python -u scripts/ab_bench.py --run $v --configs $c --reps 2
      done ;;
    bitcmp)  # bit comparison of library builds (R06_BITLIBS, R06_BITCFG, R06_PROFILE)
      step bitcmp 900 gpurun_out/${tag}_bitcmp_${R06_PROFILE:-hpipm}.jsonl python -u scripts/bitcmp.py --libs ${R06_BITLIBS:-oscar_mpc_planner_mr_modification_amd/build/ab/r05/libmpcg.so,prod} --configs ${R06_BITCFG:-C2,C1,C4,C5,C3,JS,JD} --profile ${R06_PROFILE:-hpipm} ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
echo all-done
