"""A/B timing of kernel variants (compile-time switches of csrc/mpcg_sqp.h).

    python scripts/ab_bench.py --build base: bsel:-DMPCG_BOUNDS_SEL=1      # CPU: build the variants
    python scripts/ab_bench.py --run base,bsel --configs C2,C3,C4 [--reps 2]  # GPU: bench each

Each variant is a full libmpcg.so under build/ab/<name>/ with the given extra flags; the
GPU side runs bench.py (no CPU leg) once per (rep, variant, config), alternating variants,
in child processes with MPCG_LIB set, and prints one JSON line each."""
import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
ABDIR = os.path.join(ROOT, "oscar_mpc_planner_mr_modification_amd", "build", "ab")


def lib(name):
    if name == "prod":  # the production library
        return os.path.join(ROOT, "oscar_mpc_planner_mr_modification_amd", "libmpcg.so")
    return os.path.join(ABDIR, name, "libmpcg.so")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--build", nargs="*", help="name:flag,flag ...")
    ap.add_argument("--run", default=None)
    ap.add_argument("--configs", default="C2")
    ap.add_argument("--reps", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    args = ap.parse_args()
    if args.build:
        from oscar_mpc_planner_mr_modification_amd import _build
        for spec in args.build:
            name, _, flags = spec.partition(":")
            fl = [f for f in flags.split(",") if f]
            os.makedirs(os.path.dirname(lib(name)), exist_ok=True)
            print(_build.build_lib(force=True, extra_flags=fl, out=lib(name)), fl, flush=True)
        return
    for rep in range(args.reps):
        for cfg in args.configs.split(","):
            for name in args.run.split(","):
                # (an earlier round's library, ABI 8: its mpcg_problem is a prefix of ABI 9's)
                env = dict(os.environ, MPCG_LIB=lib(name), MPCG_ABI_ACCEPT_OLDER="8")
                r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--config", cfg, "--no-cpu",
                                    "--steps", str(args.steps), "--warmup", "2"], env=env, capture_output=True,
                                   text=True, timeout=600)
                line = [x for x in r.stdout.splitlines() if x.startswith("{")]
                if r.returncode != 0 or not line:
                    print(json.dumps({"variant": name, "config": cfg, "error": r.stderr[-500:]}), flush=True)
                    sys.exit(1)
                d = json.loads(line[-1])
                print(json.dumps({"variant": name, "config": cfg, "rep": rep, "value": d["value"],
                                  "kernel_ms": d["roofline"]["kernel_ms"], "ms_per_step": d["ms_per_step"],
                                  "qp_iters": d["solver_stats"]["qp_iters_per_solve"],
                                  "qp_profile": d["solver_stats"].get("qp_profile"),
                                  "alt": d.get("qp_profile_alt")}), flush=True)


if __name__ == "__main__":
    main()
