"""Rounding sensitivity of the exit decisions, CPU only (test infrastructure).

    python scripts/rounding_proxy.py [--configs C2,C4,C5]

Builds a second copy of the C oracle that differs from oracle/Makefile's only in
floating-point contraction (-march=x86-64-v3 -ffp-contract=fast: FMAs wherever the
compiler finds a*b+c, i.e. a different but equally legal rounding of the same
algorithm, as the GPU kernel's FMAs and reduction trees are), solves the bench's
full batch with both, and reports how many exit codes differ.  A config whose
oracle disagrees with itself under a legal change of rounding has exit decisions
that no second implementation can match bit for bit."""
import argparse
import json
import os
import subprocess
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "scripts")]


def main():
    import oracle_py
    from parity_full import DEFAULT_SCENES, inputs

    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="C2,C4,C5")
    ap.add_argument("--threads", type=int, default=8)
    args = ap.parse_args()
    tmp = tempfile.mkdtemp(prefix="orc_fma_")
    src = os.path.join(ROOT, "oracle", "mpcg_oracle.c")
    for cfg in args.configs.split(","):
        model = "unicycle_slack" if cfg == "C5" else "unicycle"
        alt = os.path.join(tmp, f"{model}.so")
        if not os.path.exists(alt):
            subprocess.run(["gcc", "-O2", "-std=c99", "-fPIC", "-fopenmp", "-march=x86-64-v3", "-ffp-contract=fast"] +
                           (["-DORC_SLACK_MODEL"] if cfg == "C5" else []) + ["-shared", "-o", alt, src, "-lm"],
                           check=True)
        lay, b = inputs(cfg, DEFAULT_SCENES[cfg])
        base_path = oracle_py.LIBS[model]
        ra = oracle_py.Oracle(lay).solve_batch(b.params, b.warm, b.xinit, nthreads=args.threads)
        oracle_py._libs.pop(model, None)
        oracle_py.LIBS[model] = alt
        try:
            rb = oracle_py.Oracle(lay).solve_batch(b.params, b.warm, b.xinit, nthreads=args.threads)
        finally:
            oracle_py._libs.pop(model, None)
            oracle_py.LIBS[model] = base_path
        same = ra["status"] == rb["status"]
        ok = same & (ra["status"] == 1)
        dis = np.flatnonzero(~same)
        print(json.dumps({
            "config": cfg, "solves": int(len(same)), "exit_agreement": float(same.mean()),
            "exit_disagreements": int(len(dis)),
            "max_abs_dx_success": float(np.abs(ra["xtraj"][ok] - rb["xtraj"][ok]).max()) if ok.any() else None,
            "disagreeing": [{"i": int(i), "exit": [int(ra["status"][i]), int(rb["status"][i])],
                             "sqp_iter": [int(ra["sqp_iter"][i]), int(rb["sqp_iter"][i])],
                             "qp_status": [int(ra["qp_status"][i]), int(rb["qp_status"][i])]} for i in dis[:20]],
        }), flush=True)


if __name__ == "__main__":
    main()
