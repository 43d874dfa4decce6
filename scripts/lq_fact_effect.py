"""What HPIPM's lq_fact 1 (BALANCE mode) would change on the bench batches -- CPU, oracle only.

    python scripts/lq_fact_effect.py [--configs C2,C1,C4,C5,C5B,JS] > profiles/r06d_lq_fact_effect.jsonl

The oracle's default build (HPIPM's forms, square-root Riccati, BLASFEO's pivot rule) on each bench batch,
without and with the LQ switch (orc_problem.qp_lq_fact: after a Cholesky factorisation whose predictor
direction has a linear KKT residual above 1e-5, the QP's remaining factorisations are LQ ones).  One JSON
line per config: QPs and solves that switched, exit-code changes, successful trajectories moved by more
than 1e-4, last-QP status counts.  Test infrastructure (imports the oracle); DESIGN.md §2.2."""
import argparse
import json
import os
import sys
from collections import Counter

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "scripts")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="C2,C1,C4,C5,C5B,JS")
    ap.add_argument("--threads", type=int, default=8)
    a = ap.parse_args()
    import oracle_py
    from parity_full import DEFAULT_SCENES, inputs
    for cfg in a.configs.split(","):
        lay, b = inputs(cfg, DEFAULT_SCENES[cfg])
        r = {lq: oracle_py.Oracle(lay, qp_warm_start=2, qp_warm_first=0, qp_lq_fact=lq).solve_batch(
            b.params, b.warm, b.xinit, nthreads=a.threads) for lq in (0, 1)}
        x, y = r[0], r[1]
        n = len(x["status"])
        ch = x["status"] != y["status"]
        dx = np.abs(x["xtraj"] - y["xtraj"]).reshape(n, -1).max(1)
        ok = (x["status"] == 1) & (y["status"] == 1)
        print(json.dumps({"config": cfg, "solves": n, "lq_qps": int(y["qp_lq"].sum()),
                          "solves_with_lq": int((y["qp_lq"] > 0).sum()), "exit_changes": int(ch.sum()),
                          "exit_transitions": {f"{s}->{t}": c for (s, t), c in
                                               Counter(zip(x["status"][ch].tolist(), y["status"][ch].tolist())).items()},
                          "success_frac": [float((x["status"] == 1).mean()), float((y["status"] == 1).mean())],
                          "success_dx_over_1e-4": int((ok & (dx > 1e-4)).sum()),
                          "max_abs_dx_success": float(dx[ok].max()) if ok.any() else None,
                          "qp_status_counts": [np.bincount(x["qp_status"], minlength=4).tolist(),
                                               np.bincount(y["qp_status"], minlength=4).tolist()]}), flush=True)


if __name__ == "__main__":
    main()
