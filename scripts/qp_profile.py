"""CPU record behind DESIGN.md §2.2 (round 5): the interior point's two profiles and what each of
HPIPM's restated features does, on the bench batches, with the oracle (test infrastructure):

* robust: round 4's constants (mu0 1, thr0 1, t_min 1e-12, mu_max 1e8, no primal move, no
  conditional corrector, no refinement, sigma clipped);
* hpipm: HPIPM's BALANCE mode as acados configures it (the default);
* hpipm without each feature (itref_corr_max 0, cond_pred_corr 0, init_move 0);
* hpipm with the literal-forms build (the rounding-decided solves of the profile).

Per run: success, RTI / IPM iterations per solve, solves with a capped QP, centring and refinement
solves per solve, and the solves on which each variant parts from hpipm (exit code, or successful
trajectories more than 1e-4 apart).

    python scripts/qp_profile.py [configs] > profiles/r05_qp_profile.txt
"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "scripts")]

import oracle_py  # noqa: E402
from parity_full import DEFAULT_SCENES, inputs  # noqa: E402

NT = int(os.environ.get("OMP_NUM_THREADS", "8") or 8)
VARIANTS = [("robust", dict(qp_profile="robust")), ("hpipm", {}), ("hpipm itref 0", dict(qp_itref_corr_max=0)),
            ("hpipm cond_pred_corr 0", dict(qp_cond_pred_corr=0)), ("hpipm init_move 0", dict(qp_init_move=0)),
            ("hpipm literal forms", dict(forms="literal"))]


def parted(a, c):
    B = len(a["status"])
    dx = np.abs(a["xtraj"] - c["xtraj"]).reshape(B, -1).max(1)
    return (a["status"] != c["status"]) | ((a["status"] == 1) & (c["status"] == 1) & (dx > 1e-4))


def main():
    cfgs = sys.argv[1].split(",") if len(sys.argv) > 1 else ["C2", "C1", "C4", "C5", "C5B", "C3", "JS", "JD"]
    for cfg in cfgs:
        lay, b = inputs(cfg, DEFAULT_SCENES[cfg])
        B = b.params.shape[0]
        print(f"## {cfg}: {B} solves (bench batch)", flush=True)
        R = {}
        for name, o in VARIANTS:
            t0 = time.time()
            r = oracle_py.Oracle(lay, **o).solve_batch(b.params, b.warm, b.xinit, nthreads=NT)
            R[name] = r
            line = (f"  {name:24s} success {np.mean(r['status'] == 1):.4f} rti/solve {r['sqp_iter'].mean():.2f} "
                    f"ipm/solve {r['qp_iter'].mean():.2f} capped-QP solves {int((r['qp_maxiter'] > 0).sum())} "
                    f"centring/solve {r['qp_center'].mean():.3f} refinement/solve {r['qp_itref'].mean():.3f}")
            if name != "hpipm" and "hpipm" in R:
                p = parted(R["hpipm"], r)
                line += f" | parts from hpipm on {int(p.sum())} {np.flatnonzero(p)[:8].tolist()}"
            print(line + f" ({time.time() - t0:.1f}s)", flush=True)
        p = parted(R["hpipm"], R["robust"])
        print(f"  robust vs hpipm: parted {int(p.sum())} of {B}", flush=True)


if __name__ == "__main__":
    main()
