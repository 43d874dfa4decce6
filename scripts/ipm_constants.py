"""CPU experiments behind DESIGN.md §2.2 (the interior point's constants and safeguards),
on the bench batches, with the oracle (test infrastructure):

1. the t / lambda floor qp_t_min against the rounding-decided SH-MPC copies: for each floor,
   the copies on which the two kernel-agnostic oracle builds (HPIPM forms, literal forms)
   part, and those on which the kernel-forms build ends like neither;
2. what the chosen floor does elsewhere (exit agreement and max |dx| against no floor);
3. the cold-start constants qp_mu0 / qp_thr0 (HPIPM's thr0 is 0.1);
4. the interior point's divergence test qp_mu_max in full SQP (rounding-decided solves) and in
   SQP-RTI (what it changes against round 3's 1e16).

    python scripts/ipm_constants.py [parts: 1 2 3 4] > profiles/r04_ipm_constants.txt
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "scripts")]

import oracle_py  # noqa: E402
from parity_full import inputs  # noqa: E402

NT = int(os.environ.get("OMP_NUM_THREADS", "8") or 8)


def run(lay, b, forms="hpipm", **opts):
    # these experiments chose the robust profile's constants (round 4)
    opts.setdefault("qp_profile", "robust")
    return oracle_py.Oracle(lay, forms=forms, **opts).solve_batch(b.params, b.warm, b.xinit, nthreads=NT)


def parted(a, c):
    B = len(a["status"])
    dx = np.abs(a["xtraj"] - c["xtraj"]).reshape(B, -1).max(1)
    return (a["status"] != c["status"]) | ((a["status"] == 1) & (dx > 1e-4))


def summary(r):
    return (f"success {np.mean(r['status'] == 1):.4f} rti/solve {r['sqp_iter'].mean():.2f} "
            f"ipm/solve {r['qp_iter'].mean():.2f} solves with a capped QP {int((r['qp_maxiter'] > 0).sum())}")


def main():
    parts = set(sys.argv[1:]) or {"1", "2", "3", "4"}
    if "1" in parts:
        part1()
    if "2" in parts:
        part2()
    if "3" in parts:
        part3()
    if "4" in parts:
        part4()


def part1():
    print("# 1. t / lambda floor vs rounding-decided SH-MPC copies (2048 scenes x 4 copies)")
    batches = {c: inputs(c, 2048) for c in ("C5", "C5B")}
    for tmin in (0.0, 1e-16, 1e-14, 1e-13, 1e-12, 1e-8):
        for cfg, (lay, b) in batches.items():
            R = {f: run(lay, b, f, qp_t_min=tmin) for f in ("hpipm", "literal", "kernel")}
            dec = parted(R["hpipm"], R["literal"])
            neither = parted(R["kernel"], R["hpipm"]) & parted(R["kernel"], R["literal"])
            print(f"{cfg} qp_t_min {tmin:g}: rounding-decided {int(dec.sum())} {np.flatnonzero(dec)[:12].tolist()} "
                  f"kernel-forms like neither {int(neither.sum())} | {summary(R['hpipm'])}", flush=True)


def part2():
    print("\n# 2. the floor 1e-12 against no floor elsewhere (HPIPM-forms build)")
    for cfg, S in (("C2", 1024), ("C1", 1024), ("C4", 512), ("C3", 1024), ("JS", 1024), ("JD", 1024)):
        lay, b = inputs(cfg, S)
        a, c = run(lay, b, qp_t_min=0.0), run(lay, b, qp_t_min=1e-12)
        same = a["status"] == c["status"]
        ok = same & (a["status"] == 1)
        dx = np.abs(a["xtraj"] - c["xtraj"]).reshape(len(same), -1)[ok].max() if ok.any() else 0.0
        print(f"{cfg} {len(same)} solves: exit agreement {same.mean():.6f} max |dx| {dx:.2e} "
              f"ipm/solve {a['qp_iter'].mean():.3f} -> {c['qp_iter'].mean():.3f}", flush=True)


def part3():
    print("\n# 3. cold-start constants (t = max(gap, thr0), lambda = mu0 / t, dz = 0)")
    for cfg, S in (("C2", 512), ("C5", 1024), ("C4", 512), ("C3", 1024)):
        lay, b = inputs(cfg, S)
        for mu0, thr0 in ((1.0, 1.0), (1.0, 0.1), (10.0, 0.1), (10.0, 1.0)):
            print(f"{cfg} mu0 {mu0:g} thr0 {thr0:g}: {summary(run(lay, b, qp_mu0=mu0, qp_thr0=thr0))}", flush=True)


def part4():
    print("\n# 4. divergence test qp_mu_max: full SQP rounding-decided solves (HPIPM vs literal forms), SQP-RTI changes")
    for cfg, S in (("C4", 2048), ("C2", 1024)):
        lay, b = inputs(cfg, S)
        for mmax in (1e16, 1e10, 1e8):
            a = run(lay, b, solver_type="SQP", qp_mu_max=mmax)
            c = run(lay, b, "literal", solver_type="SQP", qp_mu_max=mmax)
            dec = parted(a, c)
            print(f"{cfg} SQP qp_mu_max {mmax:g}: rounding-decided {int(dec.sum())} (exit-decided "
                  f"{int((a['status'] != c['status']).sum())}) | {summary(a)}", flush=True)
    for cfg, S in (("C2", 1024), ("C4", 2048), ("C5", 2048), ("C5B", 2048), ("C1", 1024)):
        lay, b = inputs(cfg, S)
        a, c = run(lay, b, qp_mu_max=1e16), run(lay, b, qp_mu_max=1e8)
        same = a["status"] == c["status"]
        ok = same & (a["status"] == 1)
        dx = np.abs(a["xtraj"] - c["xtraj"]).reshape(len(same), -1)[ok].max() if ok.any() else 0.0
        print(f"{cfg} SQP-RTI qp_mu_max 1e16 -> 1e8: exit changes {int((~same).sum())}, max |dx| of successful "
              f"{dx:.2e}, ipm/solve {a['qp_iter'].mean():.3f} -> {c['qp_iter'].mean():.3f}", flush=True)


if __name__ == "__main__":
    main()
