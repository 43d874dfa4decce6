"""Bit comparison of kernel builds (GPU box; test infrastructure): the bench batch of each config
through two or more libmpcg.so builds (MPCG_LIB, one child process each), outputs compared exactly.

    python scripts/bitcmp.py --libs prod,build/ab/x/libmpcg.so --configs C2,C4 [--profile hpipm]
"""
import argparse
import json
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def child(cfg, profile, out):
    import numpy as np
    import torch

    from oscar_mpc_planner_mr_modification_amd import native
    sys.path.insert(0, os.path.join(ROOT, "scripts"))
    from parity_full import DEFAULT_SCENES, inputs
    lay, b = inputs(cfg, DEFAULT_SCENES[cfg])
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to("cuda:0")  # noqa: E731
    o = native.solve_batch_device(native.problem_from_layout(lay, qp_profile=profile), t(b.params), t(b.warm),
                                  t(b.xinit))
    np.savez(out, **{k: v.cpu().numpy() for k, v in o.items()})


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--libs", default="prod")
    ap.add_argument("--configs", default="C2")
    ap.add_argument("--profile", default="hpipm")
    ap.add_argument("--child", nargs=3, help=argparse.SUPPRESS)
    a = ap.parse_args()
    if a.child:
        child(*a.child)
        return
    import numpy as np
    libs = [os.path.join(ROOT, "oscar_mpc_planner_mr_modification_amd", "libmpcg.so") if x == "prod" else
            os.path.join(ROOT, x) for x in a.libs.split(",")]
    tmp = tempfile.mkdtemp()
    for cfg in a.configs.split(","):
        outs = []
        for i, lib in enumerate(libs):
            f = os.path.join(tmp, f"{cfg}_{i}.npz")
            subprocess.run([sys.executable, os.path.abspath(__file__), "--child", cfg, a.profile, f],
                           env=dict(os.environ, MPCG_LIB=lib, MPCG_ABI_ACCEPT_OLDER="8"), check=True)
            outs.append(np.load(f))
        ref = outs[0]
        for lib, o in zip(libs[1:], outs[1:]):
            rec = {"config": cfg, "lib": os.path.relpath(lib, ROOT), "profile": a.profile}
            for k in ref.files:
                x, y = ref[k], o[k]
                same = np.array_equal(x, y, equal_nan=True) if x.dtype.kind == "f" else np.array_equal(x, y)
                rec[k] = "equal" if same else float(np.nanmax(np.abs(x.astype(np.float64) - y.astype(np.float64))))
            # the solves whose outputs differ at all (first few listed)
            bad = np.zeros(len(ref["exit"]), bool)
            for k in ref.files:
                x, y = ref[k].reshape(len(bad), -1), o[k].reshape(len(bad), -1)
                bad |= ~((x == y) | (np.isnan(x) & np.isnan(y)) if x.dtype.kind == "f" else (x == y)).all(axis=1)
            rec["n_diff_solves"] = int(bad.sum())
            rec["first_diff"] = [int(i) for i in np.flatnonzero(bad)[:8]]
            print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
