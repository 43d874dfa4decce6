"""Diagnostic of the split launch's work-queue variant on C1 (GPU box; test infrastructure).

    python scripts/split_queue_diag.py --lib build/ab/splitq/libmpcg.so [--iters 1,2,10]

For each SQP-RTI iteration count, the C1 bench batch through the production library and the given build
(one child process each); reports the solves that differ and, for each of the first few, whether its
outputs equal another solve's production outputs exactly (which solve's data it carries)."""
import argparse
import json
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def child(cfg, iters, out):
    import numpy as np
    import torch

    from oscar_mpc_planner_mr_modification_amd import native
    sys.path.insert(0, os.path.join(ROOT, "scripts"))
    from parity_full import DEFAULT_SCENES, inputs
    lay, b = inputs(cfg, DEFAULT_SCENES[cfg])
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to("cuda:0")  # noqa: E731
    o = native.solve_batch_device(native.problem_from_layout(lay, qp_profile="hpipm", sqp_iters=int(iters)),
                                  t(b.params), t(b.warm), t(b.xinit))
    np.savez(out, **{k: v.cpu().numpy() for k, v in o.items()})


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", default=None)
    ap.add_argument("--config", default="C1")
    ap.add_argument("--iters", default="1,2,10")
    ap.add_argument("--child", nargs=3, help=argparse.SUPPRESS)
    a = ap.parse_args()
    if a.child:
        child(*a.child)
        return
    import numpy as np
    prod = os.path.join(ROOT, "oscar_mpc_planner_mr_modification_amd", "libmpcg.so")
    tmp = tempfile.mkdtemp()
    for it in a.iters.split(","):
        outs = []
        for i, lib in enumerate([prod, os.path.join(ROOT, a.lib)]):
            f = os.path.join(tmp, f"{it}_{i}.npz")
            subprocess.run([sys.executable, os.path.abspath(__file__), "--child", a.config, it, f],
                           env=dict(os.environ, MPCG_LIB=lib, MPCG_ABI_ACCEPT_OLDER="8"), check=True)
            outs.append(np.load(f))
        ref, o = outs
        n = len(ref["exit"])
        xr, xo = ref["xtraj"].reshape(n, -1), o["xtraj"].reshape(n, -1)
        bad = ~(xr == xo).all(axis=1) | (ref["exit"] != o["exit"]) | ~(ref["info"].reshape(n, -1) == o["info"].reshape(n, -1)).all(axis=1)
        idx = np.flatnonzero(bad)
        rows = {xr[j].tobytes(): j for j in range(n)}
        carries = []
        for s in idx[:12]:
            carries.append({"solve": int(s), "equals_prod_solve": rows.get(xo[s].tobytes()),
                            "exit_prod": int(ref["exit"][s]), "exit_build": int(o["exit"][s]),
                            "info_prod": ref["info"].reshape(n, -1)[s].tolist(), "info_build": o["info"].reshape(n, -1)[s].tolist(),
                            "dx": float(np.abs(xr[s] - xo[s]).max())})
        print(json.dumps({"config": a.config, "sqp_iters": int(it), "lib": a.lib, "n_diff": int(bad.sum()),
                          "first_diff": int(idx[0]) if len(idx) else None, "diff_below_1024": int((idx < 1024).sum()),
                          "samples": carries}), flush=True)


if __name__ == "__main__":
    main()
