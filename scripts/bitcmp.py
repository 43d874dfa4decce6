"""Bit-for-bit comparison of two kernel builds on the bench batch of a config (GPU).

    python scripts/bitcmp.py dump <out.npz> --config C2     (MPCG_LIB selects the build)
    python scripts/bitcmp.py cmp <a.npz> <b.npz>

A transformation that keeps every floating-point operation of the solve (same operations, other
lanes or another order of independent work) must give identical outputs."""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def dump(path, config, scenes):
    import torch

    from oscar_mpc_planner_mr_modification_amd import native

    sys.path.insert(0, os.path.join(ROOT, "scripts"))
    from parity_full import inputs

    lay, b = inputs(config, scenes)
    dev = torch.device("cuda:0")
    params, warm, xinit = b.params, b.warm, b.xinit
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    out = native.solve_batch_device(native.problem_from_layout(lay), t(params), t(warm), t(xinit))
    torch.cuda.synchronize()
    np.savez(path, **{k: v.cpu().numpy() for k, v in out.items()})
    print(path, {k: v.shape for k, v in out.items()})


def cmp(a, b):
    A, B = np.load(a), np.load(b)
    bad = 0
    for k in A.files:
        x, y = A[k], B[k]
        same = x.shape == y.shape and np.array_equal(x.view(np.uint8), y.view(np.uint8))
        if not same:
            bad += 1
            d = np.abs(x.astype(np.float64) - y.astype(np.float64))
            print(k, "DIFFERS: max abs", float(np.nanmax(d)), "entries", int((x != y).sum()))
    print("bit-identical" if bad == 0 else f"{bad} arrays differ")
    return bad


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("mode", choices=["dump", "cmp"])
    ap.add_argument("files", nargs="+")
    ap.add_argument("--config", default="C2")
    ap.add_argument("--scenes", type=int, default=512)
    a = ap.parse_args()
    if a.mode == "dump":
        dump(a.files[0], a.config, a.scenes)
    else:
        sys.exit(1 if cmp(*a.files) else 0)
