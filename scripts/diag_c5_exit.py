"""Diagnose exit-code disagreements between the GPU solve and the oracle on
the C5 bench batch (same inputs: the GPU producer's)."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle_py  # noqa: E402
from oscar_mpc_planner_mr_modification_amd import native  # noqa: E402
from oscar_mpc_planner_mr_modification_amd.layouts import config_layout  # noqa: E402
from oscar_mpc_planner_mr_modification_amd.scenario import make_shmpc_scenes  # noqa: E402

S = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
lay = config_layout("C5")
dev = torch.device("cuda:0")
sc = make_shmpc_scenes(lay, S)
t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
pr = native.problem_from_layout(lay)
inp = native.prepare_scenario_device(pr, 4, t(sc.stage_params), t(sc.state), t(sc.samples), 0.65, 3.0,
                                     main_warm=t(sc.main_warm))
out = native.solve_batch_device(pr, inp["params"], inp["warm"], inp["xinit"])
torch.cuda.synchronize()
g = {k: v.cpu().numpy() for k, v in out.items()}
h = {k: v.cpu().numpy() for k, v in inp.items()}
o = oracle_py.Oracle(lay)
ref = o.solve_batch(h["params"], h["warm"], h["xinit"], nthreads=16)
bad = np.where(g["exit"] != ref["status"])[0]
print("mismatches", len(bad), "of", len(g["exit"]))
for i in bad[:20]:
    r = o.solve(h["params"][i], h["warm"][i], h["xinit"][i])
    print(i, "gpu exit", g["exit"][i], "info", g["info"][i].tolist(), "| oracle exit", r["exit"], "sqp", r["sqp_iter"],
          "qp", r["qp_iter"], "qp_status", r["qp_status"], "res_eq %.3e" % r["res_eq"],
          "max|dx| %.2e" % np.abs(g["xtraj"][i] - r["xtraj"]).max())
    for it in range(1, 11):
        o.pr.sqp_iters = it
        r1 = o.solve(h["params"][i], h["warm"][i], h["xinit"][i])
        print("   oracle iters", it, "exit", r1["exit"], "qp", r1["qp_iter"], "st", r1["qp_status"], "res_eq %.3e" % r1["res_eq"])
    o.pr.sqp_iters = 10
np.savez(os.path.join(ROOT, "gpurun_out", "c5_mismatch.npz"), idx=bad, params=h["params"][bad], warm=h["warm"][bad],
         xinit=h["xinit"][bad], gpu_exit=g["exit"][bad], gpu_info=g["info"][bad], gpu_x=g["xtraj"][bad])
