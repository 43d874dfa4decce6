import sys, numpy as np, torch, collections
sys.path.insert(0, '.'); sys.path.insert(0, 'oracle')
import producers_oracle as PO
from oscar_mpc_planner_mr_modification_amd import native
from oscar_mpc_planner_mr_modification_amd.layouts import config_layout
from oscar_mpc_planner_mr_modification_amd.synthetic import make_scenes, ROBOT_RADIUS, DECELERATION
lay = config_layout("C2"); sc = make_scenes(lay, 16, 8, seed=321)
sc.prev_elapsed[0] = 0.37; sc.prev_elapsed[-1] = 0.2 * 19
ref = PO.prepare(lay, sc, ROBOT_RADIUS, 0.05, DECELERATION)
pr = native.problem_from_layout(lay)
out = native.prepare_device(pr, native.scenes_to_device(sc, torch.device("cuda:0")), ROBOT_RADIUS, 0.05, DECELERATION)
torch.cuda.synchronize()
got = out["params"].cpu().numpy()
bad = np.argwhere(got != ref["params"])
inv = {v: k for k, v in lay.pmap.items()}
print(collections.Counter(inv[i].rsplit('_',1)[-1] if 'lin' in inv[i] else inv[i] for i in bad[:, 2]).most_common(10))
print(collections.Counter(int(b) for b in bad[:, 1]).most_common(5))
print(collections.Counter(int(b % 8) for b in bad[:, 0]).most_common(8))
i = bad[0]; print(i, inv[i[2]], got[tuple(i)], ref["params"][tuple(i)])
