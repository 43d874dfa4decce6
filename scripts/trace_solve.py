"""Side-by-side interior-point trace of one solve: the GPU kernel's diagnostic build
(-DMPCG_TRACE=<solve>, printf of rs / re / ri / mu per IPM iteration) and the oracle's
ORC_DEBUG trace of the same inputs (test infrastructure; GPU box).

    python scripts/trace_solve.py --config C5 --scene 1949 --solve 3 [--braking]

Builds build/trace/libmpcg_trace.so on the CPU side first:
    python scripts/trace_solve.py --build-only --solve 3
"""
import argparse
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "scripts")]
TRACE_DIR = os.path.join(ROOT, "oscar_mpc_planner_mr_modification_amd", "build", "trace")


def lib_path(solve=-1):
    return os.path.join(TRACE_DIR, "libmpcg_trace.so" if solve < 0 else f"libmpcg_trace{solve}.so")


def scene_inputs(cfg, scene, braking):
    from parity_full import inputs
    if cfg == "C5" and braking:
        from oscar_mpc_planner_mr_modification_amd.layouts import config_layout
        from oscar_mpc_planner_mr_modification_amd.scenario import make_shmpc_batch
        lay = config_layout(cfg)
        return lay, make_shmpc_batch(lay, 1, first_scene=scene, previous_plan_warm=False)
    return inputs(cfg, 1, first=scene)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C5")
    ap.add_argument("--scene", type=int, default=1949)
    ap.add_argument("--solve", type=int, default=3, help="solve index inside the scene's batch")
    ap.add_argument("--lib-solve", type=int, default=-1, help="the trace build's MPCG_TRACE (-1: every solve)")
    ap.add_argument("--braking", action="store_true")
    ap.add_argument("--build-only", action="store_true")
    ap.add_argument("--ws", type=int, default=0)
    args = ap.parse_args()
    if args.build_only:
        from oscar_mpc_planner_mr_modification_amd import _build
        os.makedirs(TRACE_DIR, exist_ok=True)
        print(_build.build_lib(force=True, extra_flags=[f"-DMPCG_TRACE={args.lib_solve}"], out=lib_path(args.lib_solve)))
        return
    lay, b = scene_inputs(args.config, args.scene, args.braking)
    np.savez(os.path.join(ROOT, "gpurun_out", "trace_inputs.npz"), params=b.params, warm=b.warm, xinit=b.xinit)
    # the GPU side in a child process (the trace library replaces libmpcg.so there)
    code = (f"import sys, numpy as np, torch; sys.path[:0]={[ROOT]!r}; "
            "from oscar_mpc_planner_mr_modification_amd import native; "
            "from oscar_mpc_planner_mr_modification_amd.layouts import config_layout; "
            f"lay = config_layout({args.config!r}); d = np.load({os.path.join(ROOT, 'gpurun_out', 'trace_inputs.npz')!r}); "
            "t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to('cuda:0'); "
            f"o = native.solve_batch_device(native.problem_from_layout(lay, qp_warm_start={args.ws}, qp_warm_first={int(args.ws == 2)}), "
            "t(d['params']), t(d['warm']), t(d['xinit'])); torch.cuda.synchronize(); "
            "print('GPU exit', o['exit'].cpu().numpy(), 'info', o['info'].cpu().numpy().tolist(), flush=True); "
            "np.save(" + repr(os.path.join(ROOT, "gpurun_out", "trace_gpu_xtraj.npy")) + ", o['xtraj'].cpu().numpy())")
    env = dict(os.environ, MPCG_LIB=lib_path(args.lib_solve))
    print("==== GPU trace", flush=True)
    subprocess.run([sys.executable, "-c", code], env=env, check=True, timeout=300)
    import oracle_py
    print("==== oracle trace", flush=True)
    i = args.solve
    os.environ["ORC_DEBUG"] = "1"
    r = oracle_py.Oracle(lay, qp_warm_start=args.ws, qp_warm_first=int(args.ws == 2)).solve_batch(b.params[i:i + 1], b.warm[i:i + 1],
                                                                 b.xinit[i:i + 1], nthreads=1)
    sys.stderr.flush()
    print("oracle exit", r["status"], "sqp", r["sqp_iter"], "qp", r["qp_iter"], "maxit", r["qp_maxiter"], flush=True)
    xg = np.load(os.path.join(ROOT, "gpurun_out", "trace_gpu_xtraj.npy"))
    print("max |dx| of solve", i, float(np.abs(xg[i] - r["xtraj"][0]).max()), flush=True)


if __name__ == "__main__":
    main()
