"""Side-by-side interior-point trace of one solve: the GPU kernel's diagnostic build
(-DMPCG_TRACE=<solve>, printf of rs / re / ri / mu per IPM iteration) and the oracle's
ORC_DEBUG trace of the same inputs (test infrastructure; GPU box).

    python scripts/trace_solve.py --config C5 --scene 1949 --solve 3 [--braking]
    python scripts/trace_solve.py --config C2 --scenes 1024 --solve 7414 --lib-solve 7414 \
        --solver-type SQP --variant full

--scenes S runs the bench batch of S scenes (the solve keeps its batch position, so the
launch is the one the parity record saw); without it only the scene `--scene` is solved and
`--solve` is the index inside that scene's batch.  --variant full launches the FULL kernel
variant (stats buffer: what scripts/parity_full.py's residual pass runs), lean the batched
path's.

Builds build/trace/libmpcg_trace<solve>.so (the config's instance family only) on the CPU side first:
    python scripts/trace_solve.py --build-only --config C5 --lib-solve 3
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


def scene_inputs(cfg, scene, braking, scenes=None):
    from parity_full import inputs
    if cfg == "C5" and braking:
        from oscar_mpc_planner_mr_modification_amd.layouts import config_layout
        from oscar_mpc_planner_mr_modification_amd.scenario import make_shmpc_batch
        lay = config_layout(cfg)
        return lay, make_shmpc_batch(lay, scenes or 1, first_scene=0 if scenes else scene, previous_plan_warm=False)
    if scenes:
        return inputs(cfg, scenes)
    return inputs(cfg, 1, first=scene)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C5")
    ap.add_argument("--scene", type=int, default=1949)
    ap.add_argument("--scenes", type=int, default=None, help="solve the bench batch of this many scenes")
    ap.add_argument("--solve", type=int, default=3, help="solve index inside the batch")
    ap.add_argument("--lib-solve", type=int, default=-1, help="the trace build's MPCG_TRACE (-1: every solve)")
    ap.add_argument("--braking", action="store_true")
    ap.add_argument("--build-only", action="store_true")
    ap.add_argument("--ws", type=int, default=2)
    ap.add_argument("--warm-first", type=int, default=0)
    ap.add_argument("--solver-type", default="SQP_RTI", choices=("SQP_RTI", "SQP"))
    ap.add_argument("--variant", default="lean", choices=("lean", "full"))
    ap.add_argument("--qp-profile", default="hpipm", choices=("hpipm", "robust"),
                    help="the interior point's profile (DESIGN.md §2.2) of both sides; the product default "
                         "(native_spec.DEFAULT_OPTIONS) is HPIPM's")
    ap.add_argument("--forms", default="hpipm", choices=("hpipm", "literal", "kernel"),
                    help="the oracle build to trace (oracle/mpcg_oracle.c \"Arithmetic forms\")")
    args = ap.parse_args()
    if args.build_only:
        from oscar_mpc_planner_mr_modification_amd import _build
        os.makedirs(TRACE_DIR, exist_ok=True)
        fam = {"C1": "tmpc20", "C2": "tmpc20", "C4": "tmpc30", "JS": "tmpc30", "JD": "tmpc30", "C5": "shmpc",
               "C5B": "shmpc", "C3": "bicycle"}[args.config]
        srcs = ["mpcg_kernels.hip", "mpcg_prepare.hip", f"mpcg_inst_{fam}.hip"]
        print(_build.build_lib(force=True, extra_flags=[f"-DMPCG_TRACE={args.lib_solve}"], out=lib_path(args.lib_solve),
                               sources=srcs))
        return
    lay, b = scene_inputs(args.config, args.scene, args.braking, args.scenes)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    # the batch's inputs for the GPU child process: outside gpurun_out (a bench batch is
    # hundreds of MB; gpurun_out travels back)
    import tempfile
    inp = os.path.join(tempfile.gettempdir(), f"mpcg_trace_inputs_{os.getpid()}.npz")
    np.savez(inp, params=b.params, warm=b.warm, xinit=b.xinit)
    opts = dict(qp_warm_start=args.ws, qp_warm_first=args.warm_first, solver_type=args.solver_type,
                qp_profile=args.qp_profile)
    # the GPU side in a child process (the trace library replaces libmpcg.so there)
    code = (f"import sys, numpy as np, torch; sys.path[:0]={[ROOT]!r}; "
            "from oscar_mpc_planner_mr_modification_amd import native; "
            "from oscar_mpc_planner_mr_modification_amd.layouts import config_layout; "
            f"lay = config_layout({'C5' if args.config == 'C5B' else args.config!r}); d = np.load({inp!r}); "
            "t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to('cuda:0'); "
            f"o = native.solve_batch_device(native.problem_from_layout(lay, **{opts!r}), "
            f"t(d['params']), t(d['warm']), t(d['xinit']), stats={args.variant == 'full'}); torch.cuda.synchronize(); "
            f"i = {args.solve}; "
            "print('GPU exit', int(o['exit'][i]), 'info', o['info'][i].cpu().numpy().tolist(), flush=True); "
            "np.save(" + repr(os.path.join(ROOT, "gpurun_out", "trace_gpu_xtraj.npy")) + ", o['xtraj'][i].cpu().numpy())")
    env = dict(os.environ, MPCG_LIB=lib_path(args.lib_solve))
    print("==== GPU trace", opts, args.variant, flush=True)
    subprocess.run([sys.executable, "-c", code], env=env, check=True, timeout=300)
    import oracle_py
    print("==== oracle trace", args.forms, flush=True)
    i = args.solve
    os.environ["ORC_DEBUG"] = "1"
    r = oracle_py.Oracle(lay, forms=args.forms, **opts).solve_batch(b.params[i:i + 1], b.warm[i:i + 1],
                                                                        b.xinit[i:i + 1], nthreads=1)
    del os.environ["ORC_DEBUG"]
    sys.stderr.flush()
    print("oracle exit", r["status"], "sqp", r["sqp_iter"], "qp", r["qp_iter"], "maxit", r["qp_maxiter"], flush=True)
    xg = np.load(os.path.join(ROOT, "gpurun_out", "trace_gpu_xtraj.npy"))
    print("max |dx| of solve", i, float(np.abs(xg - r["xtraj"][0]).max()), flush=True)


if __name__ == "__main__":
    main()
