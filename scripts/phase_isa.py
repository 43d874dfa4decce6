"""Per-phase instruction and fp64 attribution of one sqp_kernel instance (CPU only; VERDICT r03
item 7).  Compiles the instance family with -DMPCG_MARKERS (ISA phase markers, mpcg_sqp.h
STAMP_*), splits the lean kernel's instruction stream at the markers, counts per phase the
fp64 VALU instructions (and their flops: an fma counts 2, x 64 lanes = "issued"), all VALU,
LDS, scalar and memory instructions, and weights each phase by how often a solve executes it
(from the executed SQP and IPM iteration counts).  The useful (analytic) flops per phase come
from flopmodel.py.

    python scripts/phase_isa.py --config C2 [--sqp 9.73 --ipm 44.4] > profiles/r04_phase_isa_c2.txt
"""
import argparse
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
CSRC = os.path.join(ROOT, "oscar_mpc_planner_mr_modification_amd", "csrc")
FAMILY = {"C1": "tmpc20", "C2": "tmpc20", "C4": "tmpc30", "JS": "tmpc30", "JD": "tmpc30", "C5": "shmpc", "C3": "bicycle"}
CFG = {"C1": "20ELi4ELi4ELi0ELi5ELi0", "C2": "20ELi8ELi8ELi0ELi5ELi0", "C4": "30ELi12ELi12ELi0ELi5ELi0",
       "JS": "30ELi4ELi4ELi0ELi5ELi0", "JD": "30ELi5ELi5ELi0ELi5ELi0", "C5": "20ELi0ELi0ELi24ELi6ELi0",
       "C3": "30ELi0ELi0ELi12ELi6ELi1"}
# mpcg_sqp.h STAMP_END indices
EXTRA = os.environ.get("PHASE_ISA_FLAGS", "").split()
PHASES = {0: "linearisation", 1: "QP start", 2: "residuals (+ predictor barrier terms)", 3: "barrier terms + Newton gradient",
          4: "Riccati factorisation", 5: "vector chains + feedback", 7: "row steps, step length", 8: "iterate update"}


def classify(op):
    if op.startswith("v_") and "_f64" in op:
        return "f64"
    if op.startswith("v_"):
        return "valu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_", "buffer_", "flat_")):
        return "mem"
    if op.startswith("scratch_"):
        return "scratch"
    if op.startswith("s_"):
        return "salu"
    return "other"


def f64_flops(op):
    return 2 if ("fma" in op or "fmac" in op) else 1


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C2")
    ap.add_argument("--sqp", type=float, default=None, help="executed SQP-RTI iterations per solve")
    ap.add_argument("--ipm", type=float, default=None, help="executed IPM iterations per solve")
    args = ap.parse_args()
    fam = FAMILY[args.config]
    asm = f"/tmp/phase_isa_{fam}.s"
    subprocess.run(["hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", f"-I{os.path.join(ROOT, 'include')}",
                    f"-I{CSRC}", "-DMPCG_MARKERS", *EXTRA, "--cuda-device-only", "-S", os.path.join(CSRC, f"mpcg_inst_{fam}.hip"),
                    "-o", asm], check=True, stderr=subprocess.DEVNULL)
    lines = open(asm).read().split("\n")
    name = f"_ZN4mpcg10sqp_kernelINS_3CfgILi{CFG[args.config]}EEELb0E"
    start = next(i for i, l in enumerate(lines) if l.startswith(name) and ":" in l)
    end = next(i for i in range(start, len(lines)) if "s_endpgm" in lines[i])
    # regions: from "@@begin" to "@@end i"; laps do not split
    acc = {}
    cur = None
    for l in lines[start:end]:
        t = l.strip()
        if "@@begin" in t:
            cur = {"f64": 0, "flops": 0, "valu": 0, "lds": 0, "mem": 0, "scratch": 0, "salu": 0, "other": 0, "n": 0}
            continue
        m = re.search(r"@@end (\d+)", t)
        if m:
            if cur is not None:
                a = acc.setdefault(int(m.group(1)), {"regions": 0})
                a["regions"] += 1
                for k, v in cur.items():
                    a[k] = a.get(k, 0) + v
            cur = None
            continue
        if cur is None or not t or t.startswith((";", ".")) or t.endswith(":"):
            continue
        op = t.split()[0]
        c = classify(op)
        cur[c] += 1
        cur["n"] += 1
        if c == "f64":
            cur["flops"] += f64_flops(op)
    # executions per solve of each phase's code (every unrolled copy runs once per pass)
    from oscar_mpc_planner_mr_modification_amd import flopmodel
    from oscar_mpc_planner_mr_modification_amd.layouts import config_layout
    lay = config_layout(args.config)
    S = args.sqp if args.sqp is not None else 10.0
    Q = args.ipm if args.ipm is not None else 44.0
    # the residual pass runs once more per QP than the IPM iterations (the exit test); the
    # predictor / corrector loop (not unrolled: one copy of each phase's code) runs the chains
    # and the row steps twice per IPM iteration, the factorisation once (predictor) and the
    # barrier pass's work once (corrector; the predictor's is fused into the residuals)
    per = {0: S, 1: S, 2: Q + S, 3: Q, 4: Q, 5: 2 * Q, 7: 2 * Q, 8: Q}
    print(f"# {args.config} lean sqp_kernel: static instructions per phase (all unrolled copies of the "
          f"phase's code), weighted by {S} SQP-RTI and {Q} IPM iterations per solve")
    print(f"# {'phase':40s} {'copies':>6s} {'insts':>7s} {'f64':>6s} {'valu':>6s} {'lds':>5s} {'salu':>5s} {'mem+scr':>7s}"
          f" {'insts/solve':>12s} {'share':>6s} {'f64 lane-flops/solve':>21s}")
    tot_i = sum(a["n"] * per.get(p, 0) for p, a in acc.items())
    tot_f = 0
    rows = []
    for p in sorted(acc):
        a = acc[p]
        ips = a["n"] * per.get(p, 0)
        fl = a["flops"] * 64 * per.get(p, 0)
        tot_f += fl
        rows.append((p, ips, fl))
        print(f"  {p} {PHASES.get(p, '?'):38s} {a['regions']:6d} {a['n']:7d} {a['f64']:6d} {a['valu']:6d} {a['lds']:5d} "
              f"{a['salu']:5d} {a['mem']:4d}+{a['scratch']:<4d} {ips:12.0f} {ips / tot_i:6.1%} {fl:21.3e}")
    lin = flopmodel.linearisation_ops(lay) * S
    parts = {k: v * Q for k, v in flopmodel.ipm_iteration_ops_by_part(lay).items()}
    ipm = sum(parts.values())
    print(f"# total issued instructions per solve {tot_i:.4g}; issued fp64 lane-flops per solve {tot_f:.4g} "
          f"(x 64 lanes, masked lanes included)")
    print(f"# analytic (flopmodel.py): linearisation {lin:.4g} + interior point {ipm:.4g} = {lin + ipm:.4g} flop per solve")
    issued = {p: fl for p, _, fl in rows}
    insts = {p: i for p, i, _ in rows}
    groups = [("linearisation", [0], lin), ("Riccati factorisation", [4], parts["factorisation"]),
              ("rest of the interior point", [1, 2, 3, 5, 7, 8],
               parts["residuals"] + parts["barrier"] + parts["newton_solves"] + parts["update"])]
    print(f"# {'group':28s} {'issued lane-flops':>18s} {'analytic':>10s} {'issued/analytic':>16s} {'share of insts':>15s}")
    for g, ps, an in groups:
        fi = sum(issued.get(p, 0) for p in ps)
        ii = sum(insts.get(p, 0) for p in ps)
        print(f"  {g:28s} {fi:18.4g} {an:10.4g} {fi / an:16.2f} {ii / tot_i:15.1%}")
    print(f"  {'total':28s} {tot_f:18.4g} {lin + ipm:10.4g} {tot_f / (lin + ipm):16.2f}")


if __name__ == "__main__":
    main()
