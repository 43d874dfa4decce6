"""What a linearisation kernel of its own would cost in launch tails -- CPU, oracle only.

    python scripts/split_tail_model.py --configs C4,JD,C3 > profiles/r06m_split_tail_model.jsonl

The IPM iterations of every QP of every solve of the bench batch come from the oracle (the default build; the GPU
follows it solve for solve): the total after k RTI iterations minus the total after k - 1 (an RTI loop's first k
iterations do not depend on how many follow).  Per solve and RTI iteration the work is L + q (q IPM iterations; L
the linearisation in IPM-iteration units, from the phase stamps).  The batch is list-scheduled in index order onto
the resident slots (four solves per CU x 256 CUs), as the hardware deals workgroups:
  * fused (today's one-kernel SQP loop): one job per solve, sum over its RTI iterations;
  * split: per RTI iteration a linearisation launch (jobs L) and an interior-point launch (jobs q) over the solves
    still running, each launch ending on its last job.
Prints the two makespans in IPM-iteration units and their ratio: the tail the split adds, before any gain from
its register allocation.  Test infrastructure (imports the oracle)."""
import argparse
import heapq
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "scripts")]

# linearisation cost of one RTI iteration in units of one IPM iteration (phase stamps, DESIGN.md §3.8 / §3.3:
# C4 7.4 % of cycles at 9.1 RTI and 61.6 IPM iterations per solve; C3 18 % at 10 / 54; JD as JS)
LIN_UNITS = {"C4": 0.074 * 61.6 / 9.14 / (1 - 0.074), "JD": 0.10 * 58.0 / 9.77 / 0.90,
             "JS": 0.10 * 56.6 / 9.85 / 0.90, "C3": 0.18 * 53.9 / 10.0 / 0.82, "C2": 0.114 * 53.7 / 9.73 / 0.886}


def list_schedule(jobs, slots):
    """makespan of the jobs dealt in order to the first free of `slots` machines"""
    if len(jobs) == 0:
        return 0.0
    h = [0.0] * min(slots, len(jobs))
    heapq.heapify(h)
    for d in jobs:
        t = heapq.heappop(h)
        heapq.heappush(h, t + d)
    return max(h)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="C4,JD,C3")
    ap.add_argument("--slots", type=int, default=1024)
    ap.add_argument("--threads", type=int, default=8)
    a = ap.parse_args()
    import oracle_py
    from parity_full import DEFAULT_SCENES, inputs
    for cfg in a.configs.split(","):
        lay, b = inputs(cfg, DEFAULT_SCENES[cfg])
        iters = lay.sqp_iters
        tot = [np.zeros(len(b.params), np.int64)]
        done = []
        for k in range(1, iters + 1):
            r = oracle_py.Oracle(lay, sqp_iters=k).solve_batch(b.params, b.warm, b.xinit, nthreads=a.threads)
            tot.append(r["qp_iter"].astype(np.int64))
            done.append(r["sqp_iter"] >= k)  # the solve ran its k-th RTI iteration
        q = np.stack([tot[k] - tot[k - 1] for k in range(1, iters + 1)], 1)  # [solve][RTI iteration]
        act = np.stack(done, 1)
        L = LIN_UNITS[cfg]
        fused = list_schedule(((L + q) * act).sum(1), a.slots)
        split = sum(list_schedule(np.full(int(act[:, k].sum()), L), a.slots) +
                    list_schedule(q[act[:, k], k], a.slots) for k in range(iters))
        print(json.dumps({"config": cfg, "solves": int(len(q)), "slots": a.slots, "lin_units": round(L, 3),
                          "ipm_per_qp_mean": float(q[act].mean()), "ipm_per_qp_max": int(q[act].max()),
                          "ipm_per_qp_p99": float(np.percentile(q[act], 99)),
                          "makespan_fused": round(float(fused), 1), "makespan_split": round(float(split), 1),
                          "split_over_fused": round(float(split / fused), 3)}), flush=True)


if __name__ == "__main__":
    main()
