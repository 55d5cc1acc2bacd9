#!/usr/bin/env python3
"""Rehearsal of the driver's multi-GPU bench workload on ONE GPU.

``bench.py --gpus P`` weak-scales to ``make_tree(15 + log2 P)`` with N = 19 (P = 8: the
depth-17 tree, SURVEY's C4, 10.35 M DoF). RCCL refuses several ranks on one device, so this script runs
the same P per-rank handles -- same partition, halo plans, coarse step, kernels and MINRES
schedule -- through the in-process group transport (``RankGroup``) and checks the gathered
solution against the analytic resistor-network answer (oracle). Group solve
times are printed for information only: the group transport serialises all ranks on one
stream, so they are not multi-GPU timings.

    python scripts/group_rehearsal.py [--ranks 8] [--levels 15] [--N 19] [--solver direct]
"""

from __future__ import annotations

import argparse
import math
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO))
sys.path.insert(0, str(REPO / "tests"))

import numpy as np  # noqa: E402
import torch  # noqa: E402,F401  (HIP runtime before libnxhip.so)

import distributed_model as DM  # noqa: E402
from networks_fenicsx_amd import network_generation as ng  # noqa: E402
from networks_fenicsx_amd.group import RankGroup  # noqa: E402
from oracle import nx_oracle as O  # noqa: E402


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--ranks", type=int, default=8)
    ap.add_argument("--levels", type=int, default=15, help="tree generations at one rank")
    ap.add_argument("--N", type=int, default=19)
    ap.add_argument("--solver", choices=("direct", "minres"), default="direct")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--reverse", action="store_true",
                    help="with --exchange: time the ranks again in reverse order (is a rank's "
                         "time its own or its place in the sequence?)")
    ap.add_argument("--exchange", action="store_true",
                    help="also time every rank's one-launch exchange step alone "
                         "(nx_debug_xr_rehearse: its exchanges emulated)")
    args = ap.parse_args()
    levels = args.levels + int(round(math.log2(args.ranks)))
    t0 = time.perf_counter()
    G = ng.make_tree(levels, levels, levels)
    grp = RankGroup(G, args.N, args.ranks, color_strategy="smallest_last")
    print(f"make_tree({levels}) + {args.ranks} rank meshes: {time.perf_counter() - t0:.1f} s",
          flush=True)
    try:
        grp.compute_forms(p_bc_ex=lambda x: x[1])
        grp.set_direct(args.solver == "direct")
        grp.assemble()
        it, rr, conv = grp.solve(1e-12, 50000, 4)
        print(f"first solve: {it} iterations, relres {rr:.3e}, converged {conv}", flush=True)
        ts = []
        for _ in range(args.reps):
            t1 = time.perf_counter()
            grp.assemble()
            grp.solve(1e-12, 50000, 4)
            ts.append(time.perf_counter() - t1)
        mesh0 = grp.meshes[0]
        src, dst = mesh0.edges
        P = O.build_problem(mesh0.node_coordinates, src, dst, args.N)
        xa = O.resistor_network_solution(P, lambda x: x[1])
        perm, _ = O.build_permutation(P)
        xa = xa[perm]
        x = np.full(xa.size, np.nan)
        for a, xl in zip(grp.assemblers, grp.solutions()):
            x[DM.global_rows(a.local_problem, mesh0.num_edges, mesh0.bifurcation_index)] = xl
        err = float(np.linalg.norm(x - xa) / np.linalg.norm(xa))
        rows = [a.local_problem.n_own for a in grp.assemblers]
        print(f"DoF {xa.size}, rows per rank {min(rows)}..{max(rows)}, "
              f"group assemble+solve median {1e3 * sorted(ts)[len(ts) // 2]:.2f} ms "
              f"(serialised ranks), rel. error vs analytic {err:.3e}", flush=True)
        print(f"solver {grp.solver_used}", flush=True)
        want = (1, 2) if grp.solver_used == "direct" else (3,)
        ok = conv and it in want and err < 1e-10 and not np.isnan(x).any()
        if args.exchange and grp.solver_used == "direct":
            # every rank's exchange step alone (one launch per rank, as on its own GPU), its
            # exchanges emulated from this graph-path solve's sums; then its answer again
            ms = [a.handle.xr_rehearse(1e-12, 20) for a in grp.assemblers]
            if args.reverse:
                # (a rehearsal overwrites the graph path's summed partials it emulates its
                # exchanges from: solve on the graph path again first)
                grp.assemble()
                grp.solve(1e-12, 50000, 4)
                rev = [a.handle.xr_rehearse(1e-12, 20) for a in grp.assemblers[::-1]][::-1]
                print("exchange step per rank, timed in reverse order (us): "
                      + " ".join(f"{1e3 * m:.1f}" for m in rev), flush=True)
            x2 = np.full(xa.size, np.nan)
            for a in grp.assemblers:
                x2[DM.global_rows(a.local_problem, mesh0.num_edges,
                                  mesh0.bifurcation_index)] = a.handle.solution()
            err2 = float(np.linalg.norm(x2 - xa) / np.linalg.norm(xa))
            print("exchange step per rank (us): " + " ".join(f"{1e3 * m:.1f}" for m in ms),
                  flush=True)
            print(f"exchange step: slowest rank {1e3 * max(ms):.1f} us, rel. error vs analytic "
                  f"{err2:.3e}", flush=True)
            ok = ok and err2 < 1e-10
        print("REHEARSAL OK" if ok else "REHEARSAL FAILED", flush=True)
        return 0 if ok else 1
    finally:
        grp.close()


if __name__ == "__main__":
    sys.exit(main())
