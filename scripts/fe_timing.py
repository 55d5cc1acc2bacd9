#!/usr/bin/env python3
"""General element degrees on the GPU: assembly + plain-MINRES timing (and the direct solve,
condensed for (k, 0)) at a mid-size tree (development / DESIGN numbers).
Usage: python scripts/fe_timing.py [levels N ["k,m;k,m..."] [direct]]  ("direct": the direct
solves only, for profiling passes)"""

from __future__ import annotations

import sys
import time
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO))

from networks_fenicsx_amd import HydraulicNetworkAssembler, NetworkMesh  # noqa: E402
from networks_fenicsx_amd import network_generation as ng  # noqa: E402
from oracle import nx_oracle_fe as OF  # noqa: E402


def main() -> int:
    levels = int(sys.argv[1]) if len(sys.argv) > 1 else 9
    N = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    mesh = NetworkMesh(ng.make_tree(levels, levels, levels), N=N, color_strategy="smallest_last")
    pbc = lambda x: x[1]  # noqa: E731
    pairs = [(1, 0), (2, 0), (2, 1), (3, 2)]
    if len(sys.argv) > 3:  # e.g. "1,0;2,0;3,0"
        pairs = [tuple(int(v) for v in p.split(",")) for p in sys.argv[3].split(";")]
    direct_only = len(sys.argv) > 4 and sys.argv[4] == "direct"
    for km in pairs:
        asm = HydraulicNetworkAssembler(mesh, flux_degree=km[0], pressure_degree=km[1])
        asm.compute_forms(p_bc_ex=pbc)
        h = asm.handle
        if direct_only:
            _direct(asm, h, km)
            asm.close()
            continue
        asm.set_preconditioner(False)
        h.assemble(True, True)
        h.solve(1e-12, 200000, 32)  # warm
        t0 = time.perf_counter()
        h.assemble(True, True)
        it, rr, conv = h.solve(1e-12, 200000, 32)
        h.sync()
        ms = 1e3 * (time.perf_counter() - t0)
        line = (f"k={km[0]} m={km[1]} rows={h.n_rows} nnz={h.nnz} plain MINRES it={it} "
                f"conv={conv} {ms:.2f} ms")
        if km[1] >= 1:
            F = OF.build_problem_fe(mesh.node_coordinates, *mesh.edges, N, *km, mesh.edge_colors)
            xa = OF.resistor_network_solution_fe(F, pbc)
            x = np.concatenate([fn.x.array for fn in _functions(asm)])
            line += f" err_vs_analytic={np.linalg.norm(x - xa) / np.linalg.norm(xa):.2e}"
        print(line, flush=True)
        if asm.fe_direct_available or km == (1, 0):  # the direct solve (condensed for k >= 2)
            _direct(asm, h, km)
        asm.close()
    return 0


def _direct(asm, h, km):
    if km == (1, 0):
        asm.set_preconditioner(True)
    asm.set_direct(True)
    ts = []
    for _ in range(6):
        t0 = time.perf_counter()
        h.assemble(True, True)
        it, rr, conv = h.solve(1e-12, 200000, 4)
        h.sync()
        ts.append(1e3 * (time.perf_counter() - t0))
    print(f"k={km[0]} m={km[1]} direct passes={it} relres={rr:.2e} conv={conv} "
          f"used={h.solver()[1]} min {min(ts[1:]):.3f} ms median "
          f"{float(np.median(ts[1:])):.3f} ms", flush=True)


def _functions(asm):
    from networks_fenicsx_amd.fem import Function

    fns = [Function(V) for V in asm.flux_spaces] + [Function(asm.pressure_space),
                                                     Function(asm.lm_space)]
    return asm.scatter_solution(asm.handle.solution(), fns)


if __name__ == "__main__":
    sys.exit(main())
