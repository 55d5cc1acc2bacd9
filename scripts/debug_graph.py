"""Debug: chunked-graph vs eager MINRES on the same handle."""
import sys
sys.path.insert(0, ".")
sys.path.insert(0, "tests")
import numpy as np
from cases import CASES
from networks_fenicsx_amd import HydraulicNetworkAssembler, NetworkMesh
from oracle import nx_oracle as O

for case in sys.argv[1:]:
    make, N, strat, pbc = CASES[case]
    m = NetworkMesh(make(), N=N, color_strategy=strat)
    asm = HydraulicNetworkAssembler(m)
    asm.compute_forms(p_bc_ex=pbc)
    asm.assemble()
    h = asm.handle
    src, dst = m.edges
    P = O.build_problem(m.node_coordinates, src, dst, N, m.edge_colors)
    A, b = O.assemble_reference(P, pbc)
    Ab, bb, perm, _ = O.to_build_layout(P, A, b)
    xr = O.solve_reference(A, b)[perm]
    for mode, chunk in (("graph", 2), ("graph", 8), ("graph", 32), ("eager", 32)):
        h.set_profiling(mode == "eager")
        it, rr, conv = h.solve(1e-12, 5000, chunk)
        x = h.solution()
        print(case, mode, chunk, it, f"{rr:.2e}", f"err={np.linalg.norm(x-xr)/np.linalg.norm(xr):.2e}", flush=True)
    h.set_profiling(False)
