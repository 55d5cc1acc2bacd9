"""Debug: device MINRES residual estimate after m iterations vs the numpy model."""
import sys
sys.path.insert(0, ".")
sys.path.insert(0, "tests")
import numpy as np
from cases import CASES
from networks_fenicsx_amd import HydraulicNetworkAssembler, NetworkMesh
from oracle import nx_oracle as O

make, N, strat, pbc = CASES[sys.argv[1] if len(sys.argv) > 1 else "Y_N4"]
m = NetworkMesh(make(), N=N, color_strategy=strat)
asm = HydraulicNetworkAssembler(m)
asm.compute_forms(p_bc_ex=pbc)
asm.assemble()
h = asm.handle
src, dst = m.edges
P = O.build_problem(m.node_coordinates, src, dst, N, m.edge_colors)
A, b = O.assemble_reference(P, pbc)
Ab, bb, perm, _ = O.to_build_layout(P, A, b)
import scipy.sparse.linalg as spla
for maxit in range(1, 21):
    it, rr, conv = h.solve(1e-14, maxit, 2)
    x = h.solution()
    xs, _ = spla.minres(Ab, bb, rtol=0, maxiter=maxit)
    print(maxit, it, f"{rr:.6e}", f"gpu|x|={np.linalg.norm(x):.6e} scipy|x|={np.linalg.norm(xs):.6e} diff={np.linalg.norm(x-xs)/np.linalg.norm(xs):.2e}")
