"""Debug: preconditioned vs plain device MINRES, error vs rtol."""
import sys
sys.path.insert(0, ".")
sys.path.insert(0, "tests")
import numpy as np
from cases import CASES
from networks_fenicsx_amd import HydraulicNetworkAssembler, NetworkMesh
from networks_fenicsx_amd import network_generation as ng
from oracle import nx_oracle as O

def run(name, m, pbc):
    asm = HydraulicNetworkAssembler(m)
    asm.compute_forms(p_bc_ex=pbc)
    asm.assemble()
    h = asm.handle
    src, dst = m.edges
    P = O.build_problem(m.node_coordinates, src, dst, m.N, m.edge_colors)
    xa = O.resistor_network_solution(P, pbc)
    perm, _ = O.build_permutation(P)
    xr = xa[perm]
    for pc in (False, True):
        asm.set_preconditioner(pc)
        for rtol in (1e-8, 1e-10, 1e-12, 1e-13, 1e-14):
            it, rr, conv = h.solve(rtol, 20000, 32)
            x = h.solution()
            print(name, "pc" if pc else "--", f"rtol={rtol:.0e} it={it} conv={conv} relres={rr:.2e} err={np.linalg.norm(x-xr)/np.linalg.norm(xr):.2e} true={h.true_residual():.2e}", flush=True)

for case in sys.argv[1:]:
    if case.startswith("tree"):
        n = int(case[4:])
        run(case, NetworkMesh(ng.make_tree(n, n, n), N=15, color_strategy="smallest_last"), lambda x: x[1])
    else:
        make, N, strat, pbc = CASES[case]
        run(case, NetworkMesh(make(), N=N, color_strategy=strat), pbc)
