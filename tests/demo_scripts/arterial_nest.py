"""Arterial tree through the demo API surface: callable colouring strategy, explicit
element degrees, ``Solver(kind="nest")``, VTX output; checks flux conservation at every
bifurcation (sum of in-edge end fluxes = sum of out-edge start fluxes)."""

import sys
from pathlib import Path

import networkx as nx
import numpy as np

import dolfinx.io
from networks_fenicsx import HydraulicNetworkAssembler, NetworkMesh, Solver
from networks_fenicsx.network_generation import make_arterial_tree
from networks_fenicsx.post_processing import export_functions, extract_global_flux

out = Path(sys.argv[1])
G = make_arterial_tree(N=5, direction=np.array([0.1, 1, 0]))
net = NetworkMesh(G, N=40, color_strategy=nx.coloring.strategy_largest_first)
asm = HydraulicNetworkAssembler(net, flux_degree=1, pressure_degree=0)
asm.compute_forms(p_bc_ex=lambda x: x[1])
solver = Solver(asm, kind="nest")
solver.assemble()
sol = solver.solve()
gq = extract_global_flux(net, sol)
with dolfinx.io.VTXWriter(gq.function_space.mesh.comm, out / "global_flux.bp", [gq]) as vtx:
    vtx.write(0.0)
export_functions(functions=sol, outpath=out)
N = net.N
q = gq.x.array.reshape(-1, N, 2)
edges = gq.function_space.edges
q_start = dict(zip(edges.tolist(), q[:, 0, 0]))
q_end = dict(zip(edges.tolist(), q[:, -1, 1]))
src, dst = net.edges
for b in net.bifurcation_values:
    qin = sum(q_end[e] for e in np.flatnonzero(dst == b))
    qout = sum(q_start[e] for e in np.flatnonzero(src == b))
    assert abs(qin - qout) < 1e-9 * max(1.0, abs(qin)), (b, qin, qout)
assert solver.ksp.converged and solver.true_residual() < 1e-9
print("arterial nest OK")
