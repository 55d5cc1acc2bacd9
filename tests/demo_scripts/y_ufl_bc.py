"""Pressure boundary data given as a ufl expression of ``SpatialCoordinate`` (the Y and
double-Y demos) must give the same solution as the equivalent Python callable."""

import numpy as np

import ufl
from networks_fenicsx import HydraulicNetworkAssembler, NetworkMesh, Solver, network_generation


def run(G, N, bc):
    net = NetworkMesh(G, N=N)
    asm = HydraulicNetworkAssembler(net)
    asm.compute_forms(p_bc_ex=bc(net))
    s = Solver(asm)
    s.assemble()
    return np.concatenate([f.x.array for f in s.solve()])


for G, N, i in ((network_generation.make_tree(2, 1, 3), 4, 1),
                (network_generation.make_tree(2, 3.1, 7.3), 5, 0)):
    a = run(G, N, lambda net: ufl.SpatialCoordinate(net.mesh)[i])
    b = run(G, N, lambda net: (lambda x: x[i]))
    c = run(G, N, lambda net: 2 * ufl.SpatialCoordinate(net.mesh)[i] - 1.0)
    d = run(G, N, lambda net: (lambda x: 2 * x[i] - 1.0))
    assert np.array_equal(a, b) and np.array_equal(c, d)
    assert not np.array_equal(a, c)
print("ufl bc OK")
