"""Exercise the compat stand-ins without a GPU (run by tests/test_compat.py through
``python -m networks_fenicsx_amd.compat``)."""

import math
import sys
from pathlib import Path

import numpy as np

import dolfinx
import dolfinx.io
import ufl
from dolfinx import fem
from mpi4py import MPI
from networks_fenicsx import NetworkMesh, network_generation
from networks_fenicsx.post_processing import extract_global_flux

out = Path(sys.argv[1])
G = network_generation.make_tree(2, 1, 3)
mesh = NetworkMesh(G, N=4)
x = ufl.SpatialCoordinate(mesh.mesh)
expr = 2.0 * x[1] - ufl.sin(x[0]) + 1
pts = np.array([[0.5, 1.0], [2.0, 3.0], [0.0, 0.0]])
assert np.allclose(expr.eval(pts), 2 * pts[1] - np.sin(pts[0]) + 1)

# integrals over the network: length, and x[1] (exact with 2-point Gauss)
length = fem.assemble_scalar(fem.form(fem.Constant(mesh.mesh, 1.0) * ufl.dx))
h = mesh.cell_lengths()
assert abs(length - h.sum()) < 1e-12
m = mesh.mesh
mid = 0.5 * (m.geometry.x[m.cells[:, 0]] + m.geometry.x[m.cells[:, 1]])
iy = fem.assemble_scalar(fem.form(x[1] * ufl.dx))
assert abs(iy - np.sum(h * mid[:, 1])) < 1e-12

# a synthetic solution list -> global flux (DG1) and its integral
from networks_fenicsx_amd.fem import Function, FunctionSpace  # noqa: E402

N = mesh.N
sol = []
for c, edges in enumerate(mesh.submeshes):
    V = FunctionSpace(mesh, "flux", "P", 1, False, edges.size * (N + 1), edges, c)
    f = Function(V, name=f"flux_{c}")
    f.x.array[:] = np.repeat(edges + 1.0, N + 1)  # q = e + 1 on edge e
    sol.append(f)
sol.append(Function(FunctionSpace(mesh, "pressure", "DG", 0, True, mesh.num_edges * N,
                                  np.arange(mesh.num_edges)), name="pressure"))
sol.append(Function(FunctionSpace(mesh, "multiplier", "DG", 0, True, 1), name="lm"))
gf = extract_global_flux(mesh, sol)
iq = fem.assemble_scalar(fem.form(gf * ufl.dx))
expect = sum((e + 1.0) * h.reshape(-1, N)[e].sum() for e in range(mesh.num_edges))
assert abs(iq - expect) < 1e-12
comm = gf.function_space.mesh.comm
assert comm.allreduce(np.max(gf.x.array), op=MPI.MAX) == mesh.num_edges
assert comm.allreduce(np.min(gf.x.array), op=MPI.MIN) == 1.0
assert comm.allreduce(2.5, op=MPI.SUM) == 2.5
assert MPI.COMM_WORLD.rank == 0 and MPI.COMM_WORLD.size == 1
with dolfinx.io.VTXWriter(comm, out / "global_flux.bp", [gf]) as vtx:
    vtx.write(0.0)
    vtx.write(1.0)
d = np.load(out / "global_flux.bp" / "step_0001.npz")
assert float(d["t"]) == 1.0 and np.array_equal(d["Global_Flux/values"], gf.x.array)
assert d["Global_Flux/cell_x"].shape == (mesh.num_edges * N, 2, 3)
with dolfinx.common.Timer("nxfx:shim:test"):
    math.sqrt(2.0)
assert dolfinx.common.timing("nxfx:shim:test")[0] == 1
print("shim surface OK")
