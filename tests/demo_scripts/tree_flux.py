"""Convergence-study style run on make_tree(2, 1, 1) through the demo API surface
(mpi4py ops, dolfinx forms / VTXWriter, networks_fenicsx classes), checked against the
closed form: min q = 2 - sqrt(2), max q = 4 - 2 sqrt(2),
mean q = sqrt(2) / (1/2 + sqrt(2)). Run via ``python -m networks_fenicsx_amd.compat``."""

import math
import sys
from pathlib import Path

import numpy as np

import dolfinx
import ufl
from dolfinx import fem
from mpi4py import MPI
from networks_fenicsx import HydraulicNetworkAssembler, NetworkMesh, Solver, network_generation
from networks_fenicsx.post_processing import export_functions, extract_global_flux

out = Path(sys.argv[1])
graph = network_generation.make_tree(n=2, H=1, W=1)
expect = (2 - math.sqrt(2), 4 - 2 * math.sqrt(2), math.sqrt(2) / (0.5 + math.sqrt(2)))
for N in (2, 4, 8, 64, 512, 1024):  # demo_tree.py doubles N up to 1024
    net = NetworkMesh(graph, N=N)
    asm = HydraulicNetworkAssembler(net)
    asm.compute_forms(p_bc_ex=lambda x: x[1])
    solver = Solver(asm, petsc_options={"ksp_type": "preonly", "pc_type": "lu",
                                        "pc_factor_mat_solver_type": "mumps"}, kind="mpi")
    solver.assemble()
    sol = solver.solve()
    gq = extract_global_flux(net, sol)
    export_functions(sol, outpath=out / f"N_{N}")
    with dolfinx.io.VTXWriter(gq.function_space.mesh.comm, out / f"N_{N}" / "q.bp", [gq]) as w:
        w.write(0.0)
    c = net.comm
    qmax = c.allreduce(np.max(gq.x.array), op=MPI.MAX)
    qmin = c.allreduce(np.min(gq.x.array), op=MPI.MIN)
    total = c.allreduce(fem.assemble_scalar(fem.form(gq * ufl.dx)), op=MPI.SUM)
    length = c.allreduce(fem.assemble_scalar(fem.form(fem.Constant(net.mesh, 1.0) * ufl.dx)),
                         op=MPI.SUM)
    got = (qmin, qmax, total / length)
    for g, e in zip(got, expect):
        assert abs(g - e) < 1e-10, (N, got, expect)
    assert (out / f"N_{N}" / "q.bp" / "step_0000.npz").exists()
print("tree flux OK")
