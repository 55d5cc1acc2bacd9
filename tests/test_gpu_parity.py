"""Parity of the HIP path against the CPU oracle (run on an MI355X: ``pytest -m gpu``).

Tolerances (stated per check):
* CSR pattern and rhs: bit-exact (integer / identical floating-point formulas, no FMA);
* CSR values: bit-exact (same geometry formula as the reference mesh generator);
* SpMV: <= 1e-15 relative per row against a numpy product (summation order may differ);
* solution: <= 1e-10 relative 2-norm against the oracle's direct solve (SuperLU standing
  in for PETSc/MUMPS) and against the analytic resistor-network solution.
"""

from __future__ import annotations

import numpy as np
import pytest

from cases import CASES, GOLDEN_CASES, edge_info_graph, graph_arrays  # noqa: F401
from networks_fenicsx_amd import HydraulicNetworkAssembler, NetworkMesh, Solver
from networks_fenicsx_amd import network_generation as ng
from networks_fenicsx_amd.post_processing import extract_global_flux, integrate_dg1
from oracle import nx_oracle as O

pytestmark = pytest.mark.gpu

SOL_TOL = 1e-10


def _build(case):
    make, N, strategy, pbc = CASES[case]
    G = make()
    mesh = NetworkMesh(G, N=N, color_strategy=strategy)
    asm = HydraulicNetworkAssembler(mesh)
    asm.compute_forms(p_bc_ex=pbc)
    src, dst = mesh.edges
    P = O.build_problem(mesh.node_coordinates, src, dst, N, mesh.edge_colors)
    A, b = O.assemble_reference(P, pbc)
    return mesh, asm, P, A, b, pbc


@pytest.mark.parametrize("case", sorted(CASES))
def test_csr_and_rhs_bit_exact(case):
    mesh, asm, P, A, b, _ = _build(case)
    asm.assemble()
    Ab, bb, perm, sign = O.to_build_layout(P, A, b)
    rp, col, val = asm.handle.csr()
    np.testing.assert_array_equal(rp, Ab.indptr)
    np.testing.assert_array_equal(col, Ab.indices)
    # bit-exact values: same reference geometry formula on both sides
    np.testing.assert_array_equal(val, Ab.data)
    np.testing.assert_array_equal(asm.handle.rhs(), bb)


@pytest.mark.parametrize("case", sorted(CASES))
def test_solution_matches_direct_and_analytic(case):
    mesh, asm, P, A, b, pbc = _build(case)
    solver = Solver(asm)
    solver.assemble()
    sol = solver.solve()
    assert solver.ksp.converged
    x_ref = O.solve_reference(A, b)
    _, _, perm, _ = O.to_build_layout(P, A, b)
    x = solver.solution_vector()
    err = np.linalg.norm(x - x_ref[perm]) / np.linalg.norm(x_ref)
    assert err <= SOL_TOL, err
    xa = O.resistor_network_solution(P, pbc)
    assert np.linalg.norm(x - xa[perm]) / np.linalg.norm(xa) <= SOL_TOL
    # function grouping: [flux per colour, pressure, multiplier] in the documented order
    assert len(sol) == mesh.num_edge_colors + 2
    for c, fn in enumerate(sol[:-2]):
        edges = np.flatnonzero(mesh.edge_colors == c)
        expect = np.concatenate([x_ref[P.flux_offset[e]:P.flux_offset[e] + mesh.N + 1]
                                 for e in edges]) if edges.size else np.zeros(0)
        np.testing.assert_allclose(fn.x.array, expect, rtol=0, atol=1e-10 * np.abs(x_ref).max())
    np.testing.assert_allclose(sol[-2].x.array, x_ref[P.p_offset:P.lm_offset], rtol=0,
                               atol=1e-10 * np.abs(x_ref).max())
    np.testing.assert_allclose(sol[-1].x.array, x_ref[P.lm_offset:], rtol=0,
                               atol=1e-10 * np.abs(x_ref).max())
    assert solver.true_residual() < 1e-9


@pytest.mark.parametrize("case", ["Y_N4", "depth6_N40", "edge_info_N10"])
def test_spmv_matches_numpy(case):
    mesh, asm, P, A, b, _ = _build(case)
    asm.assemble()
    Ab, _, _, _ = O.to_build_layout(P, A, b)
    rng = np.random.default_rng(0)
    x = rng.uniform(-1, 1, Ab.shape[1])
    y = asm.handle.spmv(x)
    ref = Ab @ x
    scale = np.abs(Ab) @ np.abs(x)
    assert np.all(np.abs(y - ref) <= 1e-15 * scale + 1e-300)


def test_reassemble_is_idempotent():
    mesh, asm, P, A, b, _ = _build("depth6_N40")
    asm.assemble()
    v1 = asm.handle.csr()[2].copy()
    r1 = asm.handle.rhs().copy()
    asm.assemble()
    np.testing.assert_array_equal(asm.handle.csr()[2], v1)
    np.testing.assert_array_equal(asm.handle.rhs(), r1)
    asm.assemble(A=None, b=None, assemble_lhs=False, assemble_rhs=True)
    np.testing.assert_array_equal(asm.handle.rhs(), r1)


@pytest.mark.parametrize("N", [2, 4, 8, 64, 65, 130])
def test_demo_tree_closed_form(N):
    """demo_tree.py (make_tree(2,1,1), p_bc = y): min q = 2-sqrt2, max q = 4-2 sqrt2,
    mean q = sqrt2/(1/2+sqrt2), lambda = -(2-sqrt2). N crosses the
    64-cell chunk boundary of the assembly kernel (64, 65, 130)."""
    mesh = NetworkMesh(ng.make_tree(n=2, H=1, W=1), N=N)
    asm = HydraulicNetworkAssembler(mesh)
    asm.compute_forms(p_bc_ex=lambda x: x[1])
    solver = Solver(asm, petsc_options={"ksp_type": "preonly", "pc_type": "lu",
                                        "pc_factor_mat_solver_type": "mumps"}, kind="mpi")
    solver.assemble()
    sol = solver.solve()
    g = extract_global_flux(mesh, sol)
    s2 = np.sqrt(2.0)
    tol = 1e-10  # the north-star FP tolerance, applied pointwise here
    assert abs(g.x.array.min() - (2 - s2)) < tol
    assert abs(g.x.array.max() - (4 - 2 * s2)) < tol
    integral, length = integrate_dg1(mesh, g)
    assert abs(integral / length - s2 / (0.5 + s2)) < tol
    assert abs(sol[-1].x.array[0] + (2 - s2)) < tol


@pytest.mark.parametrize("case", GOLDEN_CASES)
def test_golden_systems(systems, case):
    """Device system and solution against every committed oracle fixture
    (tests/golden/systems.npz): CSR bit-exact where stored, rhs bit-exact, solution
    <= 1e-10 against the fixture's direct solve and its analytic answer."""
    make, N, strategy, pbc = CASES[case]
    mesh = NetworkMesh(make(), N=N, color_strategy=strategy)
    asm = HydraulicNetworkAssembler(mesh)
    asm.compute_forms(p_bc_ex=pbc)
    solver = Solver(asm)
    solver.assemble()
    sol = solver.solve()
    if f"{case}/indptr" in systems:
        rp, col, val = asm.handle.csr()
        np.testing.assert_array_equal(rp, systems[f"{case}/indptr"])
        np.testing.assert_array_equal(col, systems[f"{case}/indices"])
        np.testing.assert_array_equal(val, systems[f"{case}/data"])
    np.testing.assert_array_equal(asm.handle.rhs(), systems[f"{case}/rhs_build"])
    x = solver.solution_vector()
    for key in ("x_build", "x_analytic_build"):
        ref = systems[f"{case}/{key}"]
        assert np.linalg.norm(x - ref) / np.linalg.norm(ref) <= SOL_TOL, key
    if f"{case}/x_ref_blocks" in systems:  # C2: the functions in the reference's order
        np.testing.assert_array_equal(mesh.edge_colors, systems[f"{case}/colors"])
        ref = systems[f"{case}/x_ref_blocks"]
        got = np.concatenate([f.x.array for f in sol])
        assert np.linalg.norm(got - ref) / np.linalg.norm(ref) <= SOL_TOL


def test_large_tree_properties():
    """depth-14 binary tree at BASELINE size (1,032,160 DoF): the solution must equal
    the analytic resistor network (size-independent property) and the assembled matrix
    must be exactly symmetric with the closed-form nnz count."""
    pos, src, dst = ng.tree_arrays(15, 15, 15)
    G = ng.make_tree(15, 15, 15)
    mesh = NetworkMesh(G, N=15, color_strategy=None)
    asm = HydraulicNetworkAssembler(mesh)
    asm.compute_forms(p_bc_ex=lambda x: x[1])
    solver = Solver(asm)
    solver.assemble()
    E, B, N = 32767, 16383, 15
    assert asm.handle.n_rows == E * (2 * N + 1) + B == 1032160
    assert asm.handle.nnz == E * (7 * N + 1) + 6 * B == 3571600
    M = solver.A.to_scipy()
    assert abs(M - M.T).max() == 0.0
    solver.solve()
    P = O.build_problem(mesh.node_coordinates, src, dst, N)
    xa = O.resistor_network_solution(P, lambda x: x[1])
    perm, _ = O.build_permutation(P)
    x = solver.solution_vector()
    err = np.linalg.norm(x - xa[perm]) / np.linalg.norm(xa)
    assert err <= SOL_TOL, err


@pytest.mark.parametrize("N", [300, 700, 1024])
def test_preconditioner_long_edges(N):
    """N > 256 cells per edge (demo_tree.py doubles N up to 1024): the (64, 8) / (64, 16)
    chain layouts keep the exact preconditioner, 3 iterations to the direct solution."""
    G = ng.make_tree(3, 1, 1)
    mesh = NetworkMesh(G, N=N)
    asm = HydraulicNetworkAssembler(mesh)
    asm.compute_forms(p_bc_ex=lambda x: x[1])
    assert asm.preconditioned
    solver = Solver(asm)
    solver.assemble()
    solver.solve()
    assert solver.ksp.getIterationNumber() <= 4
    src, dst = mesh.edges
    P = O.build_problem(mesh.node_coordinates, src, dst, N, mesh.edge_colors)
    A, b = O.assemble_reference(P, lambda x: x[1])
    _, _, perm, _ = O.to_build_layout(P, A, b)
    x_ref = O.solve_reference(A, b)
    x = solver.solution_vector()
    assert np.linalg.norm(x - x_ref[perm]) / np.linalg.norm(x_ref) <= SOL_TOL


def test_not_converged_raises():
    from networks_fenicsx_amd._lib import NxNotConverged

    make, N, strategy, pbc = CASES["depth6_N40"]
    mesh = NetworkMesh(make(), N=N, color_strategy=strategy)
    asm = HydraulicNetworkAssembler(mesh)
    asm.compute_forms(p_bc_ex=pbc)
    # the exact preconditioner needs 3 iterations: a cap of 2 cannot converge
    solver = Solver(asm, petsc_options={"ksp_type": "minres", "ksp_max_it": 2,
                                        "ksp_error_if_not_converged": True})
    solver.assemble()
    with pytest.raises(NxNotConverged):
        solver.solve()
    quiet = Solver(asm, petsc_options={"ksp_type": "minres", "ksp_max_it": 10,
                                       "ksp_error_if_not_converged": False, "pc_mass": "lumped"})
    quiet.solve()
    assert not quiet.ksp.converged and quiet.ksp.getIterationNumber() == 10


def test_per_edge_resistance_and_source():
    """R per edge (e.g. from the arterial radius) and f != 0: oracle parity."""
    make, N, strategy, pbc = CASES["arterial5_N40"]
    G = make()
    mesh = NetworkMesh(G, N=N, color_strategy=strategy)
    R = 1.0 / mesh.edge_radius ** 4
    asm = HydraulicNetworkAssembler(mesh)
    asm.compute_forms(p_bc_ex=pbc, f=0.3, R=R)
    solver = Solver(asm)
    solver.assemble()
    solver.solve()
    src, dst = mesh.edges
    P = O.build_problem(mesh.node_coordinates, src, dst, N, mesh.edge_colors)
    A, b = O.assemble_reference(P, pbc, f=0.3, R=R)
    Ab, bb, perm, _ = O.to_build_layout(P, A, b)
    np.testing.assert_array_equal(asm.handle.csr()[2], Ab.data)
    np.testing.assert_array_equal(asm.handle.rhs(), bb)
    x_ref = O.solve_reference(A, b)
    x = solver.solution_vector()
    assert np.linalg.norm(x - x_ref[perm]) / np.linalg.norm(x_ref) <= SOL_TOL


def test_per_edge_source():
    """f given per graph edge (nx_set_source): CSR / rhs bit-exact, solution vs direct."""
    make, N, strategy, pbc = CASES["depth6_N40"]
    mesh = NetworkMesh(make(), N=N, color_strategy=strategy)
    f = 0.1 + 0.05 * (np.arange(mesh.num_edges) % 7)
    asm = HydraulicNetworkAssembler(mesh)
    asm.compute_forms(p_bc_ex=pbc, f=f)
    solver = Solver(asm)
    solver.assemble()
    solver.solve()
    src, dst = mesh.edges
    P = O.build_problem(mesh.node_coordinates, src, dst, N, mesh.edge_colors)
    A, b = O.assemble_reference(P, pbc, f=f)
    Ab, bb, perm, _ = O.to_build_layout(P, A, b)
    np.testing.assert_array_equal(asm.handle.rhs(), bb)
    x_ref = O.solve_reference(A, b)
    x = solver.solution_vector()
    assert np.linalg.norm(x - x_ref[perm]) / np.linalg.norm(x_ref) <= SOL_TOL
    # back to a constant: the per-edge values are dropped
    asm.compute_forms(p_bc_ex=pbc, f=0.2)
    asm.assemble()
    A2, b2 = O.assemble_reference(P, pbc, f=0.2)
    np.testing.assert_array_equal(asm.handle.rhs(), O.to_build_layout(P, A2, b2)[1])


def test_profiling_counters():
    mesh, asm, P, A, b, _ = _build("depth6_N40")
    h = asm.handle
    h.set_profiling(True)
    h.reset_profile()
    asm.assemble()
    it, rr, conv = h.solve(1e-12, 50000, 32)
    prof = h.profile()
    h.set_profiling(False)
    assert conv and prof["spmv_count"] == it
    assert prof["spmv_ms"] > 0 and prof["asm_count"] == 1
    assert h.bench_spmv(5) > 0


@pytest.mark.parametrize("case", ["Y_N4", "depth6_N40"])
def test_convergence_chunk_invariance(case):
    """Iterations run in graph chunks; after convergence every later launch of a chunk
    must be a no-op. Results must not depend on the chunk length or on graph vs eager
    launches (regression: a stale double-buffered state used to resume iterating)."""
    mesh, asm, P, A, b, _ = _build(case)
    asm.assemble()
    h = asm.handle
    ref = None
    for eager, chunk in ((False, 2), (False, 8), (False, 32), (False, 1000), (True, 32)):
        h.set_profiling(eager)
        it, rr, conv = h.solve(1e-12, 5000, chunk)
        x = h.solution()
        if ref is None:
            ref = (it, x)
        assert conv and it == ref[0]
        np.testing.assert_array_equal(x, ref[1])
    h.set_profiling(False)


@pytest.mark.parametrize("case", ["depth6_N40", "arterial5_N40", "edge_info_N10", "tree6_2d_N70",
                                  "linear_alt_N3", "Y_N4"])
def test_preconditioned_matches_plain(case):
    """Tree Schur-complement preconditioner: same solution as plain MINRES and the
    direct solve, in far fewer iterations (cycle graph: spanning-forest variant)."""
    mesh, asm, P, A, b, pbc = _build(case)
    asm.assemble()
    h = asm.handle
    x_ref = O.solve_reference(A, b)
    _, _, perm, _ = O.to_build_layout(P, A, b)
    its = {}
    for pc in (False, True):
        asm.set_preconditioner(pc)
        it, rr, conv = h.solve(1e-12, 20000, 32)
        assert conv
        its[pc] = it
        x = h.solution()
        assert np.linalg.norm(x - x_ref[perm]) / np.linalg.norm(x_ref) <= SOL_TOL
    assert its[True] <= its[False]
    if mesh.num_edges == mesh.num_nodes - 1:  # trees: exact Schur complement -> 3 iterations
        assert its[True] <= 4, its


@pytest.mark.parametrize("case", ["depth6_N40", "arterial5_N40", "tree6_2d_N70", "Y_N4",
                                  "demo_tree_N1", "edge_info_N10"])
def test_exact_and_lumped_mass(case):
    """Consistent-mass (exact Schur complement, default) and lumped-mass preconditioners
    both reach the direct solution; the exact one in <= 4 iterations on trees, the lumped
    one in O(30)."""
    mesh, asm, P, A, b, pbc = _build(case)
    asm.assemble()
    h = asm.handle
    assert h.pc_exact()
    x_ref = O.solve_reference(A, b)
    _, _, perm, _ = O.to_build_layout(P, A, b)
    its = {}
    for exact in (True, False):
        h.set_pc_exact(exact)
        it, rr, conv = h.solve(1e-12, 20000, 4)
        assert conv
        its[exact] = it
        x = h.solution()
        assert np.linalg.norm(x - x_ref[perm]) / np.linalg.norm(x_ref) <= SOL_TOL, (exact, it)
        assert h.true_residual() <= 1e-9
    h.set_pc_exact(True)
    assert its[True] <= its[False], its
    if mesh.num_edges == mesh.num_nodes - 1:  # not for the cycle graph (grounded chain)
        assert its[True] <= 4, its


def test_solver_pc_option():
    mesh, asm, P, A, b, pbc = _build("depth6_N40")
    plain = Solver(asm, petsc_options={"pc_type": "none"})
    plain.assemble()
    plain.solve()
    it_plain = plain.ksp.getIterationNumber()
    pre = Solver(asm)  # reference default options (pc_type lu) -> tree preconditioner
    pre.solve()
    assert pre.ksp.getIterationNumber() < it_plain / 5


@pytest.mark.parametrize("path", ["lds", "global"])
@pytest.mark.parametrize("case", ["depth6_N40", "edge_info_N10", "demo_tree_N1"])
def test_preconditioner_kernel_paths(case, path, monkeypatch):
    """The LDS preconditioner kernels and the global-memory fallback give the same
    iterates (up to rounding) and both reach the direct solution."""
    if path == "global":
        monkeypatch.setenv("NXHIP_PC_GLOBAL", "1")
    mesh, asm, P, A, b, pbc = _build(case)
    asm.assemble()
    it, rr, conv = asm.handle.solve(1e-12, 20000, 32)
    assert conv and (it <= 4 or mesh.num_edges != mesh.num_nodes - 1)
    x_ref = O.solve_reference(A, b)
    _, _, perm, _ = O.to_build_layout(P, A, b)
    x = asm.handle.solution()
    assert np.linalg.norm(x - x_ref[perm]) / np.linalg.norm(x_ref) <= SOL_TOL


def test_cold_spmv_benchmark_runs():
    """The cold (cache-defeating) SpMV timing rotates over >= 2 copies and is no faster
    than a tiny fraction of the warm one (sanity, not a performance gate)."""
    mesh, asm, P, A, b, _ = _build("depth6_N40")
    asm.assemble()
    warm = asm.handle.bench_spmv(20)
    cold, k = asm.handle.bench_spmv_cold(20)
    assert k >= 2 and cold > 0 and warm > 0
