"""General element degrees on the GPU: ``k_assemble_fe`` + plain MINRES against the oracle.

Tolerances:
* CSR pattern: identical to the host layout; values and rhs bit-exact against the host
  evaluation of the same term tables (same cell-length formula, same summation order);
* values against the oracle's forms: <= 1e-14 relative (element tensors integrated two
  ways: exact rationals vs Gauss-Legendre);
* solution: <= 1e-10 relative 2-norm against the oracle's direct solve and, for
  continuous pressure (m >= 1), against the analytic resistor-network answer.
"""

from __future__ import annotations

import numpy as np
import pytest

from cases import CASES
from networks_fenicsx_amd import HydraulicNetworkAssembler, NetworkMesh, Solver
from networks_fenicsx_amd.layout_fe import evaluate_terms
from networks_fenicsx_amd.post_processing import extract_global_flux, integrate_dg1
from oracle import nx_oracle as O
from oracle import nx_oracle_fe as OF

pytestmark = pytest.mark.gpu

SOL_TOL = 1e-10
PAIRS = [(2, 0), (3, 0), (2, 1), (3, 1), (3, 2)]


def _setup(case, km, f=None, R=None):
    make, N, strategy, pbc = CASES[case]
    mesh = NetworkMesh(make(), N=N, color_strategy=strategy)
    asm = HydraulicNetworkAssembler(mesh, flux_degree=km[0], pressure_degree=km[1])
    asm.compute_forms(p_bc_ex=pbc, f=f, R=R)
    src, dst = mesh.edges
    F = OF.build_problem_fe(mesh.node_coordinates, src, dst, N, *km, mesh.edge_colors)
    A, b = OF.assemble_reference_fe(F, pbc, f=0.0 if f is None else f,
                                    R=1.0 if R is None else R)
    return mesh, asm, F, A, b, pbc


def _edge_bc(F, pbc):
    pb = O._nodal(pbc, F.base.pos3)
    src, dst = F.base.src, F.base.dst
    leaf = np.zeros(pb.size, dtype=bool)
    leaf[F.base.leaf_in] = True
    root = np.zeros(pb.size, dtype=bool)
    root[F.base.root_out] = True
    bc = np.zeros((src.size, 2))
    bc[:, 0] = np.where(root[src], -pb[src], 0.0)
    bc[:, 1] = np.where(leaf[dst], pb[dst], 0.0)
    return bc


@pytest.mark.parametrize("case", ["Y_N4", "edge_info_N10", "depth6_N40"])
@pytest.mark.parametrize("km", PAIRS)
@pytest.mark.parametrize("struct", ["1", "0"])  # (k, 0): the edge templates (default) / the gather tables
def test_fe_csr_and_rhs(case, km, struct, monkeypatch):
    monkeypatch.setenv("NXHIP_FE_STRUCT", struct)
    R = 1.0 + np.arange(len(CASES[case][0]().edges())) % 3
    mesh, asm, F, A, b, pbc = _setup(case, km, f=0.7, R=R)
    asm.assemble()
    lay = asm.fe_layout
    rp, col, val = asm.handle.csr()
    np.testing.assert_array_equal(rp, lay.rowptr)
    np.testing.assert_array_equal(col, lay.col)
    _, h = O.cell_geometry(F.base)
    hv, hr = evaluate_terms(lay, R, 0.7, _edge_bc(F, pbc), h)
    np.testing.assert_array_equal(val, hv)  # bit-exact: same terms, same order
    np.testing.assert_array_equal(asm.handle.rhs(), hr)
    # the edge templates are built for every pair on these graphs (so "1" ran them)
    k, m = km
    N = CASES[case][1]
    assert asm.handle.fe_templates()[1] == k * N + 1 + (N if m == 0 else m * N - 1)
    assert 1 <= asm.handle.fe_templates()[0] <= 8


@pytest.mark.parametrize("case", ["Y_N4", "double_Y_N5", "edge_info_N10", "depth6_N40",
                                  "arterial5_N40"])
@pytest.mark.parametrize("km", PAIRS)
def test_fe_solution(case, km):
    mesh, asm, F, A, b, pbc = _setup(case, km)
    solver = Solver(asm)
    solver.assemble()
    sol = solver.solve()
    assert solver.ksp.converged and not asm.preconditioned
    x_ref = O.solve_reference(A, b)
    # functions in the oracle's block order: flux per colour, pressure, multipliers
    got = np.concatenate([fn.x.array for fn in sol])
    assert np.linalg.norm(got - x_ref) / np.linalg.norm(x_ref) <= SOL_TOL
    if km[1] >= 1:
        xa = OF.resistor_network_solution_fe(F, pbc)
        assert np.linalg.norm(got - xa) / np.linalg.norm(xa) <= SOL_TOL
    assert solver.true_residual() < 1e-9


def test_fe_source_and_resistance():
    case, km = "double_Y_N5", (2, 1)
    R = np.array([1.0, 2.5, 0.5, 3.0, 1.5, 2.0, 1.0])[: len(CASES[case][0]().edges())]
    mesh, asm, F, A, b, pbc = _setup(case, km, f=0.3, R=R)
    solver = Solver(asm)
    solver.assemble()
    sol = solver.solve()
    x_ref = O.solve_reference(A, b)
    got = np.concatenate([fn.x.array for fn in sol])
    assert np.linalg.norm(got - x_ref) / np.linalg.norm(x_ref) <= SOL_TOL


@pytest.mark.parametrize("km", [(2, 0), (3, 1)])
def test_fe_per_edge_source(km):
    case = "edge_info_N10"
    E = len(CASES[case][0]().edges())
    f = 0.2 + 0.1 * (np.arange(E) % 3)
    mesh, asm, F, A, b, pbc = _setup(case, km, f=f)
    asm.assemble()
    _, h = O.cell_geometry(F.base)
    _, hr = evaluate_terms(asm.fe_layout, np.ones(E), f, _edge_bc(F, pbc), h)
    np.testing.assert_array_equal(asm.handle.rhs(), hr)
    solver = Solver(asm)
    sol = solver.solve()
    x_ref = O.solve_reference(A, b)
    got = np.concatenate([fn.x.array for fn in sol])
    assert np.linalg.norm(got - x_ref) / np.linalg.norm(x_ref) <= SOL_TOL


@pytest.mark.parametrize("km", [(2, 0), (3, 1)])
def test_fe_global_flux(km):
    """DG_k global flux: q is constant per edge (f = 0), so its integral is sum q_e L_e."""
    mesh, asm, F, A, b, pbc = _setup("depth6_N40", km)
    solver = Solver(asm)
    solver.assemble()
    sol = solver.solve()
    g = extract_global_flux(mesh, sol)
    k = km[0]
    assert g.function_space.element.basix_element.degree == k
    assert g.x.array.size == mesh.num_edges * mesh.N * (k + 1)
    total, length = integrate_dg1(mesh, g)
    x1 = O.resistor_network_solution(O.build_problem(mesh.node_coordinates, *mesh.edges,
                                                     mesh.N, mesh.edge_colors), pbc)
    P1 = O.build_problem(mesh.node_coordinates, *mesh.edges, mesh.N, mesh.edge_colors)
    _, h = O.cell_geometry(P1)
    expect = float(np.sum(x1[P1.flux_offset] * h.sum(axis=1)))
    assert abs(total - expect) <= 1e-9 * abs(expect)
    assert abs(length - h.sum()) <= 1e-12 * h.sum()


def test_fe_reassemble_idempotent():
    mesh, asm, F, A, b, pbc = _setup("edge_info_N10", (3, 1))
    asm.assemble()
    v1 = asm.handle.csr()[2].copy()
    r1 = asm.handle.rhs().copy()
    asm.assemble()
    np.testing.assert_array_equal(asm.handle.csr()[2], v1)
    np.testing.assert_array_equal(asm.handle.rhs(), r1)


@pytest.mark.parametrize("km", [(1, 0), (2, 0), (3, 2)])
def test_fe_single_edge(km):
    """One edge, one cell: no multipliers; the device solve equals the direct solve."""
    import networkx as nx

    G = nx.DiGraph()
    G.add_node(0, pos=np.array([0.0, 0.0]))
    G.add_node(1, pos=np.array([0.0, 2.0]))
    G.add_edge(0, 1)
    mesh = NetworkMesh(G, N=1)
    pbc = CASES["Y_N4"][3]
    asm = HydraulicNetworkAssembler(mesh, flux_degree=km[0], pressure_degree=km[1])
    asm.compute_forms(p_bc_ex=pbc)
    solver = Solver(asm)
    solver.assemble()
    sol = solver.solve()
    F = OF.build_problem_fe(mesh.node_coordinates, *mesh.edges, 1, *km, mesh.edge_colors)
    x_ref = O.solve_reference(*OF.assemble_reference_fe(F, pbc))
    got = np.concatenate([fn.x.array for fn in sol])
    assert np.linalg.norm(got - x_ref) / np.linalg.norm(x_ref) <= SOL_TOL


@pytest.mark.parametrize("case", ["Y_N4", "double_Y_N5", "depth6_N40", "arterial5_N40",
                                  "tree6_2d_N70"])
@pytest.mark.parametrize("k", [2, 3, 4])
@pytest.mark.parametrize("struct", ["1", "0"])  # residual from the edge templates (default) / the CSR
def test_fe_direct_condensed(case, k, struct, monkeypatch):
    """(k, 0) through the condensed P1/DG0 system (nx_fe_set_direct): the direct path runs
    (no MINRES), within SOL_TOL of the oracle's LU, its reported residual is the true one,
    <= 1e-12 after at most two refinement passes; a second solve with other coefficients
    (the auxiliary lumped mass rebuilt) stays exact. Both residual kernels (k_fe_tres from the
    edge templates, k_residual_ck from the CSR) report it."""
    E = len(CASES[case][0]().edges())
    R = 1.0 + 0.5 * (np.arange(E) % 3)
    monkeypatch.setenv("NXHIP_FE_STRUCT", struct)
    mesh, asm, F, A, b, pbc = _setup(case, (k, 0), f=0.4, R=R)
    assert asm.fe_direct_available
    solver = Solver(asm)
    solver.assemble()
    sol = solver.solve()
    assert solver.ksp.solver_used == "direct" and solver.ksp.converged
    assert 1 <= solver.ksp.iterations <= 3
    x_ref = O.solve_reference(A, b)
    got = np.concatenate([fn.x.array for fn in sol])
    assert np.linalg.norm(got - x_ref) / np.linalg.norm(x_ref) <= SOL_TOL
    tr = solver.true_residual()
    assert tr <= 1e-12
    assert abs(solver.ksp.residual_estimate - tr) <= 1e-6 * tr + 1e-16
    # other coefficients: the same handles, the condensed masses rebuilt from the new R
    R2 = 2.0 - 0.25 * (np.arange(E) % 4)
    asm.compute_forms(p_bc_ex=pbc, f=0.1, R=R2)
    solver.assemble()
    sol = solver.solve()
    assert solver.ksp.solver_used == "direct" and solver.ksp.converged
    A2, b2 = OF.assemble_reference_fe(F, pbc, f=0.1, R=R2)
    x2 = O.solve_reference(A2, b2)
    got = np.concatenate([fn.x.array for fn in sol])
    assert np.linalg.norm(got - x2) / np.linalg.norm(x2) <= SOL_TOL


def _setup_cyclic(case, km, f=None, R=None):
    from cases import CYCLIC, p_y

    make, N = CYCLIC[case]
    mesh = NetworkMesh(make(), N=N)
    asm = HydraulicNetworkAssembler(mesh, flux_degree=km[0], pressure_degree=km[1])
    asm.compute_forms(p_bc_ex=p_y, f=f, R=R)
    src, dst = mesh.edges
    F = OF.build_problem_fe(mesh.node_coordinates, src, dst, N, *km, mesh.edge_colors)
    A, b = OF.assemble_reference_fe(F, p_y, f=0.0 if f is None else f,
                                    R=1.0 if R is None else R)
    return mesh, asm, F, A, b, p_y


@pytest.mark.parametrize("case", ["edge_info_N10", "lattice4x5_N6", "lattice6x6_N3"])
@pytest.mark.parametrize("k", [2, 3])
def test_fe_direct_cycles(case, k):
    """A graph with cycles (the reference's edge-info graph, two lattices with 12 / 25
    cycles): the (k, 0) direct solve through the condensed system runs -- the auxiliary tree
    solve corrected by the Woodbury step of the cycle chains' dropped couplings, built from
    the condensed mass (fe_cyc_build) -- within SOL_TOL of the oracle's LU, its reported
    residual the true one; new coefficients rebuild the correction."""
    from cases import CYCLIC

    E = len(CYCLIC[case][0]().edges())
    R = 1.0 + 0.5 * (np.arange(E) % 3)
    mesh, asm, F, A, b, pbc = _setup_cyclic(case, (k, 0), f=0.2, R=R)
    assert asm.fe_direct_available
    solver = Solver(asm)
    solver.assemble()
    sol = solver.solve()
    assert solver.ksp.solver_used == "direct" and solver.ksp.converged
    assert asm.handle.direct_path() == "condensed"
    got = np.concatenate([fn.x.array for fn in sol])
    x_ref = O.solve_reference(A, b)
    assert np.linalg.norm(got - x_ref) / np.linalg.norm(x_ref) <= SOL_TOL
    tr = solver.true_residual()
    assert tr <= 1e-12
    assert abs(solver.ksp.residual_estimate - tr) <= 1e-6 * tr + 1e-16
    R2 = 2.0 - 0.25 * (np.arange(E) % 4)
    asm.compute_forms(p_bc_ex=pbc, f=0.1, R=R2)
    solver.assemble()
    sol = solver.solve()
    assert solver.ksp.solver_used == "direct" and solver.ksp.converged
    A2, b2 = OF.assemble_reference_fe(F, pbc, f=0.1, R=R2)
    x2 = O.solve_reference(A2, b2)
    got = np.concatenate([fn.x.array for fn in sol])
    assert np.linalg.norm(got - x2) / np.linalg.norm(x2) <= SOL_TOL


@pytest.mark.parametrize("case,km", [("depth6_N40", (2, 1)), ("arterial5_N40", (3, 2)),
                                     ("tree6_2d_N70", (2, 1))])
def test_fe_cp_node_records_bits(case, km, monkeypatch):
    """The node kernels read each node's packed record (``CpTree::rec``) instead of its
    lists: the same sums in the same order, so x is bit-identical to the lists' path
    (``NXHIP_CP_NOREC=1``, read when the tables are attached)."""
    xs = []
    for norec in ("0", "1"):
        if norec == "1":
            monkeypatch.setenv("NXHIP_CP_NOREC", "1")
        else:
            monkeypatch.delenv("NXHIP_CP_NOREC", raising=False)
        mesh, asm, F, A, b, pbc = _setup(case, km, f=0.3)
        asm.set_direct(True)
        asm.assemble()
        it, rr, conv = asm.handle.solve(1e-12, 100, 4)
        assert conv and asm.handle.direct_path() == "node-condensed"
        xs.append(asm.handle.solution())
        asm.close()
    np.testing.assert_array_equal(xs[0], xs[1])


@pytest.mark.parametrize("km", [(2, 1), (3, 2)])
def test_fe_cp_pipelined_node_forest(km, monkeypatch):
    """The node forest pipelined across its level barriers (``k_cp_nodes_rec``), its levels
    below the first of more than 128 nodes as subtree chunks (one workgroup each, records
    re-ordered inside the levels): the same bits as the level-by-level kernels
    (``NXHIP_CP_PIPE=0``), on a depth-12 tree (levels of up to 4096 nodes), and the analytic
    answer."""
    from networks_fenicsx_amd import network_generation as ng

    mesh = NetworkMesh(ng.make_tree(13, 13, 13), N=3, color_strategy="smallest_last")
    asm = HydraulicNetworkAssembler(mesh, flux_degree=km[0], pressure_degree=km[1])
    try:
        asm.compute_forms(p_bc_ex=lambda x: x[1])
        asm.set_direct(True)
        xs = []
        for pipe, via_lds in (("0", "0"), ("1", "1"), ("1", "1"), ("1", "0")):
            monkeypatch.setenv("NXHIP_CP_PIPE", pipe)
            monkeypatch.setenv("NXHIP_CP_XS", via_lds)  # the back-substitution's rows via LDS
            asm.assemble()
            it, rr, conv = asm.handle.solve(1e-12, 100, 4)
            assert conv and asm.handle.direct_path() == "node-condensed", (pipe, it, rr)
            xs.append(asm.handle.solution())
        for x in xs[1:]:
            np.testing.assert_array_equal(xs[0], x)
        F = OF.build_problem_fe(mesh.node_coordinates, *mesh.edges, 3, *km, mesh.edge_colors)
        xa = OF.resistor_network_solution_fe(F, lambda x: x[1])
        x = np.concatenate([fn.x.array for fn in _functions(asm)])
        assert np.linalg.norm(x - xa) / np.linalg.norm(xa) <= SOL_TOL
    finally:
        asm.close()


@pytest.mark.parametrize("km", [(2, 1), (3, 2)])
def test_fe_cp_deep_node_forest(km, monkeypatch):
    """A 150-node line (150 node levels): the level run is longer than the pipelined
    kernel's 64, so it runs level by level in one workgroup on the node records (their
    parent terms); the same bits as the lists' path (NXHIP_CP_NOREC=1, read when the tables
    are attached) and the oracle's LU to 1e-10."""
    from cases import linear_graph

    xs = []
    for norec in ("0", "1"):
        if norec == "1":
            monkeypatch.setenv("NXHIP_CP_NOREC", "1")
        mesh = NetworkMesh(linear_graph(150, ordered=lambda k: k % 3 != 0), N=2)
        asm = HydraulicNetworkAssembler(mesh, flux_degree=km[0], pressure_degree=km[1])
        try:
            asm.compute_forms(p_bc_ex=lambda x: x[0])
            asm.set_direct(True)
            asm.assemble()
            it, rr, conv = asm.handle.solve(1e-12, 100, 4)
            assert conv and asm.handle.direct_path() == "node-condensed", (it, rr)
            xs.append(np.concatenate([fn.x.array for fn in _functions(asm)]))
            if norec == "0":
                F = OF.build_problem_fe(mesh.node_coordinates, *mesh.edges, 2, *km,
                                        mesh.edge_colors)
                A, b = OF.assemble_reference_fe(F, lambda x: x[0])
                x_ref = O.solve_reference(A, b)
                assert np.linalg.norm(xs[0] - x_ref) / np.linalg.norm(x_ref) <= SOL_TOL
        finally:
            asm.close()
    np.testing.assert_array_equal(xs[0], xs[1])


def _functions(asm):
    from networks_fenicsx_amd.fem import Function

    fns = [Function(V) for V in asm.flux_spaces] + [Function(asm.pressure_space),
                                                     Function(asm.lm_space)]
    return asm.scatter_solution(asm.handle.solution(), fns)


@pytest.mark.parametrize("case", ["Y_N4", "double_Y_N5", "depth6_N40", "arterial5_N40",
                                  "linear_alt_N3"])
@pytest.mark.parametrize("km", [(2, 1), (3, 2), (3, 1), (4, 3)])
def test_fe_continuous_pressure_direct(case, km):
    """Continuous pressure (k > m >= 1) by condensation onto the graph nodes (nx_fe_set_cp:
    per edge its forward sweep, the node system by one workgroup, per edge its
    back-substitution): the direct path runs (no MINRES) in at most three passes, within
    SOL_TOL of the oracle's LU (independently integrated tensors), its reported residual
    the true one; a second solve with other coefficients stays exact."""
    E = len(CASES[case][0]().edges())
    R = 1.0 + 0.5 * (np.arange(E) % 3)
    mesh, asm, F, A, b, pbc = _setup(case, km, f=0.4, R=R)
    assert asm.fe_direct_available
    solver = Solver(asm)
    solver.assemble()
    sol = solver.solve()
    assert solver.ksp.solver_used == "direct" and solver.ksp.converged
    assert asm.handle.direct_path() == "node-condensed"
    assert 1 <= solver.ksp.iterations <= 3
    x_ref = O.solve_reference(A, b)
    got = np.concatenate([fn.x.array for fn in sol])
    assert np.linalg.norm(got - x_ref) / np.linalg.norm(x_ref) <= SOL_TOL
    tr = solver.true_residual()
    assert tr <= 1e-12
    assert abs(solver.ksp.residual_estimate - tr) <= 1e-6 * tr + 1e-16
    R2 = 2.0 - 0.25 * (np.arange(E) % 4)
    asm.compute_forms(p_bc_ex=pbc, f=0.1, R=R2)
    solver.assemble()
    sol = solver.solve()
    assert solver.ksp.solver_used == "direct" and solver.ksp.converged
    A2, b2 = OF.assemble_reference_fe(F, pbc, f=0.1, R=R2)
    x2 = O.solve_reference(A2, b2)
    got = np.concatenate([fn.x.array for fn in sol])
    assert np.linalg.norm(got - x2) / np.linalg.norm(x2) <= SOL_TOL


def test_fe_continuous_pressure_cycles_run_minres():
    """A graph with cycles: no node-condensed tables, MINRES reaches the oracle's answer."""
    mesh, asm, F, A, b, pbc = _setup("edge_info_N10", (2, 1))
    assert not asm.fe_direct_available
    solver = Solver(asm)
    solver.assemble()
    sol = solver.solve()
    assert solver.ksp.solver_used == "minres" and solver.ksp.converged
    got = np.concatenate([fn.x.array for fn in sol])
    x_ref = O.solve_reference(A, b)
    assert np.linalg.norm(got - x_ref) / np.linalg.norm(x_ref) <= SOL_TOL


@pytest.mark.parametrize("case", ["depth6_N40", "arterial5_N40"])
@pytest.mark.parametrize("k", [2, 3])
def test_fe_condensed_template_residual_bits(case, k, monkeypatch):
    """The condensed route with the edge templates (assembly k_fe_tasm, residual k_fe_tres)
    gives x bit for bit as with the gather tables and the CSR residual (the same matrix and
    rhs bits, the same solve); the reported residuals agree to rounding."""
    E = len(CASES[case][0]().edges())
    R = 1.0 + 0.5 * (np.arange(E) % 3)
    mesh, asm, F, A, b, pbc = _setup(case, (k, 0), f=0.4, R=R)
    assert asm.handle.fe_templates()[0] > 0
    solver = Solver(asm)
    out = []
    for struct in ("1", "0"):
        monkeypatch.setenv("NXHIP_FE_STRUCT", struct)
        solver.assemble()
        solver.solve()
        assert solver.ksp.solver_used == "direct" and solver.ksp.iterations == 1
        out.append((asm.handle.solution(), solver.ksp.residual_estimate))
    np.testing.assert_array_equal(out[0][0], out[1][0])
    assert abs(out[0][1] - out[1][1]) <= 1e-3 * out[1][1] + 1e-16
