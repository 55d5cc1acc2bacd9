"""The CPU oracle against its known answers (before it is trusted as the checker)."""

import numpy as np
import pytest

from cases import CASES, GOLDEN_CASES
from networks_fenicsx_amd import NetworkMesh
from oracle import nx_oracle as O

SMALL = ["Y_N4", "demo_tree_N2", "demo_tree_N1", "double_Y_N5", "depth6_N40",
         "arterial5_N40", "edge_info_N10", "linear_alt_N3"]


def _problem(case):
    make, N, strategy, pbc = CASES[case]
    m = NetworkMesh(make(), N=N, color_strategy=strategy)
    src, dst = m.edges
    return m, O.build_problem(m.node_coordinates, src, dst, N, m.edge_colors), pbc


@pytest.mark.parametrize("case", SMALL)
def test_direct_solution_equals_resistor_network(case):
    m, P, pbc = _problem(case)
    A, b = O.assemble_reference(P, pbc)
    x = O.solve_reference(A, b)
    xa = O.resistor_network_solution(P, pbc)
    assert np.linalg.norm(x - xa) / np.linalg.norm(xa) < 1e-12


@pytest.mark.parametrize("case", SMALL)
def test_build_layout_is_symmetric_and_equivalent(case):
    m, P, pbc = _problem(case)
    A, b = O.assemble_reference(P, pbc)
    Ab, bb, perm, sign = O.to_build_layout(P, A, b)
    assert abs(Ab - Ab.T).max() == 0.0
    x = O.solve_reference(A, b)
    np.testing.assert_allclose(Ab @ x[perm], bb, atol=1e-12)
    # nnz formula of SURVEY.md 8: E(7N+1) + 2 * sum of bifurcation degrees
    deg = P.degree
    assert A.nnz == P.src.size * (7 * P.N + 1) + 2 * int(deg[deg > 1].sum())


def test_reference_signs():
    """Y graph (make_tree(2,1,3), N=4): the block entries the reference forms define."""
    m, P, pbc = _problem("Y_N4")
    A, b = O.assemble_reference(P, pbc)
    A = A.toarray()
    N = 4
    e = 0  # root edge (0 -> 1): flux DoFs of colour 0 first
    q0, qN = P.flux_offset[e], P.flux_offset[e] + N
    p0 = P.p_offset
    assert A[p0, q0] == -1 and A[p0, q0 + 1] == 1  # phi dq/ds (assembly.py:254)
    assert A[q0, p0] == 1 and A[q0 + 1, p0] == -1  # -p dv/ds (assembly.py:255)
    lam = P.lm_offset
    assert A[lam, qN] == 1 and A[qN, lam] == 1  # in-edge end of the junction
    e1 = 1
    assert A[lam, P.flux_offset[e1]] == -1  # out-edge start
    # rhs: -p_bc(root) at the root edge start (p_bc = y = 0 there), +p_bc at leaves (y = 1)
    assert b[q0] == 0.0
    assert b[P.flux_offset[1] + N] == 1.0 and b[P.flux_offset[2] + N] == 1.0


@pytest.mark.parametrize("N", [2, 4, 16])
def test_demo_tree_closed_form(N):
    m, P, pbc = _problem("demo_tree_N2")
    from networks_fenicsx_amd import network_generation as ng

    m = NetworkMesh(ng.make_tree(2, 1, 1), N=N)
    src, dst = m.edges
    P = O.build_problem(m.node_coordinates, src, dst, N)
    A, b = O.assemble_reference(P, lambda x: x[1])
    x = O.solve_reference(A, b)
    q = x[: P.p_offset]
    s2 = np.sqrt(2.0)
    assert abs(q.min() - (2 - s2)) < 1e-12 and abs(q.max() - (4 - 2 * s2)) < 1e-12
    assert abs(x[P.lm_offset] + (2 - s2)) < 1e-12


@pytest.mark.parametrize("case", GOLDEN_CASES)
def test_golden_systems_reproduce(systems, case):
    m, P, pbc = _problem(case)
    A, b = O.assemble_reference(P, pbc)
    Ab, bb, perm, sign = O.to_build_layout(P, A, b)
    if f"{case}/indptr" in systems:
        np.testing.assert_array_equal(Ab.indptr, systems[f"{case}/indptr"])
        np.testing.assert_array_equal(Ab.indices, systems[f"{case}/indices"])
        np.testing.assert_array_equal(Ab.data, systems[f"{case}/data"])
    np.testing.assert_array_equal(bb, systems[f"{case}/rhs_build"])
    x = O.solve_reference(A, b)[perm]
    np.testing.assert_allclose(x, systems[f"{case}/x_build"], rtol=0, atol=1e-12)
    np.testing.assert_allclose(systems[f"{case}/x_analytic_build"], systems[f"{case}/x_build"],
                               rtol=0, atol=1e-11)


def test_golden_arterial_reference_order(systems):
    """C2 (demo_arterial_tree.py: largest_first colouring, N = 40): the fixture's solution in
    the reference's function order is the oracle's, and equals the build-layout solution
    regrouped per colour; the fixture's radii are the generator's."""
    m, P, pbc = _problem("arterial5_N40")
    np.testing.assert_array_equal(m.edge_colors, systems["arterial5_N40/colors"])
    np.testing.assert_array_equal(m.edge_radius, systems["arterial5_N40/radius"])
    A, b = O.assemble_reference(P, pbc)
    x = O.solve_reference(A, b)
    np.testing.assert_allclose(x, systems["arterial5_N40/x_ref_blocks"], rtol=0, atol=1e-12)
    _, _, perm, _ = O.to_build_layout(P, A, b)
    np.testing.assert_allclose(x[perm], systems["arterial5_N40/x_build"], rtol=0, atol=1e-12)


def test_per_edge_R_and_source():
    m, P, pbc = _problem("arterial5_N40")
    R = 1.0 / m.edge_radius ** 4
    A, b = O.assemble_reference(P, pbc, f=0.0, R=R)
    x = O.solve_reference(A, b)
    xa = O.resistor_network_solution(P, pbc, R=R)
    assert np.linalg.norm(x - xa) / np.linalg.norm(xa) < 1e-12
    A2, b2 = O.assemble_reference(P, pbc, f=0.5, R=R)
    assert (A2 != A).nnz == 0
    _, h = O.cell_geometry(P)
    np.testing.assert_allclose(b2[P.p_offset:P.lm_offset], 0.5 * h.ravel())
