"""General element degrees on the CPU: the oracle restatement against its known answers,
and the host layout / term tables (``layout_fe.py``) against the oracle (no GPU).

Parity for degrees other than (1, 0) is pinned analytically (see ``oracle/nx_oracle_fe.py``):
the reference's own tests and demos only use the default degrees.
"""

import numpy as np
import pytest
import scipy.sparse as sp

from cases import CASES
from networks_fenicsx_amd import HydraulicNetworkAssembler, NetworkMesh
from networks_fenicsx_amd.element import element_tensors, stable_pair
from networks_fenicsx_amd.layout_fe import build_fe_layout, evaluate_terms
from oracle import nx_oracle as O
from oracle import nx_oracle_fe as OF

STABLE = [(1, 0), (2, 0), (3, 0), (2, 1), (3, 1), (3, 2), (4, 2)]
SMALL = ["Y_N4", "double_Y_N5", "demo_tree_N2", "edge_info_N10", "linear_alt_N3"]


def _mesh(case):
    make, N, strategy, pbc = CASES[case]
    return NetworkMesh(make(), N=N, color_strategy=strategy), pbc


@pytest.mark.parametrize("k", [1, 2, 3, 4, 5])
@pytest.mark.parametrize("m", [0, 1, 2, 3])
def test_element_tensors_two_ways(k, m):
    """Exact rational integration (product) vs Gauss-Legendre quadrature (oracle)."""
    for a, b in zip(element_tensors(k, m), OF.reference_tensors(k, m)):
        np.testing.assert_allclose(a, b, rtol=0, atol=2e-14)


def test_element_tensors_known_values():
    M, D, w = element_tensors(1, 0)
    np.testing.assert_array_equal(M, [[1 / 3, 1 / 6], [1 / 6, 1 / 3]])
    np.testing.assert_array_equal(D, [[-1.0, 1.0]])  # assembly.py:254, P1 / DG0
    M2, D2, _ = element_tensors(2, 0)
    np.testing.assert_allclose(M2, np.array([[4, 2, -1], [2, 16, 2], [-1, 2, 4]]) / 30, atol=1e-16)
    np.testing.assert_array_equal(D2, [[-1.0, 0.0, 1.0]])  # the bubble integrates to 0


@pytest.mark.parametrize("case", SMALL)
def test_degree_one_zero_equals_p1_oracle(case):
    m, pbc = _mesh(case)
    src, dst = m.edges
    P = O.build_problem(m.node_coordinates, src, dst, m.N, m.edge_colors)
    A, b = O.assemble_reference(P, pbc)
    F = OF.build_problem_fe(m.node_coordinates, src, dst, m.N, 1, 0, m.edge_colors)
    Af, bf = OF.assemble_reference_fe(F, pbc)
    assert abs(A - Af).max() <= 2.3e-16 * abs(A).max()
    np.testing.assert_array_equal(b, bf)


@pytest.mark.parametrize("case", SMALL)
@pytest.mark.parametrize("km", [(2, 1), (3, 1), (3, 2), (4, 2)])
def test_continuous_pressure_equals_resistor_network(case, km):
    m, pbc = _mesh(case)
    src, dst = m.edges
    F = OF.build_problem_fe(m.node_coordinates, src, dst, m.N, *km, m.edge_colors)
    A, b = OF.assemble_reference_fe(F, pbc)
    x = O.solve_reference(A, b)
    xa = OF.resistor_network_solution_fe(F, pbc)
    assert np.linalg.norm(x - xa) / np.linalg.norm(xa) < 1e-12


@pytest.mark.parametrize("km", [(1, 1), (1, 2), (2, 2)])
def test_unstable_pairs_are_singular(km):
    """Why the assembler refuses k <= m >= 1: the reference's direct solve would fail."""
    m, pbc = _mesh("demo_tree_N2")
    src, dst = m.edges
    F = OF.build_problem_fe(m.node_coordinates, src, dst, m.N, *km, m.edge_colors)
    A, _ = OF.assemble_reference_fe(F, pbc)
    s = np.linalg.svd(A.toarray(), compute_uv=False)
    assert s[-1] / s[0] < 1e-14
    assert not stable_pair(*km)
    with pytest.raises(ValueError, match="singular"):
        HydraulicNetworkAssembler(m, flux_degree=km[0], pressure_degree=km[1])


def _reference_in_device_layout(m, lay, pbc, f, R):
    src, dst = m.edges
    F = OF.build_problem_fe(m.node_coordinates, src, dst, m.N, lay.k, lay.m, m.edge_colors)
    A, b = OF.assemble_reference_fe(F, pbc, f=f, R=R)
    perm = np.empty(lay.n_rows, dtype=np.int64)
    sign = np.ones(lay.n_rows)
    perm[lay.flux_rows.ravel()] = (F.flux_offset[:, None]
                                   + np.arange(lay.k * m.N + 1)[None, :]).ravel()
    perm[lay.p_rows] = F.p_offset + np.arange(F.n_p)
    sign[lay.p_rows] = -1.0
    perm[lay.lm_rows] = F.lm_offset + np.arange(lay.lm_nodes.size)
    Ar = (sp.diags(sign) @ A[perm][:, perm]).tocsr()
    return F, Ar, sign * b[perm], perm


def _edge_bc(m, F, pbc):
    src, dst = m.edges
    pb = O._nodal(pbc, F.base.pos3)
    leaf = np.zeros(pb.size, dtype=bool)
    leaf[F.base.leaf_in] = True
    root = np.zeros(pb.size, dtype=bool)
    root[F.base.root_out] = True
    bc = np.zeros((src.size, 2))
    bc[:, 0] = np.where(root[src], -pb[src], 0.0)
    bc[:, 1] = np.where(leaf[dst], pb[dst], 0.0)
    return bc


@pytest.mark.parametrize("case", ["Y_N4", "edge_info_N10", "depth6_N40"])
@pytest.mark.parametrize("km", STABLE)
def test_layout_terms_reproduce_the_forms(case, km):
    """The host term tables, evaluated like k_assemble_fe, give the oracle's symmetric system."""
    m, pbc = _mesh(case)
    src, dst = m.edges
    lay = build_fe_layout(m.node_coordinates, src, dst, m.degrees, m.N, *km)
    f, R = 0.7, 1.0 + np.arange(src.size) % 3
    F, Ar, br, _ = _reference_in_device_layout(m, lay, pbc, f, R)
    _, h = O.cell_geometry(F.base)
    val, rhs = evaluate_terms(lay, R, f, _edge_bc(m, F, pbc), h)
    Ad = sp.csr_matrix((val, lay.col, lay.rowptr), shape=(lay.n_rows, lay.n_rows))
    assert abs(Ad - Ar).max() <= 1e-14 * abs(Ar).max()
    assert abs(Ad - Ad.T).max() == 0.0
    np.testing.assert_allclose(rhs, br, rtol=0, atol=1e-15 * max(1.0, np.abs(br).max()))
    # every row sorted, no duplicates, structural pattern covers the oracle's nonzeros
    d = np.diff(lay.col.astype(np.int64))
    starts = lay.rowptr[1:-1]
    assert np.all((d > 0) | np.isin(np.arange(1, lay.col.size), starts))
    assert Ad.nnz >= Ar.nnz


def test_layout_sizes():
    m, _ = _mesh("Y_N4")  # 3 edges, N = 4, one bifurcation, 4 nodes
    src, dst = m.edges
    lay = build_fe_layout(m.node_coordinates, src, dst, m.degrees, 4, 2, 1)
    # flux 3*(2*4+1) + interior pressure 3*(1*4-1) + node pressure 4 + multiplier 1
    assert lay.n_rows == 27 + 9 + 4 + 1
    assert lay.p_rows.size == 4 + 9
    lay0 = build_fe_layout(m.node_coordinates, src, dst, m.degrees, 4, 3, 0)
    assert lay0.n_rows == 3 * 13 + 3 * 4 + 1


@pytest.mark.parametrize("km", [(2, 0), (2, 1), (3, 2)])
@pytest.mark.parametrize("N", [1, 2])
def test_layout_single_edge(km, N):
    """Edge cases: one edge (no bifurcation, no multiplier), one cell per edge."""
    import networkx as nx

    G = nx.DiGraph()
    G.add_node(0, pos=np.array([0.0, 0.0]))
    G.add_node(1, pos=np.array([0.0, 2.0]))
    G.add_edge(0, 1)
    m = NetworkMesh(G, N=N)
    pbc = CASES["Y_N4"][3]
    src, dst = m.edges
    lay = build_fe_layout(m.node_coordinates, src, dst, m.degrees, N, *km)
    assert lay.lm_nodes.size == 0
    F, Ar, br, _ = _reference_in_device_layout(m, lay, pbc, 0.0, np.ones(1))
    _, h = O.cell_geometry(F.base)
    val, rhs = evaluate_terms(lay, np.ones(1), 0.0, _edge_bc(m, F, pbc), h)
    Ad = sp.csr_matrix((val, lay.col, lay.rowptr), shape=(lay.n_rows, lay.n_rows))
    assert abs(Ad - Ar).max() <= 1e-14 * abs(Ar).max()
    np.testing.assert_allclose(rhs, br, rtol=0, atol=1e-15)
    x = O.solve_reference(*OF.assemble_reference_fe(F, pbc))
    if km[1] >= 1:
        xa = OF.resistor_network_solution_fe(F, pbc)
        assert np.linalg.norm(x - xa) / np.linalg.norm(xa) < 1e-12


def test_per_edge_source_reduces_to_constant():
    m, pbc = _mesh("edge_info_N10")
    src, dst = m.edges
    F = OF.build_problem_fe(m.node_coordinates, src, dst, m.N, 2, 1, m.edge_colors)
    _, b1 = OF.assemble_reference_fe(F, pbc, f=0.4)
    _, b2 = OF.assemble_reference_fe(F, pbc, f=np.full(src.size, 0.4))
    np.testing.assert_array_equal(b1, b2)
    P = O.build_problem(m.node_coordinates, src, dst, m.N, m.edge_colors)
    np.testing.assert_array_equal(O.assemble_reference(P, pbc, f=0.4)[1],
                                  O.assemble_reference(P, pbc, f=np.full(src.size, 0.4))[1])
