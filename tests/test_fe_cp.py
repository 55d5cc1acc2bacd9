"""Continuous pressure (k > m >= 1) solved by condensation onto the graph nodes (CPU model of
the device's nx_fe_set_cp solve, layout_fe.cp_model).

Each edge's flux and interior pressure nodes are eliminated onto its border -- the pressure
at its end nodes (shared with the other edges there) and the multipliers of the
bifurcations at its ends: per cell the interior nodes by the exact reference blocks scaled by
s = R h (element.condensed_cell_blocks), then the vertices (q, p) along the edge with 2 x 2
pivots; the border system over the graph nodes is negative definite and eliminated leaf to
root on the node forest. Checked against scipy's sparse LU of the full system (the MUMPS
stand-in) to 1e-10 on the reference's demo graphs, for (2, 1), (3, 1), (3, 2), (4, 3); the
reference blocks' scaling identity A(s) = T A(1) T; graphs with a cycle get no tables."""

from __future__ import annotations

import numpy as np
import pytest
import scipy.sparse as sp
import scipy.sparse.linalg as spla

from cases import CASES, CYCLIC
from networks_fenicsx_amd import NetworkMesh
from networks_fenicsx_amd.element import condensed_cell_blocks, element_tensors
from networks_fenicsx_amd.layout_fe import build_cp_tables, build_fe_layout, cp_model, evaluate_terms


def _cell_h(pos, src, dst, N):
    L = np.linalg.norm(pos[dst] - pos[src], axis=1)
    return np.repeat((L / N)[:, None], N, axis=1)


def _system(G, N, k, m, strategy=None):
    mesh = NetworkMesh(G, N=N, color_strategy=strategy)
    src, dst = mesh.edges
    pos = np.asarray(mesh.node_coordinates, dtype=np.float64)
    lay = build_fe_layout(pos, src, dst, mesh.degrees, N, k, m)
    E = mesh.num_edges
    R = 1.0 + 0.25 * (np.arange(E) % 3)
    bc = np.random.default_rng(3).standard_normal((E, 2))
    h = _cell_h(pos, src, dst, N)
    val, rhs = evaluate_terms(lay, R, 0.3, bc, h)
    A = sp.csr_matrix((val, lay.col, lay.rowptr), shape=(lay.n_rows, lay.n_rows))
    return mesh, lay, A, val, rhs, R, h


@pytest.mark.parametrize("case", ["Y_N4", "double_Y_N5", "tree5_N15", "arterial5_N40",
                                  "linear_alt_N3"])
@pytest.mark.parametrize("km", [(2, 1), (3, 1), (3, 2), (4, 3)])
def test_node_condensed_solve_equals_lu(case, km):
    make, N, strategy, _ = CASES[case]
    k, m = km
    N = min(N, 12)
    mesh, lay, A, val, rhs, R, h = _system(make(), N, k, m, strategy)
    src, dst = mesh.edges
    tab = build_cp_tables(lay, src, dst)
    assert tab is not None
    x_ref = spla.spsolve(A.tocsc(), rhs)
    x = cp_model(lay, tab, val, rhs, R, h)
    assert np.linalg.norm(x - x_ref) <= 1e-10 * np.linalg.norm(x_ref)
    # the true residual of the model's x (one pass, no refinement)
    assert np.linalg.norm(rhs - A @ x) <= 1e-11 * np.linalg.norm(rhs)


@pytest.mark.parametrize("km", [(2, 1), (3, 2), (4, 3)])
def test_condensed_cell_blocks_scaling(km):
    """The condensed cell matrix of A(s) = [[s M, -D^T], [-D, 0]] equals s^(t_r + t_c) Kh."""
    k, m = km
    Kh, Ch, Eh, Fh, tI = condensed_cell_blocks(k, m)
    Mref, Dref, _ = element_tensors(k, m)
    nq, npl = k + 1, m + 1
    s = 0.37
    A = np.zeros((nq + npl, nq + npl))
    A[:nq, :nq] = s * Mref
    A[:nq, nq:] = -Dref.T
    A[nq:, :nq] = -Dref
    V = [0, nq, k, nq + m]
    I = list(range(1, k)) + [nq + a for a in range(1, m)]
    K = A[np.ix_(V, V)] - A[np.ix_(V, I)] @ np.linalg.solve(A[np.ix_(I, I)], A[np.ix_(I, V)])
    t = np.array([1, -1, 1, -1])
    np.testing.assert_allclose(K, Kh * s ** ((t[:, None] + t[None, :]) // 2), rtol=1e-13,
                               atol=1e-13)


def test_cycles_have_no_tables():
    G = CYCLIC["edge_info_N10"][0]()
    mesh, lay, A, val, rhs, R, h = _system(G, 4, 2, 1)
    src, dst = mesh.edges
    assert build_cp_tables(lay, src, dst) is None
