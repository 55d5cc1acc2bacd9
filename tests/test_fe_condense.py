"""General flux degree k with DG0 pressure, solved through the P1/DG0 structure (CPU).

The divergence against a DG0 pressure touches only a cell's two vertex fluxes, so the
interior flux DoFs appear in the flux rows alone: condensing them per cell leaves the
P1/DG0 system with the cell mass R h [[alpha, beta], [beta, alpha]] (element.
condensed_flux_mass) in place of R h [[1/3, 1/6], [1/6, 1/3]] -- what the device's direct tree
solve inverts with (alpha, beta) (nx_fe_set_direct). Checked here on the host: condensing the
rhs with C, solving the P1-layout system with the rescaled masses and recovering the
interior values with K and Mii_inv gives the solution of the full (k, 0) system (scipy
sparse LU) to 1e-12, and the Schur identity the tree solve relies on holds for (alpha,
beta): (B M_s^-1 B^T)^-1 = (B D^-1 B^T)^-1 - beta R h I."""

from __future__ import annotations

import numpy as np
import pytest
import scipy.sparse as sp
import scipy.sparse.linalg as spla

from cases import CASES
from networks_fenicsx_amd import NetworkMesh
from networks_fenicsx_amd.element import condensed_flux_mass
from networks_fenicsx_amd.layout import build_local_problem
from networks_fenicsx_amd.layout_fe import build_fe_aux_maps, build_fe_layout, evaluate_terms
from oracle import nx_oracle as O


def _cell_h(pos, src, dst, N):
    L = np.linalg.norm(pos[dst] - pos[src], axis=1)
    return np.repeat((L / N)[:, None], N, axis=1)


@pytest.mark.parametrize("case", ["Y_N4", "double_Y_N5", "tree5_N15", "arterial5_N40"])
@pytest.mark.parametrize("k", [2, 3, 4])
def test_condensed_solve_equals_full(case, k):
    make, N, strategy, pbc = CASES[case]
    N = min(N, 12)
    m = NetworkMesh(make(), N=N, color_strategy=strategy)
    src, dst = m.edges
    pos = m.node_coordinates
    lay = build_fe_layout(pos, src, dst, m.degrees, N, k, 0)
    R = 1.0 + 0.25 * (np.arange(m.num_edges) % 3)
    bc = np.random.default_rng(1).standard_normal((m.num_edges, 2))
    h = _cell_h(np.asarray(pos, dtype=np.float64), src, dst, N)
    val, rhs = evaluate_terms(lay, R, 0.3, bc, h)
    A = sp.csr_matrix((val, lay.col, lay.rowptr), shape=(lay.n_rows, lay.n_rows))
    x = spla.spsolve(A.tocsc(), rhs)
    # the P1 system of the same graph (oracle, device layout), masses rescaled to (alpha, beta)
    lp = build_local_problem(pos, src, dst, m.degrees, N)
    mp = build_fe_aux_maps(lay, lp)
    alpha, beta, C, K, Mii = condensed_flux_mass(k)
    P = O.build_problem(pos, src, dst, N, m.edge_colors)
    A1, b1 = O.assemble_reference(P, pbc, R=R)
    Ab, _, _, _ = O.to_build_layout(P, A1, b1)
    Ab = Ab.tolil()
    per1 = 2 * N + 1
    n_e = lp.n_edge_dofs
    Ad = Ab.toarray()
    for r in range(n_e):
        if r % per1 % 2:
            continue  # pressure rows: +-1 only
        for c in range(n_e):
            if c % per1 % 2 == 0 and c // per1 == r // per1 and Ad[r, c] != 0.0:
                Ad[r, c] *= 3 * alpha if r == c else 6 * beta
    # condensed rhs: vertex rows b_v - C b_i per adjacent cell; pressure and multipliers copied
    nb = np.zeros(Ab.shape[0])
    E = m.num_edges
    bi = rhs[mp.i_fe].reshape(E, N, k - 1)
    bv = rhs[mp.v_fe].reshape(E, N + 1).copy()
    bv[:, :N] -= bi @ C[0]
    bv[:, 1:] -= bi @ C[1]
    nb[mp.v_aux] = bv.ravel()
    nb[mp.p_aux] = rhs[mp.p_fe]
    nb[mp.l_aux] = rhs[mp.l_fe]
    xa = np.linalg.solve(Ad, nb)
    xv = xa[mp.v_aux].reshape(E, N + 1)
    Rh = (np.asarray(R)[:, None] * h)[:, :, None]
    xi = (bi @ Mii.T) / Rh - (xv[:, :N, None] * K[:, 0][None, None, :]
                              + xv[:, 1:, None] * K[:, 1][None, None, :])
    got = np.zeros(lay.n_rows)
    got[mp.v_fe] = xv.ravel()
    got[mp.i_fe] = xi.ravel()
    got[mp.p_fe] = xa[mp.p_aux]
    got[mp.l_fe] = xa[mp.l_aux]
    assert np.linalg.norm(got - x) <= 1e-12 * np.linalg.norm(x)


@pytest.mark.parametrize("k", [1, 2, 3, 4, 5])
def test_schur_identity_for_condensed_masses(k):
    alpha, beta, _, _, _ = condensed_flux_mass(k)
    N, h, R = 7, 0.37, 1.9
    Ms = np.zeros((N + 1, N + 1))
    for c in range(N):
        Ms[c:c + 2, c:c + 2] += R * h * np.array([[alpha, beta], [beta, alpha]])
    B = np.zeros((N, N + 1))
    B[np.arange(N), np.arange(N)] = 1.0
    B[np.arange(N), np.arange(N) + 1] = -1.0
    S = B @ np.linalg.solve(Ms, B.T)
    SL = B @ np.linalg.solve(np.diag(Ms.sum(1)), B.T)
    np.testing.assert_allclose(np.linalg.inv(S), np.linalg.inv(SL) - beta * R * h * np.eye(N),
                               atol=1e-12)


@pytest.mark.parametrize("k", [2, 3])
def test_flattened_constants_as_the_kernels_index_them(k):
    """The constants nx_fe_set_direct uploads (assembly.py: C | K | Mii, row-major) read
    with k_fe_condense's / k_fe_expand's indexing: C row 0 at cst[i], row 1 at cst[km + i],
    K[j] at cst[2 km + 2 j + {0, 1}], Mii[j][i] at cst[4 km + j km + i]; the exact condensed
    ratios a / b = (-1)^(k+1) (k+1) and (a + b) / b that nx_set_cell_mass receives."""
    alpha, beta, C, K, Mii = condensed_flux_mass(k)
    km = k - 1
    cst = np.concatenate([C.ravel(), K.ravel(), Mii.ravel()])
    assert cst.size == 4 * km + km * km
    for i in range(km):
        assert cst[i] == C[0, i] and cst[km + i] == C[1, i]
    for j in range(km):
        assert cst[2 * km + 2 * j] == K[j, 0] and cst[2 * km + 2 * j + 1] == K[j, 1]
        for i in range(km):
            assert cst[4 * km + j * km + i] == Mii[j, i]
    ratio = (-1) ** (k + 1) * (k + 1)
    assert abs(alpha / beta - ratio) < 1e-12
    assert abs((alpha + beta) / beta - (ratio + 1)) < 1e-12
    # the pivots of T = tridiag(1, 2 ratio, 1) with ratio at both ends stay away from zero
    N = 9
    T = np.diag(np.full(N + 1, 2.0 * ratio)) + np.diag(np.ones(N), 1) + np.diag(np.ones(N), -1)
    T[0, 0] = T[N, N] = ratio
    Ms = np.zeros((N + 1, N + 1))
    for c in range(N):
        Ms[c:c + 2, c:c + 2] += np.array([[alpha, beta], [beta, alpha]])
    np.testing.assert_allclose(T * beta, Ms, atol=1e-15)
