"""General degrees (k, 0) on several ranks: the rank layouts (``layout_fe.build_fe_rank_layout``)
against the one-rank layout (CPU).

Bar: on one rank the rank layout IS the one-rank layout (every table equal); on 2-4 ranks
every owned row of every rank, mapped to the one-rank numbering, holds exactly the one-rank
row's columns and (by the host evaluation of the term tables) bit-identical values and rhs;
every row is owned once; the halo plans line up (what a rank sends is the global DoF its
peer's ghost column names).
"""

from __future__ import annotations

import numpy as np
import pytest

from cases import CASES
from networks_fenicsx_amd import NetworkMesh
from networks_fenicsx_amd.layout import build_local_problem
from networks_fenicsx_amd.layout_fe import (build_fe_layout, build_fe_rank_layout,
                                            evaluate_terms, fe_global_rows)


def _mesh(case):
    make, N, strategy, _ = CASES[case]
    return NetworkMesh(make(), N=N, color_strategy=strategy)


def _ghost_global(lay, lp, N, k):
    """One-rank row of every ghost column (from the P1 rank layout's global ids)."""
    per1, per = 2 * N + 1, k * N + 1 + N
    E = lay.n_edges_global
    g = np.asarray(lp.ghost_global, dtype=np.int64)
    e, j = np.divmod(np.minimum(g, E * per1 - 1), per1)
    return np.where(g >= E * per1, E * per + (g - E * per1), e * per + np.where(j == 0, 0, k * N))


def _terms(lay, mesh, R, f):
    edges = np.arange(lay.E) if lay.edges is None else lay.edges
    src, dst = mesh.edges
    pos = mesh.node_coordinates
    h = np.linalg.norm(pos[dst[edges]] - pos[src[edges]], axis=1)[:, None] / mesh.N
    h = np.repeat(h, mesh.N, axis=1)
    bc = np.stack([0.3 + 0.01 * edges, -0.2 - 0.02 * edges], axis=1)
    return evaluate_terms(lay, R[edges], f[edges], bc, h)


@pytest.mark.parametrize("case", ["Y_N4", "edge_info_N10", "double_Y_N5"])
@pytest.mark.parametrize("k", [2, 3])
def test_one_rank_layout_is_the_layout(case, k):
    mesh = _mesh(case)
    src, dst = mesh.edges
    full = build_fe_layout(mesh.node_coordinates, src, dst, mesh.degrees, mesh.N, k, 0)
    lp = build_local_problem(mesh.node_coordinates, src, dst, mesh.degrees, mesh.N, 0, 1)
    one = build_fe_rank_layout(mesh.node_coordinates, src, dst, mesh.N, k, lp)
    for name in ("rowptr", "col", "table_kind", "table_val", "a_ptr", "a_idx", "a_ent", "b_ptr",
                 "b_idx", "b_ent", "flux_rows", "p_rows", "lm_nodes", "lm_rows", "edge_x"):
        np.testing.assert_array_equal(getattr(one, name), getattr(full, name), err_msg=name)
    assert one.n_rows == full.n_rows and one.n_ghost == 0


@pytest.mark.parametrize("case", ["Y_N4", "edge_info_N10", "double_Y_N5", "depth6_N40",
                                  "arterial5_N40"])
@pytest.mark.parametrize("P", [2, 3, 4])
@pytest.mark.parametrize("k", [2, 3])
def test_rank_layouts_cover_the_layout(case, P, k):
    mesh = _mesh(case)
    src, dst = mesh.edges
    N, E = mesh.N, mesh.num_edges
    full = build_fe_layout(mesh.node_coordinates, src, dst, mesh.degrees, N, k, 0)
    R = 1.0 + 0.25 * (np.arange(E) % 5)
    f = 0.1 + 0.05 * (np.arange(E) % 3)
    fv, fr = _terms(full, mesh, R, f)
    owned = np.zeros(full.n_rows, dtype=np.int64)
    lays, lps, gids = [], [], []
    for r in range(P):
        lp = build_local_problem(mesh.node_coordinates, src, dst, mesh.degrees, N, r, P)
        lay = build_fe_rank_layout(mesh.node_coordinates, src, dst, N, k, lp)
        assert lay.n_ghost == lp.n_ghost and lay.E == lp.edges.size
        rows = fe_global_rows(lay, mesh.degrees)
        cols = np.concatenate([rows, _ghost_global(lay, lp, N, k)])
        owned[rows] += 1
        v, b = _terms(lay, mesh, R, f)
        for i in range(lay.n_rows):
            g = rows[i]
            s0, s1 = lay.rowptr[i], lay.rowptr[i + 1]
            t0, t1 = full.rowptr[g], full.rowptr[g + 1]
            got = sorted(zip(cols[lay.col[s0:s1]].tolist(), v[s0:s1].tolist()))
            want = sorted(zip(full.col[t0:t1].tolist(), fv[t0:t1].tolist()))
            assert got == want, (r, i, g)
            assert b[i] == fr[g]
        lays.append(lay)
        lps.append(lp)
        gids.append(cols)
    np.testing.assert_array_equal(owned, 1)  # every row owned exactly once
    # halo: what rank r sends to peer q, in order, is q's ghost columns from r
    for r, (lay, cols) in enumerate(zip(lays, gids)):
        for j, q in enumerate(lay.peers.tolist()):
            sent = cols[lay.send_idx[lay.send_off[j]:lay.send_off[j + 1]]]
            lq = lays[q]
            jq = lq.peers.tolist().index(r)
            recv = gids[q][lq.n_rows + np.arange(lq.recv_off[jq], lq.recv_off[jq + 1])]
            np.testing.assert_array_equal(sent, recv)


def _partition(mesh, k, m, P):
    from networks_fenicsx_amd.layout import partition_edges
    from networks_fenicsx_amd.layout_fe import build_fe_partition

    src, dst = mesh.edges
    full = build_fe_layout(mesh.node_coordinates, src, dst, mesh.degrees, mesh.N, k, m)
    owner = partition_edges(src, dst, mesh.node_coordinates.shape[0], P)
    return full, [build_fe_partition(full, src, dst, owner, r, P) for r in range(P)]


@pytest.mark.parametrize("case", ["Y_N4", "edge_info_N10", "double_Y_N5", "depth6_N40",
                                  "arterial5_N40"])
@pytest.mark.parametrize("P", [2, 3, 4])
@pytest.mark.parametrize("km", [(2, 1), (3, 1), (3, 2), (2, 0)])
def test_partitions_cover_the_layout(case, P, km):
    """Any pair, continuous pressure's shared node rows included (``build_fe_partition``):
    every owned row is the one-rank row (columns, values and rhs bit for bit), the ghost
    edges give the remote cells' terms, every row is owned once, the halo plans line up."""
    mesh = _mesh(case)
    E = mesh.num_edges
    full, lays = _partition(mesh, *km, P)
    R = 1.0 + 0.25 * (np.arange(E) % 5)
    f = 0.1 + 0.05 * (np.arange(E) % 3)
    fv, fr = _terms(full, mesh, R, f)
    owned = np.zeros(full.n_rows, dtype=np.int64)
    gids = []
    for r, lay in enumerate(lays):
        rows = fe_global_rows(lay, mesh.degrees)
        cols = np.concatenate([rows, lay.ghost_rows])
        owned[rows] += 1
        v, b = _terms(lay, mesh, R, f)
        for i in range(lay.n_rows):
            g = rows[i]
            s0, s1 = lay.rowptr[i], lay.rowptr[i + 1]
            t0, t1 = full.rowptr[g], full.rowptr[g + 1]
            assert (np.diff(lay.col[s0:s1]) > 0).all()  # sorted local columns
            got = sorted(zip(cols[lay.col[s0:s1]].tolist(), v[s0:s1].tolist()))
            want = sorted(zip(full.col[t0:t1].tolist(), fv[t0:t1].tolist()))
            assert got == want, (r, i, g)
            assert b[i] == fr[g]
        gids.append(cols)
    np.testing.assert_array_equal(owned, 1)
    for r, (lay, cols) in enumerate(zip(lays, gids)):
        for j, q in enumerate(lay.peers.tolist()):
            sent = cols[lay.send_idx[lay.send_off[j]:lay.send_off[j + 1]]]
            lq = lays[q]
            jq = lq.peers.tolist().index(r)
            recv = gids[q][lq.n_rows + np.arange(lq.recv_off[jq], lq.recv_off[jq + 1])]
            np.testing.assert_array_equal(sent, recv)


@pytest.mark.parametrize("case", ["edge_info_N10", "depth6_N40"])
@pytest.mark.parametrize("P", [2, 3])
def test_partition_is_the_rank_layout_for_dg0(case, P):
    """(k, 0): the generic partition and the P1-derived rank layout are the same tables (no
    ghost edges: DG0's multiplier rows read no cells)."""
    mesh = _mesh(case)
    src, dst = mesh.edges
    full, lays = _partition(mesh, 2, 0, P)
    for r, part in enumerate(lays):
        lp = build_local_problem(mesh.node_coordinates, src, dst, mesh.degrees, mesh.N, r, P)
        lay = build_fe_rank_layout(mesh.node_coordinates, src, dst, mesh.N, 2, lp)
        assert part.n_own_edges == part.E == lay.E and part.n_ghost == lay.n_ghost
        for name in ("rowptr", "col", "a_ptr", "a_idx", "a_ent", "b_ptr", "b_idx", "b_ent",
                     "flux_rows", "p_rows", "lm_rows", "edge_x", "peers", "send_off",
                     "send_idx", "recv_off"):
            np.testing.assert_array_equal(getattr(part, name), getattr(lay, name), err_msg=name)


@pytest.mark.parametrize("case", ["Y_N4", "double_Y_N5", "depth6_N40", "arterial5_N40"])
@pytest.mark.parametrize("P", [2, 3])
@pytest.mark.parametrize("km", [(2, 1), (3, 2)])
def test_cp_rank_tables(case, P, km):
    """The node-condensed solve's rank tables (``build_cp_rank_tables``): every node row is
    written by exactly one rank, from one of its own edges incident to the node; the edge
    kernels cover every edge once; the node rhs slots are 2n / 2n + 1."""
    from networks_fenicsx_amd.layout_fe import build_cp_rank_tables, build_cp_tables

    mesh = _mesh(case)
    src, dst = mesh.edges
    full, lays = _partition(mesh, *km, P)
    tab = build_cp_tables(full, src, dst)
    n = tab.n_nodes
    written = np.zeros(full.n_rows, dtype=np.int64)
    edges_run = np.zeros(mesh.num_edges, dtype=np.int64)
    for lay in lays:
        tr, gid, nrowx = build_cp_rank_tables(tab, lay)
        nrowx = nrowx.reshape(n, 2)
        edges_run[gid] += 1
        np.testing.assert_array_equal(tr.eb.reshape(-1, 4), tab.eb.reshape(-1, 4)[gid])
        nb = tr.nrow.reshape(n, 2)
        np.testing.assert_array_equal(nb[:, 0], 2 * np.arange(n))
        for nd in range(n):
            if nrowx[nd, 0] < 0:
                assert tr.nown[nd] == -1
                continue
            g = lay.global_rows[nrowx[nd]]
            assert g[0] == tab.nrow[2 * nd]
            written[g[0]] += 1
            if tab.nrow[2 * nd + 1] >= 0:
                assert g[1] == tab.nrow[2 * nd + 1]
                written[g[1]] += 1
            e = gid[tr.nown[nd]]
            assert nd in (tab.eb[4 * e], tab.eb[4 * e + 1])
    np.testing.assert_array_equal(edges_run, 1)
    node_rows = tab.nrow.reshape(n, 2)
    np.testing.assert_array_equal(written[node_rows[:, 0]], 1)
    lam = node_rows[node_rows[:, 1] >= 0, 1]
    np.testing.assert_array_equal(written[lam], 1)
