"""DoF layout and gather-assembly tables for general element degrees.

``HydraulicNetworkAssembler(mesh, flux_degree=k, pressure_degree=m)`` (reference
``assembly.py:121-146``) with ``(k, m) != (1, 0)``. The P1/DG0 default keeps its own layout
and kernels (``layout.py``, ``k_assemble*``); this module serves every other stable pair.

Device layout (``n_rows`` owned rows, no ghosts):

* every graph edge ``e`` (``graph.edges()`` order) owns ``kN+1`` flux rows (the Lagrange
  nodes along the edge, source -> target) followed by its edge-interior pressure rows:
  ``N`` cell values for DG0, else the ``mN-1`` interior nodes of continuous P_m;
* continuous pressure only: one row per graph node that has an edge (ascending id) --
  the pressure value shared by every edge meeting there (``assembly.py:135-145``: the
  pressure space lives on the whole network mesh);
* one multiplier row per bifurcation (ascending node id).

Pressure rows and their rhs are negated, as in the P1 path, so the matrix is symmetric.

Several ranks (DG0 pressure, ``build_fe_rank_layout``): a rank holds the edges, owned
multipliers and ghost columns of its P1/DG0 rank layout (``layout.build_local_problem``) --
its local edges' rows, then its owned multipliers, then the ghost columns in the P1 layout's
order (the multipliers of cut bifurcations owned elsewhere and the remote flux ends its
multiplier rows read). The halo plan is the P1 rank layout's, renumbered.

Assembly tables: every nonzero and every rhs entry is a short sum of terms
``table_val[ent] x factor`` (factor ``R_e h_c``, ``f h_c``, ``edge_bc`` or 1; see
``include/nxhip.h`` ``nx_create_fe``). The terms are generated cell by cell from the
reference element tensors (:mod:`element`) and grouped per output in generation order,
so the device sums them in a fixed order (``k_assemble_fe``).
"""

from __future__ import annotations

from dataclasses import dataclass

import numpy as np

from .element import element_tensors, stable_pair

__all__ = ["FeLayout", "build_fe_layout", "build_fe_rank_layout", "build_fe_partition",
           "fe_global_rows", "fe_row_owner", "build_cp_rank_tables", "KIND_CONST", "KIND_MASS", "KIND_SOURCE", "KIND_BC"]

KIND_CONST, KIND_MASS, KIND_SOURCE, KIND_BC = 0, 1, 2, 3


@dataclass
class FeLayout:
    N: int
    k: int
    m: int
    E: int
    n_rows: int
    rowptr: np.ndarray  # int32 (n_rows+1,)
    col: np.ndarray  # int32 (nnz,)
    table_kind: np.ndarray  # int32
    table_val: np.ndarray  # f64
    a_ptr: np.ndarray  # int32 (nnz+1,)
    a_idx: np.ndarray  # int32
    a_ent: np.ndarray  # int32
    b_ptr: np.ndarray  # int32 (n_rows+1,)
    b_idx: np.ndarray  # int32
    b_ent: np.ndarray  # int32
    flux_rows: np.ndarray  # (E, kN+1) device rows of each edge's flux nodes
    p_rows: np.ndarray  # device row of every pressure DoF, in the function's order
    p_nodes: np.ndarray  # graph nodes carrying a pressure DoF (m >= 1)
    lm_nodes: np.ndarray  # bifurcations, ascending
    lm_rows: np.ndarray
    edge_x: np.ndarray  # (E, 6) source xyz, target xyz
    # several ranks (build_fe_rank_layout): the ghost columns after the owned rows, the
    # global edge id of every local edge, and the halo plan (nx_set_halo's arrays)
    n_ghost: int = 0
    edges: np.ndarray | None = None
    n_edges_global: int = 0
    peers: np.ndarray | None = None
    send_off: np.ndarray | None = None
    send_idx: np.ndarray | None = None
    recv_off: np.ndarray | None = None
    n_own_edges: int = -1  # build_fe_partition: edges [0, n_own_edges) own rows, the rest
    global_rows: np.ndarray | None = None  # are ghost edges (coefficients only)
    ghost_rows: np.ndarray | None = None

    @property
    def nnz(self) -> int:
        return int(self.col.size)


def _tables(k: int, m: int):
    """The term table (kinds, values) and its entry indices for the pair (k, m)."""
    Mref, Dref, wref = element_tensors(k, m)
    nq, npl = k + 1, wref.size
    ent = {"mass": np.arange(nq * nq).reshape(nq, nq),
           "b": nq * nq + np.arange(npl * nq).reshape(npl, nq)}
    ent["plus"] = nq * nq + npl * nq
    ent["minus"] = ent["plus"] + 1
    ent["src"] = ent["minus"] + 1 + np.arange(npl)
    ent["bc"] = int(ent["src"][-1]) + 1
    table_kind = np.concatenate([np.full(nq * nq, KIND_MASS), np.full(npl * nq, KIND_CONST),
                                 [KIND_CONST, KIND_CONST], np.full(npl, KIND_SOURCE),
                                 [KIND_BC]]).astype(np.int32)
    # negated pressure rows: divergence -Dref (row p, col q); gradient -Dref^T (row q, col p)
    table_val = np.concatenate([Mref.ravel(), -Dref.ravel(), [1.0, -1.0], -wref, [1.0]])
    return table_kind, table_val, ent, nq, npl


def _cell_terms(qrow, prow, cell, ent, nq, npl, E, N):
    """Every cell's mass and divergence / gradient terms, in generation order."""
    rows, cols, idx, ents = [], [], [], []
    for i in range(nq):
        for j in range(nq):
            rows.append(qrow[:, :, i]); cols.append(qrow[:, :, j])  # noqa: E702
            idx.append(cell); ents.append(np.full((E, N), ent["mass"][i, j]))  # noqa: E702
    for a in range(npl):
        for j in range(nq):
            rows.append(prow[:, :, a]); cols.append(qrow[:, :, j])  # noqa: E702
            idx.append(cell); ents.append(np.full((E, N), ent["b"][a, j]))  # noqa: E702
            rows.append(qrow[:, :, j]); cols.append(prow[:, :, a])  # noqa: E702
            idx.append(cell); ents.append(np.full((E, N), ent["b"][a, j]))  # noqa: E702
    return rows, cols, idx, ents


def _csr_and_rhs(rows, cols, idx, ents, br, bi, be, n_rows):
    """Terms grouped per (row, column) in generation order -> CSR pattern and term lists;
    rhs terms grouped per row."""
    R = np.concatenate([np.ravel(x) for x in rows])
    C = np.concatenate([np.ravel(x) for x in cols])
    Ix = np.concatenate([np.ravel(x) for x in idx])
    T = np.concatenate([np.ravel(x) for x in ents])
    order = np.lexsort((np.arange(R.size), C, R))  # by row, column, then generation order
    R, C, Ix, T = R[order], C[order], Ix[order], T[order]
    new = np.ones(R.size, dtype=bool)
    new[1:] = (R[1:] != R[:-1]) | (C[1:] != C[:-1])
    starts = np.flatnonzero(new)
    a_ptr = np.append(starts, R.size)
    col = C[starts]
    rowptr = np.zeros(n_rows + 1, dtype=np.int64)
    np.cumsum(np.bincount(R[starts], minlength=n_rows), out=rowptr[1:])
    BR = np.concatenate([np.ravel(x) for x in br])
    BI = np.concatenate([np.ravel(x) for x in bi])
    BE = np.concatenate([np.ravel(x) for x in be])
    border = np.argsort(BR, kind="stable")
    b_ptr = np.zeros(n_rows + 1, dtype=np.int64)
    np.cumsum(np.bincount(BR, minlength=n_rows), out=b_ptr[1:])
    if max(a_ptr[-1], rowptr[-1], n_rows) >= np.iinfo(np.int32).max:
        raise ValueError("problem too large for 32-bit CSR indices")
    return rowptr, col, a_ptr, Ix, T, b_ptr, BI[border], BE[border]


def build_fe_layout(pos: np.ndarray, src: np.ndarray, dst: np.ndarray, degree: np.ndarray,
                    N: int, k: int, m: int) -> FeLayout:
    """Layout and term tables for flux degree ``k`` and pressure degree ``m``."""
    if not stable_pair(k, m):
        raise ValueError(
            f"flux_degree={k}, pressure_degree={m}: continuous pressure needs a flux degree "
            "above the pressure degree, otherwise the system is singular")
    src = np.asarray(src, dtype=np.int64)
    dst = np.asarray(dst, dtype=np.int64)
    E = src.size
    n_nodes = pos.shape[0]
    nf = k * N + 1
    npe = N if m == 0 else m * N - 1
    per = nf + npe
    base = np.arange(E, dtype=np.int64) * per
    flux_rows = base[:, None] + np.arange(nf)[None, :]
    p_nodes = np.flatnonzero(degree > 0) if m >= 1 else np.zeros(0, dtype=np.int64)
    node_row = np.full(n_nodes, -1, dtype=np.int64)
    node_row[p_nodes] = E * per + np.arange(p_nodes.size)
    lm_nodes = np.flatnonzero(degree > 1)
    lm_row = np.full(n_nodes, -1, dtype=np.int64)
    lm_row[lm_nodes] = E * per + p_nodes.size + np.arange(lm_nodes.size)
    n_rows = E * per + p_nodes.size + lm_nodes.size

    c = np.arange(N)
    qrow = base[:, None, None] + (c[:, None] * k + np.arange(k + 1)[None, :])[None]  # (E,N,k+1)
    if m == 0:
        prow = (base[:, None] + nf + c[None, :])[:, :, None]  # (E,N,1)
    else:
        ppos = c[:, None] * m + np.arange(m + 1)[None, :]  # (N, m+1) positions 0..mN
        prow = np.broadcast_to(base[:, None, None] + nf + ppos[None] - 1, (E, N, m + 1)).copy()
        prow = np.where(ppos[None] == 0, node_row[src][:, None, None], prow)
        prow = np.where(ppos[None] == m * N, node_row[dst][:, None, None], prow)

    table_kind, table_val, ent, nq, npl = _tables(k, m)
    cell = np.arange(E, dtype=np.int64)[:, None] * N + c[None, :]  # (E, N)
    rows, cols, idx, ents = _cell_terms(qrow, prow, cell, ent, nq, npl, E, N)
    # junctions (assembly.py:268-277): +1 at in-edge ends, -1 at out-edge starts, both blocks
    e_in = np.flatnonzero(lm_row[dst] >= 0)
    e_out = np.flatnonzero(lm_row[src] >= 0)
    for e_set, lam, qr, en in ((e_in, lm_row[dst[e_in]], flux_rows[e_in, -1], ent["plus"]),
                               (e_out, lm_row[src[e_out]], flux_rows[e_out, 0], ent["minus"])):
        z = np.zeros(e_set.size, dtype=np.int64)
        rows += [lam, qr]; cols += [qr, lam]  # noqa: E702
        idx += [z, z]; ents += [np.full(e_set.size, en), np.full(e_set.size, en)]  # noqa: E702
    # rhs: source on pressure rows, boundary data at both flux ends of every edge
    e_ids = np.arange(E, dtype=np.int64)
    br = [prow[:, :, a] for a in range(npl)] + [flux_rows[:, 0], flux_rows[:, -1]]
    bi = [cell for _ in range(npl)] + [2 * e_ids, 2 * e_ids + 1]
    be = [np.full((E, N), ent["src"][a]) for a in range(npl)] + [np.full(E, ent["bc"])] * 2
    rowptr, col, a_ptr, Ix, T, b_ptr, BI, BE = _csr_and_rhs(rows, cols, idx, ents, br, bi, be,
                                                            n_rows)

    if m == 0:
        p_rows = (base[:, None] + nf + c[None, :]).ravel()
    else:
        p_rows = np.concatenate([node_row[p_nodes],
                                 (base[:, None] + nf + np.arange(m * N - 1)[None, :]).ravel()])
    pos3 = np.zeros((n_nodes, 3))
    pos3[:, : pos.shape[1]] = pos
    edge_x = np.concatenate([pos3[src], pos3[dst]], axis=1)
    i32 = lambda a: np.ascontiguousarray(a, dtype=np.int32)  # noqa: E731
    return FeLayout(N, k, m, E, int(n_rows), i32(rowptr), i32(col), table_kind,
                    np.ascontiguousarray(table_val), i32(a_ptr), i32(Ix), i32(T), i32(b_ptr),
                    i32(BI), i32(BE), flux_rows, p_rows, p_nodes, lm_nodes,
                    lm_row[lm_nodes], edge_x, n_edges_global=E)


def build_fe_rank_layout(pos: np.ndarray, src: np.ndarray, dst: np.ndarray, N: int, k: int,
                         lp) -> FeLayout:
    """One rank's (k, 0) layout over the edges, owned multipliers and ghost columns of its
    P1/DG0 rank layout ``lp`` (``layout.build_local_problem``, several ranks). Its rows are
    the one-rank layout's rows of those edges and multipliers (``fe_global_rows``): the same
    terms, the remote flux ends of an owned multiplier row as ghost columns."""
    m = 0
    src = np.asarray(src, dtype=np.int64)
    dst = np.asarray(dst, dtype=np.int64)
    edges = np.asarray(lp.edges, dtype=np.int64)
    E = edges.size
    nf, npe = k * N + 1, N
    per = nf + npe
    per1 = 2 * N + 1
    n_lm = int(np.asarray(lp.lm_nodes).size)
    n_own = E * per + n_lm
    n_own1 = int(lp.n_own)
    n_edge1 = E * per1
    base = np.arange(E, dtype=np.int64) * per
    flux_rows = base[:, None] + np.arange(nf)[None, :]

    def col_of(c1):  # P1 rank column -> this layout's column
        c1 = np.asarray(c1, dtype=np.int64)
        s, j = np.divmod(np.minimum(c1, n_edge1 - 1) if E else c1 * 0, per1)
        edge_col = s * per + np.where(j == 0, 0, nf - 1)
        return np.where(c1 >= n_own1, n_own + (c1 - n_own1),
                        np.where(c1 >= n_edge1, E * per + (c1 - n_edge1), edge_col))

    c = np.arange(N)
    qrow = base[:, None, None] + (c[:, None] * k + np.arange(k + 1)[None, :])[None]
    prow = (base[:, None] + nf + c[None, :])[:, :, None]
    table_kind, table_val, ent, nq, npl = _tables(k, m)
    cell = np.arange(E, dtype=np.int64)[:, None] * N + c[None, :]
    rows, cols, idx, ents = _cell_terms(qrow, prow, cell, ent, nq, npl, E, N)
    # flux end rows -> their multiplier (owned row or ghost column): lp.edge_lm
    elm = np.asarray(lp.edge_lm, dtype=np.int64).reshape(E, 2)
    for end, en in ((0, ent["minus"]), (1, ent["plus"])):
        on = np.flatnonzero(elm[:, end] >= 0)
        rows.append(flux_rows[on, 0 if end == 0 else -1])
        cols.append(col_of(elm[on, end]))
        idx.append(np.zeros(on.size, dtype=np.int64))
        ents.append(np.full(on.size, en))
    # owned multiplier rows -> every incident flux end (local or ghost): lp's rows
    lrp = np.asarray(lp.lm_rowptr, dtype=np.int64)
    lcol = np.asarray(lp.lm_col, dtype=np.int64)
    lval = np.asarray(lp.lm_val, dtype=np.float64)
    lrow = np.repeat(np.arange(n_lm), np.diff(lrp))
    rows.append(E * per + lrow)
    cols.append(col_of(lcol))
    idx.append(np.zeros(lcol.size, dtype=np.int64))
    ents.append(np.where(lval > 0, ent["plus"], ent["minus"]))
    e_ids = np.arange(E, dtype=np.int64)
    br = [prow[:, :, 0], flux_rows[:, 0], flux_rows[:, -1]]
    bi = [cell, 2 * e_ids, 2 * e_ids + 1]
    be = [np.full((E, N), ent["src"][0]), np.full(E, ent["bc"]), np.full(E, ent["bc"])]
    rowptr, col, a_ptr, Ix, T, b_ptr, BI, BE = _csr_and_rhs(rows, cols, idx, ents, br, bi, be,
                                                            n_own)
    n_nodes = pos.shape[0]
    pos3 = np.zeros((n_nodes, 3))
    pos3[:, : pos.shape[1]] = pos
    edge_x = np.concatenate([pos3[src[edges]], pos3[dst[edges]]], axis=1)
    i32 = lambda a: np.ascontiguousarray(a, dtype=np.int32)  # noqa: E731
    lay = FeLayout(N, k, m, E, int(n_own), i32(rowptr), i32(col), table_kind,
                   np.ascontiguousarray(table_val), i32(a_ptr), i32(Ix), i32(T), i32(b_ptr),
                   i32(BI), i32(BE), flux_rows, (base[:, None] + nf + c[None, :]).ravel(),
                   np.zeros(0, dtype=np.int64), np.asarray(lp.lm_nodes, dtype=np.int64),
                   E * per + np.arange(n_lm, dtype=np.int64), edge_x)
    lay.n_ghost = int(lp.n_ghost)
    lay.edges = edges
    lay.n_edges_global = int(src.size)
    lay.peers = i32(lp.peers)
    lay.send_off = i32(lp.send_off)
    lay.send_idx = i32(col_of(np.asarray(lp.send_idx, dtype=np.int64)))
    lay.recv_off = i32(lp.recv_off)
    return lay


def fe_row_owner(lay: FeLayout, src: np.ndarray, dst: np.ndarray, edge_owner: np.ndarray,
                 n_nodes: int) -> np.ndarray:
    """Owning rank of every row of a one-rank layout: an edge's rows go with the edge, a
    node's shared pressure row and a bifurcation's multiplier row with the node's first
    in-edge, else its first out-edge (``layout.build_local_problem``'s rule)."""
    src = np.asarray(src, dtype=np.int64)
    dst = np.asarray(dst, dtype=np.int64)
    E = src.size
    per = lay.k * lay.N + 1 + (lay.N if lay.m == 0 else lay.m * lay.N - 1)
    first_in = np.full(n_nodes, E, dtype=np.int64)
    np.minimum.at(first_in, dst, np.arange(E))
    first_out = np.full(n_nodes, E, dtype=np.int64)
    np.minimum.at(first_out, src, np.arange(E))
    anchor = np.where(first_in < E, first_in, first_out)
    own = np.empty(lay.n_rows, dtype=np.int32)
    own[: E * per] = np.repeat(np.asarray(edge_owner, dtype=np.int32), per)
    pn = np.asarray(lay.p_nodes, dtype=np.int64)
    own[E * per: E * per + pn.size] = edge_owner[anchor[pn]]
    own[np.asarray(lay.lm_rows, dtype=np.int64)] = edge_owner[anchor[np.asarray(lay.lm_nodes)]]
    return own


def build_fe_partition(full: FeLayout, src: np.ndarray, dst: np.ndarray,
                       edge_owner: np.ndarray, rank: int, nranks: int) -> FeLayout:
    """One rank's part of a one-rank layout ``full`` by row ownership (``fe_row_owner``),
    for any pair -- continuous pressure's shared node rows included. The rank's rows are
    its owned rows in the one-rank order (its edges' rows, its node pressure rows, its
    multipliers); every other column it reads is a ghost, ordered by owner, then by the
    owner's local index, so the owner's send list and the ghost slots line up. Its edges
    are its own (ascending) then the ghost edges whose cells its rows' terms read (a shared
    node row sums the element terms of every edge at the node): coefficients and cell
    lengths cover both, rows only the owned."""
    src = np.asarray(src, dtype=np.int64)
    dst = np.asarray(dst, dtype=np.int64)
    E, N = src.size, full.N
    per = full.k * N + 1 + (N if full.m == 0 else full.m * N - 1)
    owner_e = np.asarray(edge_owner, dtype=np.int32)
    n_nodes = int(max(src.max(), dst.max())) + 1 if E else 0
    n_nodes = max(n_nodes, int(np.max(full.p_nodes, initial=-1)) + 1,
                  int(np.max(full.lm_nodes, initial=-1)) + 1)
    row_own = fe_row_owner(full, src, dst, owner_e, n_nodes)
    rows_of = [np.flatnonzero(row_own == q) for q in range(nranks)]
    loc = np.empty(full.n_rows, dtype=np.int64)  # local index on the owning rank
    for q in range(nranks):
        loc[rows_of[q]] = np.arange(rows_of[q].size)
    mine = rows_of[rank]
    n_own = mine.size
    rp = np.asarray(full.rowptr, dtype=np.int64)
    starts, ends = rp[mine], rp[mine + 1]
    cnt = ends - starts
    ent_idx = (np.repeat(starts - np.cumsum(np.concatenate([[0], cnt[:-1]])), cnt)
               + np.arange(int(cnt.sum())))  # the owned rows' entries, in order
    gcol = np.asarray(full.col, dtype=np.int64)[ent_idx]

    def ghosts_of(q):
        rq = rows_of[q]
        s_, e_ = rp[rq], rp[rq + 1]
        c_ = e_ - s_
        ix = np.repeat(s_ - np.cumsum(np.concatenate([[0], c_[:-1]])), c_) + np.arange(int(c_.sum()))
        cq = np.unique(np.asarray(full.col, dtype=np.int64)[ix])
        cq = cq[row_own[cq] != q]
        return cq[np.lexsort((loc[cq], row_own[cq]))]

    gh = ghosts_of(rank)
    col_local = np.empty(full.n_rows, dtype=np.int64)
    col_local[mine] = np.arange(n_own)
    col_local[gh] = n_own + np.arange(gh.size)
    col = col_local[gcol]
    o = np.lexsort((col, np.repeat(np.arange(n_own), cnt)))  # rows keep sorted local columns
    ent_idx, col = ent_idx[o], col[o]
    # terms of the owned entries and rhs rows; the cells / edges they read
    kind = np.asarray(full.table_kind)
    ap = np.asarray(full.a_ptr, dtype=np.int64)
    t0, t1 = ap[ent_idx], ap[ent_idx + 1]
    tcnt = t1 - t0
    tix = np.repeat(t0 - np.cumsum(np.concatenate([[0], tcnt[:-1]])), tcnt) + np.arange(int(tcnt.sum()))
    a_idx = np.asarray(full.a_idx, dtype=np.int64)[tix]
    a_ent = np.asarray(full.a_ent, dtype=np.int64)[tix]
    bp = np.asarray(full.b_ptr, dtype=np.int64)
    b0, b1 = bp[mine], bp[mine + 1]
    bcnt = b1 - b0
    bix = np.repeat(b0 - np.cumsum(np.concatenate([[0], bcnt[:-1]])), bcnt) + np.arange(int(bcnt.sum()))
    b_idx = np.asarray(full.b_idx, dtype=np.int64)[bix]
    b_ent = np.asarray(full.b_ent, dtype=np.int64)[bix]
    # a term's idx is a cell for the mass / source kinds and for the divergence entries (the
    # constants before the junctions' +-1, kept as their cell: _cell_terms), else 0 / 2e+end
    ent_junction = (full.k + 1) ** 2 + (1 if full.m == 0 else full.m + 1) * (full.k + 1)
    a_cell = np.isin(kind[a_ent], [KIND_MASS, KIND_SOURCE]) | (
        (kind[a_ent] == KIND_CONST) & (a_ent < ent_junction))
    b_cell = np.isin(kind[b_ent], [KIND_MASS, KIND_SOURCE])
    b_bc = kind[b_ent] == KIND_BC
    own_e = np.flatnonzero(owner_e == rank)
    read_e = np.unique(np.concatenate([a_idx[a_cell] // N, b_idx[b_cell] // N, b_idx[b_bc] // 2]))
    ghost_e = np.setdiff1d(read_e, own_e)
    edges = np.concatenate([own_e, ghost_e])
    e_loc = np.full(E, -1, dtype=np.int64)
    e_loc[edges] = np.arange(edges.size)
    a_idx[a_cell] = e_loc[a_idx[a_cell] // N] * N + a_idx[a_cell] % N
    b_new = b_idx.copy()
    b_new[b_cell] = e_loc[b_idx[b_cell] // N] * N + b_idx[b_cell] % N
    b_new[b_bc] = 2 * e_loc[b_idx[b_bc] // 2] + b_idx[b_bc] % 2
    b_idx = b_new
    rowptr = np.concatenate([[0], np.cumsum(cnt)])
    a_ptr = np.concatenate([[0], np.cumsum(tcnt)])
    b_ptr = np.concatenate([[0], np.cumsum(bcnt)])
    # the function rows: owned edges' flux rows, pressure in the function's order, multipliers
    flux_rows = col_local[np.asarray(full.flux_rows)[own_e]]
    p_sel = np.asarray(full.p_rows, dtype=np.int64)
    p_rows = col_local[p_sel[row_own[p_sel] == rank]]
    pn = np.asarray(full.p_nodes, dtype=np.int64)
    pn_rows = E * per + np.arange(pn.size)
    lmr = np.asarray(full.lm_rows, dtype=np.int64)
    lm_mine = row_own[lmr] == rank
    # halo plan: what each peer reads of mine, in its ghost order
    peers, send_off, send_idx, recv_off = [], [0], [], [0]
    g_owner = row_own[gh]
    for q in range(nranks):
        if q == rank:
            continue
        theirs = ghosts_of(q)
        snd = loc[theirs[row_own[theirs] == rank]]
        rcv = int(np.count_nonzero(g_owner == q))
        if snd.size == 0 and rcv == 0:
            continue
        peers.append(q)
        send_idx.extend(snd.tolist())
        send_off.append(len(send_idx))
        recv_off.append(recv_off[-1] + rcv)
    i32 = lambda a: np.ascontiguousarray(a, dtype=np.int32)  # noqa: E731
    lay = FeLayout(N, full.k, full.m, int(edges.size), int(n_own), i32(rowptr), i32(col),
                   full.table_kind, full.table_val, i32(a_ptr), i32(a_idx), i32(a_ent),
                   i32(b_ptr), i32(b_idx), i32(b_ent), flux_rows, p_rows,
                   pn[row_own[pn_rows] == rank], np.asarray(full.lm_nodes)[lm_mine],
                   col_local[lmr[lm_mine]], np.asarray(full.edge_x)[edges])
    lay.n_ghost = int(gh.size)
    lay.edges = edges
    lay.n_edges_global = E
    lay.n_own_edges = int(own_e.size)
    lay.global_rows = mine
    lay.ghost_rows = gh
    lay.peers = i32(peers)
    lay.send_off = i32(send_off)
    lay.send_idx = i32(send_idx)
    lay.recv_off = i32(recv_off)
    return lay


def fe_global_rows(lay: FeLayout, degree: np.ndarray) -> np.ndarray:
    """The one-rank layout row (``build_fe_layout`` of the whole graph) of every owned row of
    a rank layout: edge rows by global edge, multipliers by bifurcation rank (DG0)."""
    if getattr(lay, "global_rows", None) is not None:  # build_fe_partition keeps them
        return np.asarray(lay.global_rows, dtype=np.int64)
    per = lay.k * lay.N + 1 + lay.N
    edges = np.arange(lay.E) if lay.edges is None else np.asarray(lay.edges, dtype=np.int64)
    bif = np.flatnonzero(np.asarray(degree) > 1)
    lam = lay.n_edges_global * per + np.searchsorted(bif, np.asarray(lay.lm_nodes, np.int64))
    return np.concatenate([(edges[:, None] * per + np.arange(per)[None, :]).ravel(), lam])


def evaluate_terms(lay: FeLayout, R_edge: np.ndarray, f, edge_bc: np.ndarray,
                   cell_h: np.ndarray):
    """Host evaluation of the term tables (what ``k_assemble_fe`` computes), for tests and
    debugging: returns ``(val, rhs)``. ``cell_h`` is ``(E, N)``; ``f`` a constant or one value
    per edge."""
    h = np.asarray(cell_h, dtype=np.float64).ravel()
    Rc = np.repeat(np.asarray(R_edge, dtype=np.float64), lay.N)
    fc = np.repeat(np.broadcast_to(np.asarray(f, dtype=np.float64), (lay.E,)), lay.N)
    bc = np.asarray(edge_bc, dtype=np.float64).ravel()

    def term(i, e):
        kind, v = lay.table_kind[e], lay.table_val[e]
        if kind == KIND_MASS:
            return (Rc[i] * h[i]) * v
        if kind == KIND_SOURCE:
            return (fc[i] * h[i]) * v
        if kind == KIND_BC:
            return bc[i] * v
        return v

    kind = lay.table_kind[lay.a_ent]
    v = lay.table_val[lay.a_ent]
    tv = np.where(kind == KIND_MASS, (Rc[np.where(kind == KIND_MASS, lay.a_idx, 0)]
                                      * h[np.where(kind == KIND_MASS, lay.a_idx, 0)]) * v, v)
    val = np.add.reduceat(tv, lay.a_ptr[:-1]) if tv.size else np.zeros(0)
    rhs = np.zeros(lay.n_rows)
    for r in range(lay.n_rows):
        s = 0.0
        for t in range(lay.b_ptr[r], lay.b_ptr[r + 1]):
            s += term(lay.b_idx[t], lay.b_ent[t])
        rhs[r] = s
    return val, rhs


@dataclass
class FeAuxMaps:
    """Rows of the P1/DG0-structured system that the flux-degree-k / DG0 system condenses to
    (``nx_fe_set_direct``): per FE cell-vertex flux, pressure cell and multiplier, the row of
    the auxiliary P1 handle built from ``layout.build_local_problem`` of the same graph."""

    v_fe: np.ndarray  # (E (N+1),) FE rows of the vertex fluxes, edge-major (graph order)
    v_aux: np.ndarray  # their rows in the auxiliary system
    i_fe: np.ndarray  # (E N (k-1),) FE rows of the interior fluxes, cell-major
    p_fe: np.ndarray  # (E N,) FE pressure rows, edge-major
    p_aux: np.ndarray
    l_fe: np.ndarray  # (B,) FE multiplier rows, ascending node
    l_aux: np.ndarray


def fe_aux_slots(lay: FeLayout, lp) -> np.ndarray:
    """The auxiliary P1 handle's slot of every edge of the layout (its local order)."""
    ge = np.arange(lay.E) if lay.edges is None else np.asarray(lay.edges, dtype=np.int64)
    full = np.full(max(lay.n_edges_global, lay.E), -1, dtype=np.int64)
    full[np.asarray(lp.edges, dtype=np.int64)] = np.arange(np.asarray(lp.edges).size)
    slot = full[ge]
    if (slot < 0).any() or np.asarray(lp.edges).size != lay.E:
        raise ValueError("the auxiliary problem must hold the layout's edges")
    return slot


def build_fe_aux_maps(lay: FeLayout, lp) -> FeAuxMaps:
    """Row maps between a (k, 0) layout and the P1 local problem ``lp`` of the same edges
    (one rank: the whole graph; several: the rank's P1 layout that ``build_fe_rank_layout``
    followed) -- its edge slots ``lp.edges`` in its own order, multipliers by ascending node."""
    if lay.m != 0:
        raise ValueError("the condensed direct solve is DG0's (pressure_degree 0)")
    E, N, k = lay.E, lay.N, lay.k
    slot = fe_aux_slots(lay, lp)
    per1 = 2 * N + 1
    g = np.arange(N + 1)
    v_fe = lay.flux_rows[:, k * g].ravel()
    v_aux = (slot[:, None] * per1 + 2 * g[None, :]).ravel()
    c = np.arange(N)
    i_fe = (lay.flux_rows[:, (k * c)[:, None] + np.arange(1, k)[None, :]]).ravel()
    p_fe = lay.p_rows.astype(np.int64)
    p_aux = (slot[:, None] * per1 + 2 * c[None, :] + 1).ravel()
    lm1 = np.asarray(lp.lm_nodes, dtype=np.int64)
    pos = np.searchsorted(lm1, lay.lm_nodes)
    if not np.array_equal(lm1[np.minimum(pos, lm1.size - 1)], lay.lm_nodes):
        raise ValueError("multiplier nodes differ")
    l_aux = lp.n_edge_dofs + pos
    i32 = lambda a: np.ascontiguousarray(a, dtype=np.int32)  # noqa: E731
    return FeAuxMaps(i32(v_fe), i32(v_aux), i32(i_fe), i32(p_fe), i32(p_aux),
                     i32(lay.lm_rows), i32(l_aux))


@dataclass
class CpTables:
    """The continuous-pressure direct solve's tables (``nx_fe_set_cp``, include/nxhip.h):
    reference blocks, border nodes (every graph node with an edge), per edge its end nodes
    and multiplier couplings, and the node forest in level order."""

    k: int
    m: int
    nI: int
    cst: np.ndarray  # Kh | Ch | Eh | Fh
    tI: np.ndarray
    n_nodes: int
    nrow: np.ndarray  # (n, 2) pressure row, multiplier row or -1
    eb: np.ndarray  # (E, 4) source node, target node, q_0 - lam_src, q_N - lam_dst couplings
    lev_off: np.ndarray
    order: np.ndarray
    inc_off: np.ndarray
    inc: np.ndarray  # (n_inc, 2) edge, end (0 source, 1 target)
    parent: np.ndarray  # (n, 3) parent node, edge, this node's end of it (-1 at a root)
    child_off: np.ndarray
    child: np.ndarray
    nown: np.ndarray  # the edge that writes each node's rows


def build_cp_tables(lay: FeLayout, src: np.ndarray, dst: np.ndarray) -> CpTables | None:
    """Tables of the node-condensed direct solve for continuous pressure (``lay.m >= 1``), or
    ``None`` when the graph is not a forest (a cycle: MINRES)."""
    from collections import deque

    from .element import condensed_cell_blocks

    if lay.m < 1:
        raise ValueError("the node-condensed solve is continuous pressure's (m >= 1)")
    src = np.asarray(src, dtype=np.int64)
    dst = np.asarray(dst, dtype=np.int64)
    E = lay.E
    nodes = np.asarray(lay.p_nodes, dtype=np.int64)
    n = nodes.size
    idx = np.full(int(max(src.max(), dst.max())) + 1 if E else 0, -1, dtype=np.int64)
    idx[nodes] = np.arange(n)
    u, v = idx[src], idx[dst]
    per = lay.k * lay.N + 1 + lay.m * lay.N - 1
    lam = np.full(idx.size, -1, dtype=np.int64)
    lam[np.asarray(lay.lm_nodes, dtype=np.int64)] = np.asarray(lay.lm_rows, dtype=np.int64)
    nrow = np.stack([E * per + np.arange(n), lam[nodes]], axis=1)
    eb = np.stack([u, v, np.where(lam[src] >= 0, -1, 0), np.where(lam[dst] >= 0, 1, 0)], axis=1)
    # incidence (edge, end), by node then edge
    ne = np.concatenate([u, v])
    ee = np.concatenate([np.arange(E), np.arange(E)])
    en = np.concatenate([np.zeros(E, np.int64), np.ones(E, np.int64)])
    o = np.lexsort((ee, ne))
    inc = np.stack([ee[o], en[o]], axis=1)
    inc_off = np.zeros(n + 1, dtype=np.int64)
    np.cumsum(np.bincount(ne, minlength=n), out=inc_off[1:])
    # BFS forest from the lowest node of every component
    parent = np.full((n, 3), -1, dtype=np.int64)
    level = np.full(n, -1, dtype=np.int64)
    for r in range(n):
        if level[r] >= 0:
            continue
        level[r] = 0
        dq = deque([r])
        while dq:
            a = dq.popleft()
            for j in range(inc_off[a], inc_off[a + 1]):
                e, end = inc[j]
                b = v[e] if end == 0 else u[e]
                if b == a or (parent[a, 1] == e):
                    continue
                if level[b] >= 0:
                    return None  # a cycle
                level[b] = level[a] + 1
                parent[b] = (a, e, 1 - end)
                dq.append(b)
    order = np.lexsort((np.arange(n), level))
    nlev = int(level.max()) + 1 if n else 1
    lev_off = np.zeros(nlev + 1, dtype=np.int64)
    np.cumsum(np.bincount(level, minlength=nlev), out=lev_off[1:])
    has = parent[:, 0] >= 0
    ch_par = parent[has, 0]
    ch = np.flatnonzero(has)
    oc = np.lexsort((ch, ch_par))
    child = ch[oc]
    child_off = np.zeros(n + 1, dtype=np.int64)
    np.cumsum(np.bincount(ch_par, minlength=n), out=child_off[1:])
    nown = inc[inc_off[:-1], 0]
    Kh, Ch, Eh, Fh, tI = condensed_cell_blocks(lay.k, lay.m)
    cst = np.concatenate([Kh.ravel(), Ch.ravel(), Eh.ravel(), Fh.ravel()])
    i32 = lambda a: np.ascontiguousarray(a, dtype=np.int32).ravel()  # noqa: E731
    return CpTables(lay.k, lay.m, int(tI.size), cst, i32(tI), int(n), i32(nrow), i32(eb),
                    i32(lev_off), i32(order), i32(inc_off), i32(inc), i32(parent),
                    i32(child_off), i32(child), i32(nown))


def build_cp_rank_tables(tab: CpTables, part: FeLayout):
    """One rank's share of the node-condensed solve (``nx_fe_cp_ranks`` + ``nx_fe_set_cp``)
    from the one-rank tables ``tab`` and the rank's partition ``part``
    (``build_fe_partition``): ``(tab_rank, gid, nrowx)``. The rank's edges run the edge
    kernels (``eb`` of its own edges; ``gid`` their global ids); the node tables keep global
    nodes and edges, every rank solving the whole node forest over the summed blocks; ``nrow``
    names the summed node rhs (2n, 2n + 1 or -1); ``nrowx`` the local rows of the node rows
    this rank owns, and ``nown`` the local edge that writes them (-1 elsewhere)."""
    from dataclasses import replace

    own_e = np.asarray(part.edges, dtype=np.int64)[: part.n_own_edges]
    n = tab.n_nodes
    nrow_g = np.asarray(tab.nrow, dtype=np.int64).reshape(n, 2)
    grows = np.asarray(part.global_rows, dtype=np.int64)

    def local(rows):
        i = np.searchsorted(grows, rows)
        i = np.minimum(i, max(grows.size - 1, 0))
        hit = (rows >= 0) & (grows.size > 0) & (grows[i] == rows)
        return np.where(hit, i, -1)

    nrowx = np.stack([local(nrow_g[:, 0]), local(nrow_g[:, 1])], axis=1)
    nrow_nb = np.stack([2 * np.arange(n), np.where(nrow_g[:, 1] >= 0, 2 * np.arange(n) + 1, -1)],
                       axis=1)
    # the node rows' writer: the node's anchor edge when this rank owns the rows (the anchor
    # is then one of its own edges)
    e_loc = np.full(part.n_edges_global, -1, dtype=np.int64)
    e_loc[own_e] = np.arange(own_e.size)
    src_e = np.asarray(tab.eb, dtype=np.int64).reshape(-1, 4)
    # one-rank writer (nown) is any incident edge; take the owned one: the first incident
    # edge of the node that is local
    inc = np.asarray(tab.inc, dtype=np.int64).reshape(-1, 2)
    off = np.asarray(tab.inc_off, dtype=np.int64)
    nown = np.full(n, -1, dtype=np.int64)
    for nd in np.flatnonzero(nrowx[:, 0] >= 0):
        loc_edges = e_loc[inc[off[nd]:off[nd + 1], 0]]
        loc_edges = loc_edges[loc_edges >= 0]
        nown[nd] = loc_edges[0]
    i32 = lambda a: np.ascontiguousarray(a, dtype=np.int32).ravel()  # noqa: E731
    tab_r = replace(tab, nrow=i32(nrow_nb), eb=i32(src_e[own_e]), nown=i32(nown))
    return tab_r, i32(own_e), i32(nrowx)


def cp_model(lay: FeLayout, tab: CpTables, val: np.ndarray, b: np.ndarray, R: np.ndarray,
             cell_h: np.ndarray) -> np.ndarray:
    """numpy restatement of the device's node-condensed solve (k_cp_edge, k_cp_nodes,
    k_cp_back) for tests: ``x`` of the (k, m) system with values ``val`` and rhs ``b``."""
    import scipy.sparse as sp

    A = sp.csr_matrix((val, lay.col, lay.rowptr), shape=(lay.n_rows, lay.n_rows))
    N, k, m, nI, E = lay.N, lay.k, lay.m, tab.nI, lay.E
    nf = k * N + 1
    per = nf + m * N - 1
    Kh = tab.cst[:16].reshape(4, 4)
    Ch = tab.cst[16:16 + 4 * nI].reshape(4, nI)
    Eh = tab.cst[16 + 4 * nI:16 + 8 * nI].reshape(nI, 4)
    Fh = tab.cst[16 + 8 * nI:].reshape(nI, nI)
    tI = tab.tI.astype(np.int64)
    tV = np.array([1, -1, 1, -1])
    eb = tab.eb.reshape(-1, 4)
    nrow = tab.nrow.reshape(-1, 2)
    h = np.asarray(cell_h).reshape(E, N)
    x = np.zeros(lay.n_rows)
    Se, ge, facs = np.zeros((E, 4, 4)), np.zeros((E, 4)), []
    for e in range(E):
        base = e * per
        prow = lambda j: base + nf + j - 1  # noqa: E731
        irow = lambda c, i: base + c * k + 1 + i if tI[i] > 0 else prow(c * m + 1 + i - (k - 1))  # noqa: E731
        P = np.array([[0.0, 0.0], [0.0, 1.0]])
        W = np.zeros((2, 4))
        W[0, 1] = eb[e, 2]
        rho = np.array([b[base], 0.0])
        Sb, gb, fe = np.zeros((4, 4)), np.zeros(4), []
        for c in range(N):
            s = R[e] * h[e, c]
            K = Kh * s ** ((tV[:, None] + tV[None, :]) // 2)
            bI = np.array([b[irow(c, i)] for i in range(nI)])
            rV = -(Ch * s ** ((tV[:, None] - tI[None, :]) // 2)) @ bI if nI else np.zeros(4)
            Wn = np.zeros((2, 4))
            if c == 0:
                P[0, 0] += K[0, 0]; W[0, 0] += K[0, 1]; Sb[0, 0] += K[1, 1]  # noqa: E702
                rho[0] += rV[0]; gb[0] += rV[1]  # noqa: E702
                C = np.array([[K[0, 2], K[0, 3]], [0.0, 0.0]])
                Wn[0, 0], Wn[1, 0] = K[2, 1], K[3, 1]
            else:
                P += K[:2, :2]; rho += rV[:2]  # noqa: E702
                C = K[:2, 2:].copy()
            if c + 1 < N:
                Pn = K[2:, 2:].copy()
                rn = rV[2:] + np.array([b[base + k * (c + 1)], b[prow(m * (c + 1))]])
            else:
                Sb[2, 2] += K[3, 3]; gb[2] += rV[3]  # noqa: E702
                if c == 0:
                    Sb[0, 2] += K[1, 3]; Sb[2, 0] += K[3, 1]  # noqa: E702
                Wn[0, 2] += K[2, 3]; Wn[0, 3] = eb[e, 3]; Wn[1, 0] = 0.0  # noqa: E702
                W[:, 2] += C[:, 1]; C[:, 1] = 0.0  # noqa: E702
                Pn = np.array([[K[2, 2], 0.0], [0.0, 1.0]])
                rn = np.array([rV[2] + b[base + nf - 1], 0.0])
            Pi = np.linalg.inv(P)
            Pn -= C.T @ Pi @ C; Wn -= C.T @ Pi @ W; rn -= C.T @ Pi @ rho  # noqa: E702
            Sb -= W.T @ Pi @ W; gb -= W.T @ Pi @ rho  # noqa: E702
            fe.append((Pi, C, W, rho))
            P, W, rho = Pn, Wn, rn
        Pi = np.linalg.inv(P)
        Sb -= W.T @ Pi @ W; gb -= W.T @ Pi @ rho  # noqa: E702
        fe.append((Pi, np.zeros((2, 2)), W, rho))
        Se[e], ge[e] = Sb, gb
        facs.append(fe)
    n = tab.n_nodes
    inc = tab.inc.reshape(-1, 2)
    par = tab.parent.reshape(-1, 3)
    Pinv, hv, xn = np.zeros((n, 2, 2)), np.zeros((n, 2)), np.zeros((n, 2))
    blk = lambda e, ra, cb: Se[e][2 * ra:2 * ra + 2, 2 * cb:2 * cb + 2]  # noqa: E731
    lev = tab.lev_off
    for L in range(lev.size - 2, -1, -1):
        for i in range(lev[L], lev[L + 1]):
            nd = tab.order[i]
            D = np.zeros((2, 2))
            g = np.array([b[nrow[nd, 0]], b[nrow[nd, 1]] if nrow[nd, 1] >= 0 else 0.0])
            for j in range(tab.inc_off[nd], tab.inc_off[nd + 1]):
                e, end = inc[j]
                D += blk(e, end, end)
                g += ge[e][2 * end:2 * end + 2]
            if nrow[nd, 1] < 0:
                D[1, 1] = 1.0
            for j in range(tab.child_off[nd], tab.child_off[nd + 1]):
                c = tab.child[j]
                B = blk(par[c, 1], par[c, 2], 1 - par[c, 2])
                D -= B.T @ Pinv[c] @ B
                g -= B.T @ Pinv[c] @ hv[c]
            Pinv[nd], hv[nd] = np.linalg.inv(D), g
    for L in range(lev.size - 1):
        for i in range(lev[L], lev[L + 1]):
            nd = tab.order[i]
            r = hv[nd].copy()
            if par[nd, 0] >= 0:
                r -= blk(par[nd, 1], par[nd, 2], 1 - par[nd, 2]) @ xn[par[nd, 0]]
            xn[nd] = Pinv[nd] @ r
    for nd in range(n):
        x[nrow[nd, 0]] = xn[nd, 0]
        if nrow[nd, 1] >= 0:
            x[nrow[nd, 1]] = xn[nd, 1]
    for e in range(E):
        base = e * per
        prow = lambda j: base + nf + j - 1  # noqa: E731
        xb = np.concatenate([xn[eb[e, 0]], xn[eb[e, 1]]])
        yn = np.zeros(2)
        for i in range(N, -1, -1):
            Pi, C, W, rho = facs[e][i]
            y = Pi @ (rho - C @ yn - W @ xb)
            x[base + k * i] = y[0]
            if 0 < i < N:
                x[prow(m * i)] = y[1]
            if i < N:
                s = R[e] * h[e, i]
                xv = np.array([y[0], xb[0] if i == 0 else y[1], yn[0], xb[2] if i + 1 == N else yn[1]])
                bI = np.array([b[base + i * k + 1 + j] if tI[j] > 0
                               else b[prow(i * m + 1 + j - (k - 1))] for j in range(nI)])
                xI = (Fh * s ** (-(tI[:, None] + tI[None, :]) // 2)) @ bI \
                    - (Eh * s ** ((-tI[:, None] + tV[None, :]) // 2)) @ xv if nI else []
                for j in range(nI):
                    r = base + i * k + 1 + j if tI[j] > 0 else prow(i * m + 1 + j - (k - 1))
                    x[r] = xI[j]
            yn = y
    del A
    return x
