"""DoF layout, edge partitioning and halo plans (host side).

The reference's DoF layout is DOLFINx's: one P1 flux space per edge colour, one DG0
pressure space and one DG0 multiplier space on the bifurcation point cloud
(``assembly.py:121-162``), distributed by the DOLFINx graph partitioner
(``mesh.py:331-348``). Here the layout is designed for the device instead:

* every graph edge owns ``2N+1`` consecutive DoFs, interleaved
  ``[q_0, p_0, q_1, p_1, ..., p_{N-1}, q_N]`` (flux vertices / pressure cells,
  source -> target);
* one multiplier per bifurcation follows the rank's edge DoFs (ascending node id);
* with ``P`` ranks the edges are partitioned in depth-first preorder from the root(s)
  into ``P`` contiguous, equally sized chunks -- for trees these are unions of whole
  subtrees, so only a handful of bifurcations are cut;
* a bifurcation's multiplier row lives with its first in-edge (else first out-edge);
* ghost columns are the values another rank owns: the multiplier of a cut
  bifurcation (read by a flux end row) and flux end values of remote edges (read by a
  multiplier row). They are grouped by owning rank and ordered by the owner's local
  index, so the owner's send list and the receiver's ghost slots line up.

Every rank holds the full graph (broadcast by ``NetworkMesh``), so every rank derives
every other rank's plan locally -- no communication is needed to build the halo.
"""

from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np

__all__ = ["LocalProblem", "dfs_edge_order", "partition_edges", "build_local_problem",
           "global_row_ids", "team_cycle_tables"]


def dfs_edge_order(src: np.ndarray, dst: np.ndarray, n_nodes: int) -> np.ndarray:
    """Iterative DFS preorder over edges (each edge listed when entered)."""
    E = src.size
    order = np.argsort(src, kind="stable")
    counts = np.bincount(src, minlength=n_nodes)
    start = np.zeros(n_nodes + 1, dtype=np.int64)
    np.cumsum(counts, out=start[1:])
    indeg = np.bincount(dst, minlength=n_nodes)
    entered = np.zeros(E, dtype=bool)
    visited = np.zeros(n_nodes, dtype=bool)
    out = np.empty(E, dtype=np.int64)
    n_out = 0
    roots = list(np.flatnonzero((indeg == 0) & (counts > 0))) + list(range(n_nodes))
    for root in roots:
        if visited[root]:
            continue
        visited[root] = True
        stack = [(int(root), int(start[root]))]
        while stack:
            v, pos = stack[-1]
            if pos >= start[v + 1]:
                stack.pop()
                continue
            stack[-1] = (v, pos + 1)
            e = int(order[pos])
            if entered[e]:
                continue
            entered[e] = True
            out[n_out] = e
            n_out += 1
            w = int(dst[e])
            if not visited[w]:
                visited[w] = True
                stack.append((w, int(start[w])))
        if n_out == E:
            break
    return out[:n_out]


def partition_edges(src: np.ndarray, dst: np.ndarray, n_nodes: int, nranks: int) -> np.ndarray:
    """Owner rank of every edge: contiguous equal chunks of the DFS preorder."""
    E = src.size
    if nranks == 1:
        return np.zeros(E, dtype=np.int32)
    pre = dfs_edge_order(src, dst, n_nodes)
    owner = np.empty(E, dtype=np.int32)
    owner[pre] = (np.arange(E, dtype=np.int64) * nranks // max(E, 1)).astype(np.int32)
    return owner


@dataclass
class LocalProblem:
    rank: int
    nranks: int
    N: int
    edges: np.ndarray  # global edge ids owned by this rank, local order
    lm_nodes: np.ndarray  # bifurcation node ids whose multiplier row is owned here
    edge_x: np.ndarray  # (E_r, 6)
    edge_lm: np.ndarray  # (E_r, 2) int32 column of lambda at source / target, -1 = none
    lm_rowptr: np.ndarray
    lm_col: np.ndarray
    lm_val: np.ndarray
    n_ghost: int
    peers: np.ndarray = field(default_factory=lambda: np.zeros(0, np.int32))
    send_off: np.ndarray = field(default_factory=lambda: np.zeros(1, np.int32))
    send_idx: np.ndarray = field(default_factory=lambda: np.zeros(0, np.int32))
    recv_off: np.ndarray = field(default_factory=lambda: np.zeros(1, np.int32))
    # global single-rank layout index of every ghost column (diagnostics / tests)
    ghost_global: np.ndarray = field(default_factory=lambda: np.zeros(0, np.int64))
    # owning rank of every global edge (the partition; the preconditioner's coarse step
    # needs the whole map)
    edge_owner: np.ndarray = field(default_factory=lambda: np.zeros(0, np.int32))
    # cut bifurcations (incident edges on several ranks), one global order on every rank:
    # per owned multiplier row its cut index or -1; per cut index this rank's flux end rows
    # there and their coupling (+-1) when another rank owns the row (nx_set_cut)
    n_cut: int = 0
    lm_cut: np.ndarray = field(default_factory=lambda: np.zeros(0, np.int32))
    gk_off: np.ndarray = field(default_factory=lambda: np.zeros(1, np.int32))
    gk_row: np.ndarray = field(default_factory=lambda: np.zeros(0, np.int32))
    gk_coef: np.ndarray = field(default_factory=lambda: np.zeros(0, np.float64))

    @property
    def n_edge_dofs(self) -> int:
        return self.edges.size * (2 * self.N + 1)

    @property
    def n_own(self) -> int:
        return self.n_edge_dofs + self.lm_nodes.size


class _RankView:
    """Per-rank numbering derived from the global partition (used for all ranks)."""

    def __init__(self, r, N, owner_e, lm_owner, bif_nodes):
        self.edges = np.flatnonzero(owner_e == r)
        per = 2 * N + 1
        self.edge_local = np.full(owner_e.size, -1, dtype=np.int64)
        self.edge_local[self.edges] = np.arange(self.edges.size) * per
        self.lm_nodes = bif_nodes[lm_owner[bif_nodes] == r]
        self.n_edge_dofs = self.edges.size * per


def build_local_problem(pos: np.ndarray, src: np.ndarray, dst: np.ndarray, degree: np.ndarray,
                        N: int, rank: int = 0, nranks: int = 1,
                        owner: np.ndarray | None = None) -> LocalProblem:
    """Local arrays of ``rank`` for ``nx_create`` plus its halo plan."""
    n_nodes = pos.shape[0]
    E = src.size
    per = 2 * N + 1
    pos3 = np.zeros((n_nodes, 3), dtype=np.float64)
    pos3[:, : pos.shape[1]] = pos
    if owner is None:
        owner = partition_edges(src, dst, n_nodes, nranks)
    owner = np.asarray(owner, dtype=np.int32)
    bif = np.flatnonzero(degree > 1)

    # owner of each bifurcation's multiplier: first in-edge, else first out-edge
    first_in = np.full(n_nodes, E, dtype=np.int64)
    np.minimum.at(first_in, dst, np.arange(E))
    first_out = np.full(n_nodes, E, dtype=np.int64)
    np.minimum.at(first_out, src, np.arange(E))
    anchor = np.where(first_in < E, first_in, first_out)
    lm_owner = np.full(n_nodes, -1, dtype=np.int32)
    lm_owner[bif] = owner[anchor[bif]]

    views = [_RankView(r, N, owner, lm_owner, bif) for r in range(nranks)]
    # local index of every multiplier on its owning rank
    lm_local = np.full(n_nodes, -1, dtype=np.int64)
    for v in views:
        lm_local[v.lm_nodes] = v.n_edge_dofs + np.arange(v.lm_nodes.size)

    # incidence of bifurcations: (node, edge, end) with end 0 = q_0 (out-edge, -1),
    # end 1 = q_N (in-edge, +1); sorted by node then by the column on the row's rank
    is_bif = degree > 1
    e_all = np.arange(E)
    inc_node = np.concatenate([dst[is_bif[dst]], src[is_bif[src]]])
    inc_edge = np.concatenate([e_all[is_bif[dst]], e_all[is_bif[src]]])
    inc_end = np.concatenate([np.ones(int(is_bif[dst].sum()), np.int64),
                              np.zeros(int(is_bif[src].sum()), np.int64)])

    def key_edge_end(e, end):  # global key of a flux end DoF
        return ("q", int(e), int(end))

    def ghost_table(r: int):
        """Ordered ghost keys of rank r and their owners."""
        v = views[r]
        keys = {}
        # multipliers at the ends of local edges owned elsewhere
        for end, nodes in ((0, src[v.edges]), (1, dst[v.edges])):
            m = is_bif[nodes] & (lm_owner[nodes] != r)
            for b in np.unique(nodes[m]):
                keys[("lm", int(b))] = (int(lm_owner[b]), int(lm_local[b]))
        # flux ends of remote edges read by local multiplier rows
        mine = lm_owner[inc_node] == r
        remote = owner[inc_edge] != r
        for e, end in zip(inc_edge[mine & remote], inc_end[mine & remote]):
            o = int(owner[e])
            keys[key_edge_end(e, end)] = (o, int(views[o].edge_local[e] + (2 * N if end else 0)))
        ordered = sorted(keys.items(), key=lambda kv: (kv[1][0], kv[1][1]))
        return [k for k, _ in ordered], [o for _, (o, _) in ordered], [li for _, (_, li) in ordered]

    tables = [ghost_table(r) for r in range(nranks)] if nranks > 1 else [([], [], [])]
    gkeys, gowner, glocal = tables[rank]
    v = views[rank]
    n_own = v.n_edge_dofs + v.lm_nodes.size
    ghost_col = {k: n_own + i for i, k in enumerate(gkeys)}

    # edge arrays
    Er = v.edges.size
    edge_x = np.empty((Er, 6), dtype=np.float64)
    edge_x[:, :3] = pos3[src[v.edges]]
    edge_x[:, 3:] = pos3[dst[v.edges]]
    edge_lm = np.full((Er, 2), -1, dtype=np.int64)
    s_nodes, d_nodes = src[v.edges], dst[v.edges]
    if nranks == 1:
        edge_lm[:, 0] = np.where(is_bif[s_nodes], lm_local[s_nodes], -1)
        edge_lm[:, 1] = np.where(is_bif[d_nodes], lm_local[d_nodes], -1)
    else:
        # column of every multiplier this rank touches: owned, else its ghost column
        col_of = np.where(lm_owner == rank, lm_local, -1)
        for k, c in ghost_col.items():
            if k[0] == "lm":
                col_of[k[1]] = c
        edge_lm[:, 0] = np.where(is_bif[s_nodes], col_of[s_nodes], -1)
        edge_lm[:, 1] = np.where(is_bif[d_nodes], col_of[d_nodes], -1)
        assert (edge_lm[is_bif[np.stack([s_nodes, d_nodes], axis=1)]] >= 0).all()

    # multiplier rows of this rank
    mine = lm_owner[inc_node] == rank
    n_inc = inc_node[mine]
    e_inc = inc_edge[mine]
    end_inc = inc_end[mine]
    if nranks == 1:
        cols = v.edge_local[e_inc] + np.where(end_inc == 1, 2 * N, 0)
    else:
        cols = v.edge_local[e_inc] + np.where(end_inc == 1, 2 * N, 0)
        for j in np.flatnonzero(owner[e_inc] != rank).tolist():  # remote flux ends only
            cols[j] = ghost_col[key_edge_end(int(e_inc[j]), int(end_inc[j]))]
    vals = np.where(end_inc == 1, 1.0, -1.0)
    row = lm_local[n_inc] - v.n_edge_dofs
    o = np.lexsort((cols, row))
    row, cols, vals = row[o], cols[o], vals[o]
    counts = np.bincount(row, minlength=v.lm_nodes.size)
    lm_rowptr = np.zeros(v.lm_nodes.size + 1, dtype=np.int32)
    np.cumsum(counts, out=lm_rowptr[1:])

    lp = LocalProblem(rank, nranks, N, v.edges, v.lm_nodes, edge_x, edge_lm.astype(np.int32),
                      lm_rowptr, cols.astype(np.int32), vals.astype(np.float64), len(gkeys))
    bif_idx = np.full(n_nodes, -1, dtype=np.int64)
    bif_idx[bif] = np.arange(bif.size)
    lp.ghost_global = np.asarray(
        [E * per + bif_idx[k[1]] if k[0] == "lm" else k[1] * per + (2 * N if k[2] else 0)
         for k in gkeys], dtype=np.int64)
    lp.edge_owner = owner
    if nranks > 1:
        # receive plan: my ghosts grouped by owner
        peers_recv = sorted(set(gowner))
        # send plan: other ranks' ghosts that I own, in their order
        send_lists = {}
        for r in range(nranks):
            if r == rank:
                continue
            k_r, o_r, l_r = tables[r]
            idx = [li for oo, li in zip(o_r, l_r) if oo == rank]
            if idx:
                send_lists[r] = idx
        peers = sorted(set(peers_recv) | set(send_lists))
        send_off, send_idx, recv_off = [0], [], [0]
        gowner_arr = np.asarray(gowner, dtype=np.int64)
        for p in peers:
            send_idx.extend(send_lists.get(p, []))
            send_off.append(len(send_idx))
            recv_off.append(recv_off[-1] + int((gowner_arr == p).sum()))
        lp.peers = np.asarray(peers, dtype=np.int32)
        lp.send_off = np.asarray(send_off, dtype=np.int32)
        lp.send_idx = np.asarray(send_idx, dtype=np.int32)
        lp.recv_off = np.asarray(recv_off, dtype=np.int32)
        _cut_lists(lp, v, src, dst, is_bif, inc_node, inc_edge, owner, lm_owner, rank, N)
    return lp


def _cut_lists(lp: LocalProblem, v, src, dst, is_bif, inc_node, inc_edge, owner, lm_owner,
               rank: int, N: int) -> None:
    """The cut bifurcations (sorted node ids: the same K and order on every rank) and this
    rank's part of their multiplier rows: the owner forms the row over its own flux ends,
    every other rank adds -(+-1) x_q of its flux ends there (the coupling is symmetric:
    A[q, lambda] = A[lambda, q] = -1 at a source end q_0, +1 at a target end q_N)."""
    cut = np.unique(inc_node[owner[inc_edge] != lm_owner[inc_node]])
    k_of = np.full(is_bif.size, -1, dtype=np.int64)
    k_of[cut] = np.arange(cut.size)
    lp.n_cut = int(cut.size)
    lp.lm_cut = k_of[v.lm_nodes].astype(np.int32)
    per = 2 * N + 1
    ks, rows, coefs = [], [], []
    for end, nodes in ((0, src[v.edges]), (1, dst[v.edges])):
        m = is_bif[nodes] & (lm_owner[nodes] != rank)
        loc = np.flatnonzero(m)
        ks.append(k_of[nodes[loc]])
        rows.append(loc * per + (2 * N if end else 0))
        coefs.append(np.full(loc.size, 1.0 if end else -1.0))
    ks, rows, coefs = np.concatenate(ks), np.concatenate(rows), np.concatenate(coefs)
    assert (ks >= 0).all(), "a remote multiplier at a local edge end is a cut bifurcation"
    o = np.lexsort((rows, ks))
    lp.gk_row = rows[o].astype(np.int32)
    lp.gk_coef = coefs[o].astype(np.float64)
    lp.gk_off = np.searchsorted(ks[o], np.arange(cut.size + 1)).astype(np.int32)


def global_row_ids(lp: LocalProblem, n_edges_global: int, bif_index: np.ndarray) -> np.ndarray:
    """The single-rank layout row of every owned row, then of every ghost column."""
    per = 2 * lp.N + 1
    rows = (np.asarray(lp.edges, dtype=np.int64)[:, None] * per + np.arange(per)[None, :]).ravel()
    lam = n_edges_global * per + np.asarray(bif_index)[np.asarray(lp.lm_nodes, dtype=np.int64)]
    return np.concatenate([rows, lam, np.asarray(lp.ghost_global, dtype=np.int64)])


def cycle_pairs_global(lp: LocalProblem, cyc_rows: np.ndarray, n_edges_global: int,
                       bif_index: np.ndarray) -> list:
    """This rank's dropped cycle couplings (``TreePreconditioner.cyc_rows``: flux end row,
    multiplier column) as single-rank layout rows."""
    ids = global_row_ids(lp, n_edges_global, bif_index)
    return [(int(ids[q]), int(ids[c])) for q, c in np.asarray(cyc_rows).reshape(-1, 2)]


def team_cycle_tables(lp: LocalProblem, cyc_rows: np.ndarray, all_pairs, n_edges_global: int,
                      bif_index: np.ndarray):
    """``nx_set_cycles_team``'s arrays for this rank from every rank's cycle pairs (global
    rows; one global order: sorted): ``(own[2K], qloc[K], lcol[K])`` -- per column of U this
    rank's row or -1, and for this rank's own chains the flux end row and the multiplier's
    column (owned or ghost) in its numbering."""
    pairs = sorted({(int(a), int(b)) for a, b in all_pairs})
    ids = global_row_ids(lp, n_edges_global, bif_index)
    n_own = lp.n_own
    order = np.argsort(ids[:n_own], kind="stable")

    def owned(g: int) -> int:
        i = np.searchsorted(ids[:n_own], g, sorter=order)
        return int(order[i]) if i < n_own and ids[order[i]] == g else -1

    mine = {(int(ids[q]), int(ids[c])): (int(q), int(c))
            for q, c in np.asarray(cyc_rows).reshape(-1, 2)}
    own = np.array([owned(g) for pr in pairs for g in pr], dtype=np.int32)
    qloc = np.array([mine[pr][0] if pr in mine else -1 for pr in pairs], dtype=np.int32)
    lcol = np.array([mine[pr][1] if pr in mine else -1 for pr in pairs], dtype=np.int32)
    return own, qloc, lcol
