"""Tree Schur-complement preconditioner for MINRES (host-side setup).

MINRES needs a symmetric positive definite preconditioner. For the symmetric device
system ``A = [[M, G], [G^T, 0]]`` (flux rows / pressure + multiplier columns) we use

    P = blockdiag(D, S),   D = lumped (row-sum) flux mass,   S = G^T D^{-1} G,

the exact Schur complement of the lumped system. ``S`` is a weighted graph Laplacian:
its nodes are the pressure cells and the junction multipliers, and every flux DoF ``q``
is a resistor of resistance ``d_q`` (its lumped mass) between the two nodes it couples
-- or between one node and ground, at an inlet/outlet end (natural pressure BC).

On a tree network ``S`` is a tree Laplacian and ``P^{-1} r`` is computed exactly:

* every graph edge is a *chain* ``top -- p_0 -- ... -- p_{N-1} -- bottom`` of series
  resistors ``rho_0..rho_N``. With ``D_k = rho_0 + .. + rho_k`` and ``T = D_{N-1} + rho_N``
  the chain condenses to a conductance ``1/T`` between its ends plus injected currents
  ``I_top = sum_k r_k (T - D_k)/T`` and ``I_bot = sum_k r_k D_k/T``, and after the end
  values are known its cells follow from the 1-D Green's function
  ``z_k = z_top (T-D_k)/T + z_bot D_k/T + (D_k/T) sum_{j>=k} (T-D_j) r_j
  + ((T-D_k)/T) sum_{j<k} D_j r_j`` -- prefix sums, i.e. wave scans on the device;
* the junctions form a rooted forest; leaf-to-root elimination
  ``D_b = g_up + sum_down [g (1 - g/D_c) or g if grounded]``,
  ``J_b = r_b + I_bot(up chain) + sum_down [I_top + g J_c / D_c]`` then
  ``z_b = (J_b + g_up z_parent) / D_b`` root-to-leaf.

Device decomposition (csrc/nxhip.hip k_pc_up / k_pc_top / k_pc_down): the junction forest
is cut at a depth so that the *lower subtrees* (each processed by one workgroup, chains +
junction levels) number a few hundred and the *top* part (all junctions above the cut,
one workgroup, junction math only) stays small; chains whose lower end is in the top part
are handed round-robin to the lower jobs (one workgroup per job, no extra launches).

Exact variant (the default). With the *consistent* mass ``M`` instead of ``D`` the
preconditioner ``P = blockdiag(M, G^T M^{-1} G)`` makes ``P^{-1} A`` have exactly three
eigenvalues ``{1, (1 +- sqrt 5)/2}`` (Murphy, Golub & Wathen 2000), so MINRES converges
in 3 iterations. On one edge the flux constraint ``-B u = r_p`` fixes ``u`` up to its
start value ``u_0``, and ``1^T M = 1^T D = d^T`` (the column sums of the P1 mass are the
lumped mass), so ``u_0`` -- hence the whole junction system -- is identical for ``M`` and
``D``. Only the chain outputs change: the cell values are prefix sums of ``M u`` instead
of ``D u``, and ``(M - D) u`` telescopes (``u_{k+1} - u_k = -r_p[k]``) to

    (G^T M^{-1} G)^{-1} = (G^T D^{-1} G)^{-1} - (R h / 6) I   on the pressure cells,

while the flux block becomes ``M_e^{-1} r_q = (6 / (R h)) T^{-1} r_q`` with the fixed
``T = tridiag(1, 4, 1)`` (2 at both ends) of size N+1.

Graphs that are not trees use the same machinery on a spanning forest: a chain that
would close a cycle is grounded at one end. ``P`` stays SPD (a grounded Laplacian block);
only its quality drops.

Partitioned problems keep ``P^{-1}`` exact through a *coarse step*. The coarse set ``C``
holds every interface junction (edges of two or more ranks meet there) and, per rank,
the junctions on paths between its interface junctions (Steiner closure). Each rank roots
its local forest at its coarse junctions -- owned or ghost -- so every non-coarse piece
hangs from exactly one coarse junction and eliminates into it independently. The ranks'
partial ``(D, J)`` of the coarse junctions and the conductances of the chains joining two
coarse junctions are summed in one all-reduce; the result is the Schur complement of ``S``
on ``C``, again a tree Laplacian, which every rank solves redundantly (same order, same
bits). The back-substitution then starts from exact coarse values. Without the coarse
step (cut junctions grounded per rank) MINRES needs 5x the iterations at 8 ranks.
"""

from __future__ import annotations

import heapq
from collections import deque
from dataclasses import dataclass, field

import numpy as np

__all__ = ["CoarseStructure", "TreePreconditioner", "build_tree_preconditioner", "mass_tinv",
           "coarse_structure", "apply_model", "pc_up_model", "pc_finish_model"]

_EMPTY_I = np.zeros(0, dtype=np.int32)


@dataclass
class CoarseStructure:
    """Global coarse forest of a partitioned problem (identical on every rank)."""

    node: np.ndarray  # (nC,) global node id of every coarse junction, level order
    cidx: np.ndarray  # (n_nodes,) coarse index of a node, -1
    parent: np.ndarray  # (nC,) parent coarse index, -1 at a root
    pedge: np.ndarray  # (nC,) global edge joining the junction to its parent, -1
    child_off: np.ndarray  # (nC + 1,) CSR of children
    child: np.ndarray
    lvl_off: np.ndarray  # level offsets, root level first
    demoted: np.ndarray  # (E,) bool: coarse-coarse edge closing a cycle (grounded at one end)

    @property
    def n(self) -> int:
        return int(self.node.size)


def coarse_structure(src: np.ndarray, dst: np.ndarray, degree: np.ndarray,
                     owner: np.ndarray, nranks: int,
                     terminals: np.ndarray | None = None) -> CoarseStructure:
    """Interface junctions + per-rank Steiner closure, as a level-ordered forest.

    ``terminals``: junctions kept in the coarse set besides the interface ones (their
    Steiner closure too). A one-rank problem has no interface junctions; forcing some lets
    the multi-rank direct schedule run on a one-rank RCCL communicator (its GPU test)."""
    src = np.asarray(src, dtype=np.int64)
    dst = np.asarray(dst, dtype=np.int64)
    n_nodes, E = int(np.asarray(degree).size), int(src.size)
    is_bif = np.asarray(degree) > 1
    coarse = np.zeros(n_nodes, dtype=bool)
    forced = np.zeros(n_nodes, dtype=bool)
    if terminals is not None:
        forced[np.asarray(terminals, dtype=np.int64)] = True
        forced &= is_bif
    if (nranks > 1 or forced.any()) and E > 0:
        owner = np.asarray(owner, dtype=np.int64)
        ends = np.concatenate([src, dst])
        eo = np.concatenate([owner, owner])
        m = is_bif[ends]
        mn = np.full(n_nodes, nranks, dtype=np.int64)
        mx = np.full(n_nodes, -1, dtype=np.int64)
        np.minimum.at(mn, ends[m], eo[m])
        np.maximum.at(mx, ends[m], eo[m])
        terminal = (is_bif & (mx > mn)) | forced
        coarse |= terminal
        order = np.argsort(owner, kind="stable")
        bounds = np.searchsorted(owner[order], np.arange(nranks + 1))
        for r in range(nranks):
            er = order[bounds[r]:bounds[r + 1]]
            if er.size == 0:
                continue
            nodes, inv = np.unique(np.concatenate([src[er], dst[er]]), return_inverse=True)
            a, b = inv[:er.size], inv[er.size:]
            k = nodes.size
            deg = np.bincount(a, minlength=k) + np.bincount(b, minlength=k)
            inc_v = np.concatenate([a, b])
            inc_e = np.concatenate([np.arange(er.size), np.arange(er.size)])
            o = np.argsort(inc_v, kind="stable")
            inc_e = inc_e[o]
            off = np.searchsorted(inc_v[o], np.arange(k + 1))
            alive = np.ones(er.size, dtype=bool)
            term = terminal[nodes]
            # prune non-terminal leaves: what stays is the Steiner forest of the terminals
            # (the fixpoint does not depend on the order, so all current leaves go at once;
            # only the far ends of the removed edges can become leaves next)
            cand = np.flatnonzero((deg == 1) & ~term)
            while cand.size:
                leaf = np.unique(cand[(deg[cand] == 1) & ~term[cand]])
                if not leaf.size:
                    break
                rep, pos = _ragged(off, leaf)
                e = inc_e[pos]
                e = np.unique(e[alive[e]])  # the one live edge of each leaf (shared: once)
                alive[e] = False
                np.subtract.at(deg, a[e], 1)
                np.subtract.at(deg, b[e], 1)
                cand = np.concatenate([a[e], b[e]])
            keep = (deg > 0) & is_bif[nodes]
            coarse[nodes[keep]] = True
    cn = np.flatnonzero(coarse)
    demoted = np.zeros(E, dtype=bool)
    adj: dict[int, list[tuple[int, int]]] = {int(v): [] for v in cn}
    for e in np.flatnonzero(coarse[src] & coarse[dst]).tolist():
        a, b = int(src[e]), int(dst[e])
        adj[a].append((e, b))
        adj[b].append((e, a))
    depth: dict[int, int] = {}
    par: dict[int, int] = {}
    pe: dict[int, int] = {}
    disc: list[int] = []
    tree = set()
    for r in cn.tolist():
        if r in depth:
            continue
        depth[r], par[r], pe[r] = 0, -1, -1
        disc.append(r)
        q = deque([r])
        while q:
            u = q.popleft()
            for e, w in adj[u]:
                if w not in depth:
                    depth[w], par[w], pe[w] = depth[u] + 1, u, e
                    tree.add(e)
                    disc.append(w)
                    q.append(w)
    for v in cn.tolist():
        for e, _ in adj[v]:
            if e not in tree:
                demoted[e] = True
    pos = {v: i for i, v in enumerate(disc)}
    lvl = sorted(disc, key=lambda v: (depth[v], pos[v]))
    cidx = np.full(n_nodes, -1, dtype=np.int32)
    cidx[np.asarray(lvl, dtype=np.int64)] = np.arange(len(lvl), dtype=np.int32)
    nC = len(lvl)
    parent = np.array([cidx[par[v]] if par[v] != -1 else -1 for v in lvl], dtype=np.int32)
    pedge = np.array([pe[v] for v in lvl], dtype=np.int64)
    kids: list[list[int]] = [[] for _ in range(nC)]
    for i in range(nC):
        if parent[i] >= 0:
            kids[parent[i]].append(i)
    child_off = np.zeros(nC + 1, dtype=np.int32)
    np.cumsum([len(k) for k in kids], out=child_off[1:])
    child = np.array([c for k in kids for c in k], dtype=np.int32)
    dl = np.array([depth[v] for v in lvl], dtype=np.int64)
    nlv = int(dl.max()) + 1 if nC else 0
    lvl_off = np.searchsorted(dl, np.arange(nlv + 1)).astype(np.int32)
    return CoarseStructure(node=np.asarray(lvl, dtype=np.int64), cidx=cidx, parent=parent,
                           pedge=pedge, child_off=child_off, child=child, lvl_off=lvl_off,
                           demoted=demoted)


@dataclass
class TreePreconditioner:
    N: int
    # chains (one per local edge), in job order
    chain_edge: np.ndarray  # local edge slot
    chain_flip: np.ndarray  # 1: chain order runs target -> source
    chain_up: np.ndarray  # junction slot at the top end, -1 = ground
    chain_lo: np.ndarray  # junction slot at the bottom end, -1 = ground
    # junction slots, grouped by job, level order inside a job
    slot_lam: np.ndarray  # local DoF of the multiplier
    slot_pchain: np.ndarray  # chain linking to the parent (its bottom end is this slot), -1
    slot_parent: np.ndarray  # parent slot, -1
    slot_dc_off: np.ndarray  # CSR over chains whose top end is the slot
    slot_dc: np.ndarray
    dc_lo: np.ndarray  # bottom slot of every slot_dc entry (-1 = ground), precomputed
    slot_plam: np.ndarray  # multiplier row of the parent slot, -1
    # jobs: lower subtrees (chains + junction levels); chain-only jobs only when there is
    # no lower subtree
    job_chain_off: np.ndarray  # n_jobs + 1
    job_lvl_off: np.ndarray  # n_jobs + 1, offsets into lvl_slot_off
    lvl_slot_off: np.ndarray  # slot offsets of every level (per job, root level first)
    # top part (one workgroup): junction slots [top_slot0, top_slot1), levels
    top_lvl_off: np.ndarray  # slot offsets of the top levels (root level first)
    n_jobs: int
    n_slots: int
    # coarse step (several ranks): coarse index of every slot (-1 = not coarse), the local
    # chains joining two coarse junctions (their top / bottom coarse index; the bottom one
    # is the child in the coarse forest and indexes its conductance), the global forest
    # dense top part (single rank): the down workgroups compute the top junction values
    # they need as z_t = sum_s G[t, s] a_s (G = inverse of the top part's tree Schur
    # matrix, built once per solve). job_tslot: top slots whose multiplier row a job
    # updates / writes (round-robin); job_need: top slots whose value a job reads
    job_tslot_off: np.ndarray = field(default_factory=lambda: np.zeros(1, np.int32))
    job_tslot: np.ndarray = field(default_factory=lambda: _EMPTY_I)
    job_need_off: np.ndarray = field(default_factory=lambda: np.zeros(1, np.int32))
    job_need: np.ndarray = field(default_factory=lambda: _EMPTY_I)
    # producer-side inputs of the dense top: a_s = sum of u[top_uoff[s]:top_uoff[s+1]];
    # the up kernel writes every contribution to its fixed place: y' of top slot s at
    # slot_uy[s - ts0], I_top / I_bot of chain c at chain_uit[c] / chain_uib[c] (-1: not
    # a top input), and for a job root kappa J_root + I_top(root's parent chain) at
    # job_root_u[j] with kappa = dc entry job_root_dc[j]
    top_uoff: np.ndarray = field(default_factory=lambda: np.zeros(1, np.int32))
    slot_uy: np.ndarray = field(default_factory=lambda: _EMPTY_I)
    chain_uit: np.ndarray = field(default_factory=lambda: _EMPTY_I)
    chain_uib: np.ndarray = field(default_factory=lambda: _EMPTY_I)
    job_root_u: np.ndarray = field(default_factory=lambda: _EMPTY_I)
    job_root_dc: np.ndarray = field(default_factory=lambda: _EMPTY_I)
    n_coarse: int = 0
    slot_cidx: np.ndarray = field(default_factory=lambda: _EMPTY_I)
    cc_chain: np.ndarray = field(default_factory=lambda: _EMPTY_I)
    cc_top: np.ndarray = field(default_factory=lambda: _EMPTY_I)
    cc_bot: np.ndarray = field(default_factory=lambda: _EMPTY_I)
    c_parent: np.ndarray = field(default_factory=lambda: _EMPTY_I)
    c_child_off: np.ndarray = field(default_factory=lambda: np.zeros(1, np.int32))
    c_child: np.ndarray = field(default_factory=lambda: _EMPTY_I)
    c_lvl_off: np.ndarray = field(default_factory=lambda: np.zeros(1, np.int32))
    # no chain closes a cycle (grounded at one end): P^{-1} is the exact block inverse, so
    # the direct tree solve (nx_set_solver) is exact
    tree_exact: bool = False
    # graphs with cycles: per cycle-closing chain the coupling its grounded end drops, (flux
    # end row, multiplier column: a ghost column with several ranks when another rank owns
    # the row) -- the system the tree solve inverts is A minus these symmetric +-1 pairs,
    # and the direct solve corrects for them (nx_set_cycles, nx_set_cycles_team)
    cyc_rows: np.ndarray = field(default_factory=lambda: np.zeros((0, 2), np.int32))

    @property
    def n_chains(self) -> int:
        return int(self.chain_edge.size)


# LDS caps of the preconditioner kernels (csrc/nxhip.hip): chains, junction slots and
# down-chain entries per job. The top part's chains ride along (balanced), hence the
# margin on the chain cap.
_CAP_CHAINS, _CAP_SLOTS, _CAP_DC = 512, 256, 768
_CHAIN_MARGIN = 32


def _ragged(off: np.ndarray, items: np.ndarray) -> tuple[np.ndarray, np.ndarray]:
    """Concatenation of the CSR rows ``items`` (in order): (row position, entry index)."""
    starts = off[items]
    lens = off[items + 1] - starts
    total = int(lens.sum())
    if total == 0:
        return np.zeros(0, np.int64), np.zeros(0, np.int64)
    rep = np.repeat(np.arange(items.size), lens)
    first = np.cumsum(lens) - lens
    return rep, np.arange(total) - first[rep] + starts[rep]


def _csr(keys: np.ndarray, n: int) -> tuple[np.ndarray, np.ndarray]:
    """Stable grouping of positions by ``keys`` (0 <= key < n): (offsets, positions)."""
    order = np.argsort(keys, kind="stable")
    off = np.zeros(n + 1, dtype=np.int64)
    np.cumsum(np.bincount(keys, minlength=n), out=off[1:])
    return off, order


def _bfs(frontier, adj_off, adj_e, adj_w, isj, depth, parent, pchain, tree_edge) -> None:
    """Level-synchronous breadth-first search from the junctions ``frontier`` (depth already
    set), through local edges to unvisited junctions. A node's parent is its first
    discoverer in frontier order, adjacency order -- exactly what a FIFO queue gives, and
    for several roots the same as one search per root as long as no unvisited junction is
    reachable from two of them (true for the roots used here: see the caller)."""
    F = np.asarray(frontier, dtype=np.int64)
    while F.size:
        rep, pos = _ragged(adj_off, F)
        w = adj_w[pos]
        m = isj[w] & (depth[w] < 0)
        if not m.any():
            break
        w, e, u = w[m], adj_e[pos][m], F[rep][m]
        _, first = np.unique(w, return_index=True)
        first.sort()
        w, e, u = w[first], e[first], u[first]
        depth[w] = depth[u] + 1
        parent[w] = u
        pchain[w] = e
        tree_edge[e] = True
        F = w


@dataclass
class _JobRoots:
    roots: list
    promoted: list


def _split_job_roots(roots, kids, sizes, n_top: int, max_top: int,
                     balance: int = 0) -> _JobRoots:
    """Replace every job root whose subtree exceeds the LDS caps by its children (the
    root joins the top part), recursively, keeping the roots' order; stops promoting
    when the top part would exceed ``max_top``. With ``balance`` > 0, first split the
    root with the most chains while that keeps at most ``balance`` jobs. ``kids(v)`` lists
    the children of junction ``v``; ``sizes`` = (chains, slots, down-chain entries) of
    every junction's subtree (arrays over node ids)."""
    s_ch, s_sl, s_dc = sizes

    def over(v: int) -> bool:
        return (s_ch[v] > _CAP_CHAINS - _CHAIN_MARGIN or s_sl[v] > _CAP_SLOTS
                or s_dc[v] > _CAP_DC)

    promoted = []
    if balance > 0:
        import heapq

        # pieces far below the average job (small subtrees hanging from the coarse
        # junctions) join the top part whole: they would take a workgroup each and leave
        # too few jobs to split the largest subtrees (257-chain jobs at 8 ranks)
        avg = float(sum(int(s_ch[v]) for v in roots)) / max(balance, 1)
        keep = []
        for v in roots:
            if 2 * int(s_ch[v]) < avg and n_top + len(promoted) + int(s_sl[v]) <= max_top:
                sub = [v]  # level order of the subtree
                k = 0
                while k < len(sub):
                    sub.extend(kids(sub[k]))
                    k += 1
                promoted.extend(sub)
            else:
                keep.append(v)
        roots = keep
        order = {v: i for i, v in enumerate(roots)}
        heap = [(-int(s_ch[v]), order[v], v) for v in roots]
        heapq.heapify(heap)
        live = set(roots)
        while heap and n_top + len(promoted) < max_top:
            negc, _, v = heap[0]
            ks = kids(v)
            if not ks or len(live) - 1 + len(ks) > balance:
                break
            heapq.heappop(heap)
            live.discard(v)
            promoted.append(v)
            for c in ks:
                order[c] = len(order)
                live.add(c)
                heapq.heappush(heap, (-int(s_ch[c]), order[c], c))
        roots = sorted(live)  # slot_nodes order, as the depth cut's roots
    out = []
    todo = list(reversed(roots))
    while todo:
        r = todo.pop()
        ks = kids(r)
        if ks and over(r) and n_top + len(promoted) < max_top:
            promoted.append(r)
            todo.extend(reversed(ks))
        else:
            out.append(r)
    return _JobRoots(out, promoted)


def build_tree_preconditioner(lp, src: np.ndarray, dst: np.ndarray, degree: np.ndarray,
                              target_jobs: int = 256, max_top: int = 1024,
                              coarse: CoarseStructure | None = None,
                              balanced: bool = True) -> TreePreconditioner:
    """Decompose the rank-local problem ``lp`` (:class:`layout.LocalProblem`).

    ``src``/``dst`` are the global node ids of all edges, ``degree`` the global degrees.
    With several ranks the coarse forest is derived from ``lp.edge_owner`` unless given.
    Array code throughout (arrays over global node ids); the only Python loops run over
    job roots and the few junctions above the cut.
    """
    N = lp.N
    E = lp.edges.size
    src = np.asarray(src, dtype=np.int64)
    dst = np.asarray(dst, dtype=np.int64)
    n_nodes = max(int(np.asarray(degree).size),
                  int(max(src.max(initial=-1), dst.max(initial=-1))) + 1)
    es, ed = src[lp.edges], dst[lp.edges]
    if coarse is None and lp.nranks > 1:
        coarse = coarse_structure(src, dst, degree, lp.edge_owner, lp.nranks)
    isc = np.zeros(n_nodes, dtype=bool)
    if coarse is not None:
        isc[: coarse.cidx.size] = coarse.cidx >= 0
    # junction slots: owned multipliers + ghost junctions at the ends of local edges (the
    # latter are interface junctions, hence coarse); lam = local DoF of the multiplier
    lam = np.full(n_nodes, -1, dtype=np.int64)
    lm_nodes = np.asarray(lp.lm_nodes, dtype=np.int64)
    lam[lm_nodes] = lp.n_edge_dofs + np.arange(lm_nodes.size)
    if lp.nranks > 1 and E:
        ends = np.stack([es, ed], axis=1).ravel()  # (edge, end) order
        cols = np.asarray(lp.edge_lm, dtype=np.int64).ravel()
        g = (cols >= lp.n_own) & (lam[ends] < 0)
        gv, first = np.unique(ends[g], return_index=True)  # first occurrence wins
        lam[gv] = cols[g][first]
    isj = lam >= 0
    slot_nodes = np.flatnonzero(isj)  # ascending node id
    # junction adjacency through local edges: per junction, (edge, other end) by edge
    e_ar = np.arange(E, dtype=np.int64)
    ma, mb = isj[es], isj[ed]
    a_u = np.concatenate([es[ma], ed[mb]])
    a_e = np.concatenate([e_ar[ma], e_ar[mb]])
    a_w = np.concatenate([ed[ma], es[mb]])
    o = np.lexsort((a_e, a_u))
    a_u, a_e, a_w = a_u[o], a_e[o], a_w[o]
    adj_off = np.zeros(n_nodes + 1, dtype=np.int64)
    np.cumsum(np.bincount(a_u, minlength=n_nodes), out=adj_off[1:])

    # spanning forest: coarse junctions are the roots (BFS never enters another coarse
    # junction: a path between two would make its junctions coarse too, so every other
    # piece hangs from at most one coarse root and the roots' searches can run together);
    # each remaining component from its first junction touching ground, else its first
    depth = np.full(n_nodes, -1, dtype=np.int64)
    parent_j = np.full(n_nodes, -1, dtype=np.int64)
    pchain = np.full(n_nodes, -1, dtype=np.int64)
    tree_edge = np.zeros(E, dtype=bool)
    croots = slot_nodes[isc[slot_nodes]]
    depth[croots] = 0
    _bfs(croots, adj_off, a_e, a_w, isj, depth, parent_j, pchain, tree_edge)
    rest = slot_nodes[depth[slot_nodes] < 0]
    if rest.size:
        from scipy.sparse import coo_matrix
        from scipy.sparse.csgraph import connected_components

        jj = isj[es] & isj[ed]
        A = coo_matrix((np.ones(int(jj.sum())), (es[jj], ed[jj])), shape=(n_nodes, n_nodes))
        _, label = connected_components(A, directed=False)
        touch = np.zeros(n_nodes, dtype=bool)
        touch[a_u[~isj[a_w]]] = True
        # first (lowest id) ground-touching junction of each component, else the lowest
        key = np.where(touch[rest], 0, 1)
        o = np.lexsort((rest, key, label[rest]))
        lab = label[rest][o]
        lead = np.ones(lab.size, dtype=bool)
        lead[1:] = lab[1:] != lab[:-1]
        roots2 = np.sort(rest[o][lead])
        depth[roots2] = 0
        _bfs(roots2, adj_off, a_e, a_w, isj, depth, parent_j, pchain, tree_edge)

    # chain ends: top = parent side (junction or ground), bottom = other
    up = np.full(E, -1, dtype=np.int64)
    lo = np.full(E, -1, dtype=np.int64)
    is_cc = np.zeros(E, dtype=bool)  # joins two coarse junctions (coarse step)
    n_cycle = 0  # chains grounded to break a cycle
    ge = np.asarray(lp.edges, dtype=np.int64)
    both_c = isc[es] & isc[ed] if coarse is not None else np.zeros(E, dtype=bool)
    dem = both_c & coarse.demoted[ge] if coarse is not None else both_c
    up[dem] = es[dem]  # closes a cycle of the coarse graph: ground one end
    n_cycle += int(dem.sum())
    fe = both_c & ~dem  # coarse forest edge: top = parent end, bottom = child end
    if fe.any():
        child_b = coarse.pedge[coarse.cidx[ed[fe]]] == ge[fe]
        up[fe] = np.where(child_b, es[fe], ed[fe])
        lo[fe] = np.where(child_b, ed[fe], es[fe])
        is_cc[fe] = True
    ja, jb = isj[es], isj[ed]
    t = ~both_c & tree_edge  # the child is the endpoint whose parent chain is e
    cb = jb & (pchain[ed] == e_ar)
    up[t] = np.where(cb[t], es[t], ed[t])
    lo[t] = np.where(cb[t], ed[t], es[t])
    r = ~both_c & ~tree_edge
    cyc = r & ja & jb  # closes a cycle: hang from the shallower end, ground the other
    up[cyc] = np.where(depth[es[cyc]] <= depth[ed[cyc]], es[cyc], ed[cyc])
    n_cycle += int(cyc.sum())
    # the coupling a grounded cycle end drops: (flux end row, multiplier column) per chain --
    # a chain closing a cycle inside this rank, or a coarse chain closing a cycle of the
    # coarse graph (several ranks; its multiplier may be a ghost column); the tree solve
    # inverts the system without them, the direct solve adds them back (Woodbury)
    ce = np.flatnonzero(cyc | dem)
    gnd = np.where(up[ce] == es[ce], ed[ce], es[ce])  # the grounded end's junction
    cyc_rows = np.stack([ce * (2 * N + 1) + np.where(gnd == es[ce], 0, 2 * N),
                         lam[gnd]], axis=1).astype(np.int32).reshape(-1, 2)
    g1 = r & ja & ~jb
    up[g1] = es[g1]
    g2 = r & ~ja & jb
    up[g2] = ed[g2]
    flip = (((up == ed) & (up != -1)) | ((up == -1) & (lo == es) & (lo != -1))).astype(np.int8)

    # cut depth: lower subtrees rooted at depth L (coarse junctions, depth 0, stay on top)
    dvals = depth[slot_nodes]
    maxd = int(dvals.max()) if dvals.size else -1
    counts = np.bincount(dvals, minlength=maxd + 1) if dvals.size else np.zeros(0, np.int64)
    L = maxd + 1  # default: everything in the top part
    for cand in range(maxd + 1):
        if counts[cand] >= target_jobs or counts[:cand].sum() + counts[cand] > max_top:
            L = cand
            break
    if croots.size:
        L = max(L, 1)

    # children of every junction (ascending node id) as CSR over node ids
    has_p = slot_nodes[parent_j[slot_nodes] >= 0]
    ch_off, o = _csr(parent_j[has_p], n_nodes)
    ch = has_p[o]

    def kids(v: int) -> list:
        return ch[ch_off[v]:ch_off[v + 1]].tolist()

    # subtree sizes (chains, slots, down-chain entries), deepest level first
    key = np.where(lo != -1, lo, up)
    s_ch = np.bincount(key[key != -1], minlength=n_nodes).astype(np.int64)
    dcm = (up != -1) & ~is_cc
    s_dc = np.bincount(up[dcm], minlength=n_nodes).astype(np.int64)
    s_sl = isj.astype(np.int64)
    by_d = slot_nodes[np.argsort(dvals, kind="stable")]
    d_off = np.searchsorted(dvals[np.argsort(dvals, kind="stable")], np.arange(maxd + 2))
    for dl in range(maxd, 0, -1):
        vs = by_d[d_off[dl]:d_off[dl + 1]]
        ps = parent_j[vs]
        np.add.at(s_ch, ps, s_ch[vs])
        np.add.at(s_sl, ps, s_sl[vs])
        np.add.at(s_dc, ps, s_dc[vs])

    # A lower subtree must fit one workgroup of the LDS kernels (csrc/nxhip.hip kCapC /
    # kCapS / kCapDC); an uneven local forest (several ranks: pieces of different heights
    # hang from the coarse junctions) can put 4x the typical subtree below one depth-L
    # root. Such a root is promoted into the top part and its children become job roots.
    if lp.nranks > 1 and croots.size and maxd >= 1:
        # several ranks: the local forest's pieces differ in height, so a fixed cut depth
        # gives uneven jobs; split the largest subtree first, from depth 1, until there are
        # target_jobs jobs (a uniform binary tree gives the depth cut's decomposition)
        L = 1
        start = slot_nodes[dvals == 1].tolist()
        balance = target_jobs
    else:
        start = slot_nodes[dvals == L].tolist()
        balance = 0
    jr = _split_job_roots(start, kids, (s_ch, s_sl, s_dc), n_top=int(counts[:L].sum()),
                          max_top=max_top, balance=balance)
    promoted = np.zeros(n_nodes, dtype=bool)
    promoted[np.asarray(jr.promoted, dtype=np.int64)] = True
    job_roots = np.asarray(jr.roots, dtype=np.int64)
    n_lower = job_roots.size

    # slots: lower subtrees (level order inside), then top levels. All jobs' levels are
    # expanded together; the frontier stays job-major, so a stable sort by (job, level)
    # gives every job's level order
    F, Jf, lv = job_roots, np.arange(n_lower, dtype=np.int64), 0
    parts_v, parts_j, parts_l = [], [], []
    while F.size:
        parts_v.append(F)
        parts_j.append(Jf)
        parts_l.append(np.full(F.size, lv, dtype=np.int64))
        rep, pos = _ragged(ch_off, F)
        F, Jf, lv = ch[pos], Jf[rep], lv + 1
    if parts_v:
        v_all, j_all, l_all = (np.concatenate(x) for x in (parts_v, parts_j, parts_l))
        o = np.lexsort((l_all, j_all))
        lower, j_all, l_all = v_all[o], j_all[o], l_all[o]
        brk = np.flatnonzero((j_all[1:] != j_all[:-1]) | (l_all[1:] != l_all[:-1])) + 1
        lvl_slot_off = np.concatenate([[0], brk, [lower.size]])
        lvl_job = j_all[lvl_slot_off[:-1]]
        job_lvl_off = np.searchsorted(lvl_job, np.arange(n_lower + 1))
    else:
        lower = np.zeros(0, np.int64)
        lvl_slot_off = np.zeros(1, np.int64)
        job_lvl_off = np.zeros(1, np.int64)
    n_lower_slots = lower.size
    top_depth = max([L - 1] + depth[np.asarray(jr.promoted, dtype=np.int64)].tolist())
    nlev = min(top_depth + 1, maxd + 1)
    tm = (dvals < nlev) & ((dvals < L) | promoted[slot_nodes])
    tn, td = slot_nodes[tm], dvals[tm]
    o = np.argsort(td, kind="stable")
    top = tn[o]
    top_lvl_off = n_lower_slots + np.searchsorted(td[o], np.arange(nlev + 1))
    slots = np.concatenate([lower, top])
    assert slots.size == slot_nodes.size
    slot_of = np.full(n_nodes, -1, dtype=np.int64)
    slot_of[slots] = np.arange(slots.size)

    # chains: per lower job, the parent chains of its junctions + chains hanging from them
    # (grounded / cycle-closing); the rest (top part chains) go to the jobs (balanced)
    job_of_slot = np.full(slots.size, -1, dtype=np.int64)
    if n_lower:
        lv_len = np.diff(lvl_slot_off)
        job_of_slot[:n_lower_slots] = np.repeat(lvl_job, lv_len)
    chain_job = np.full(E, -1, dtype=np.int64)
    def job_at(nodes):  # the job of a chain end's slot (-1: no junction there)
        sl = slot_of[np.maximum(nodes, 0)]
        out = np.full(nodes.shape, -1, dtype=np.int64)
        ok = (nodes != -1) & (sl >= 0)
        out[ok] = job_of_slot[sl[ok]]
        return out

    jlo, jup = job_at(lo), job_at(up)
    c1 = (lo != -1) & (jlo >= 0)
    chain_job[c1] = jlo[c1]
    c2 = (lo == -1) & (up != -1) & (jup >= 0)
    chain_job[c2] = jup[c2]
    rest = np.flatnonzero(chain_job < 0)
    if n_lower > 0:
        # chains of the top part ride along with the lower jobs: one
        # workgroup per job and no extra jobs, so a launch has exactly n_lower
        # workgroups (<= #CUs); two extra chain-only workgroups started ~10 us late on
        # the GPU (scripts/phase_timing.py)
        if balanced:
            # each to the job with the fewest chains (ties: lowest job), so no job runs an
            # extra chain pass for one chain (8-rank C4: 129-chain jobs, 3 passes of 64 at
            # N = 19, beside 127-chain ones); a job's top chains are top values it reads:
            # past the dense top's K_MAX_NEED the decomposition is rebuilt round-robin
            cnt = np.bincount(chain_job[chain_job >= 0], minlength=n_lower)
            heap = [(int(c), j) for j, c in enumerate(cnt)]
            heapq.heapify(heap)
            for c in rest:
                k, j = heapq.heappop(heap)
                chain_job[c] = j
                heapq.heappush(heap, (k + 1, j))
        else:
            chain_job[rest] = np.arange(rest.size) % n_lower
        n_jobs = n_lower
    else:
        per_job = max(16, int(np.ceil(E / max(1, target_jobs)))) if E else 1
        chain_job[rest] = np.arange(rest.size) // per_job
        n_jobs = int(np.ceil(rest.size / per_job)) if rest.size else 0
    order = np.lexsort((np.arange(E), chain_job))
    job_chain_off = np.searchsorted(chain_job[order], np.arange(n_jobs + 1)).astype(np.int32)
    # chain-only jobs have no levels
    job_lvl_off = np.concatenate([job_lvl_off,
                                  np.full(n_jobs + 1 - job_lvl_off.size, job_lvl_off[-1])])

    chain_index = np.empty(E, dtype=np.int64)
    chain_index[order] = np.arange(E)
    c_up = np.where(up[order] != -1, slot_of[np.maximum(up[order], 0)], -1).astype(np.int32)
    c_lo = np.where(lo[order] != -1, slot_of[np.maximum(lo[order], 0)], -1).astype(np.int32)
    cc = is_cc[order]

    n_slots = slots.size
    slot_lam = lam[slots].astype(np.int32)
    pcs = pchain[slots]
    slot_pchain = np.where(pcs != -1, chain_index[np.maximum(pcs, 0)], -1).astype(np.int32)
    pjs = parent_j[slots]
    slot_parent = np.where(pjs != -1, slot_of[np.maximum(pjs, 0)], -1).astype(np.int32)
    dm = np.flatnonzero((c_up != -1) & ~cc)
    slot_dc_off, o = _csr(c_up[dm].astype(np.int64), n_slots)
    slot_dc = dm[o].astype(np.int32)
    dc_lo = c_lo[slot_dc] if slot_dc.size else np.zeros(0, np.int32)
    slot_plam = np.where(slot_parent >= 0, slot_lam[np.maximum(slot_parent, 0)], -1).astype(np.int32)
    pc = TreePreconditioner(
        N=N, chain_edge=order.astype(np.int32), chain_flip=flip[order].astype(np.int32),
        chain_up=c_up, chain_lo=c_lo, slot_lam=slot_lam, slot_pchain=slot_pchain,
        slot_parent=slot_parent, slot_dc_off=slot_dc_off.astype(np.int32), slot_dc=slot_dc,
        dc_lo=dc_lo.astype(np.int32), slot_plam=slot_plam,
        job_chain_off=job_chain_off, job_lvl_off=np.asarray(job_lvl_off, dtype=np.int32),
        lvl_slot_off=np.asarray(lvl_slot_off, dtype=np.int32),
        top_lvl_off=np.asarray(top_lvl_off, dtype=np.int32), n_jobs=int(n_jobs),
        n_slots=int(n_slots), tree_exact=n_cycle == 0,
        cyc_rows=cyc_rows)
    _dense_top_lists(pc)
    if balanced and n_lower > 0 and pc.job_need_off.size > 1 and \
            int(np.diff(pc.job_need_off).max()) > K_MAX_NEED:
        return build_tree_preconditioner(lp, src, dst, degree, target_jobs, max_top, coarse,
                                         balanced=False)
    if coarse is not None and coarse.n > 0:
        cid = coarse.cidx
        pc.n_coarse = coarse.n
        pc.slot_cidx = cid[slots].astype(np.int32)
        ccs = np.flatnonzero(cc).astype(np.int32)
        pc.cc_chain = ccs
        pc.cc_top = pc.slot_cidx[c_up[ccs]] if ccs.size else _EMPTY_I
        pc.cc_bot = pc.slot_cidx[c_lo[ccs]] if ccs.size else _EMPTY_I
        pc.c_parent = coarse.parent
        pc.c_child_off = coarse.child_off
        pc.c_child = coarse.child
        pc.c_lvl_off = coarse.lvl_off
    return pc


K_MAX_NEED = 128  # csrc/nxhip.hip kMaxNeed: top values one job of the dense top reads


def _dense_top_lists(pc: TreePreconditioner) -> None:
    """Per job: the top slots it owns for updates (round-robin) and the top slots whose
    values it reads (its root's parent, the top ends of its chains, its own top slots)."""
    ts0, ts1 = int(pc.top_lvl_off[0]), int(pc.top_lvl_off[-1])
    nj = pc.n_jobs
    if nj == 0 or ts1 == ts0:
        return
    ts = np.arange(ts0, ts1, dtype=np.int64)
    own_job = (ts - ts0) % nj  # round-robin
    o = np.lexsort((ts, own_job))
    pc.job_tslot = ts[o].astype(np.int32)
    pc.job_tslot_off = np.searchsorted(own_job[o], np.arange(nj + 1)).astype(np.int32)
    # needed top slots per job: its own, the top ends of its chains, its slots' parents
    cj = np.repeat(np.arange(nj, dtype=np.int64), np.diff(pc.job_chain_off))
    sl0 = pc.lvl_slot_off[pc.job_lvl_off[:-1]].astype(np.int64)
    sl1 = pc.lvl_slot_off[pc.job_lvl_off[1:]].astype(np.int64)
    sj = np.repeat(np.arange(nj, dtype=np.int64), np.where(sl1 > sl0, sl1 - sl0, 0))
    sp = pc.slot_parent[:sj.size].astype(np.int64)  # lower slots come first, job-major
    jj = np.concatenate([own_job, cj, cj, sj])
    tt = np.concatenate([ts, pc.chain_up.astype(np.int64), pc.chain_lo.astype(np.int64), sp])
    m = tt >= ts0
    key = np.unique(jj[m] * (ts1 + 1) + tt[m])  # sorted by job, then slot
    pc.job_need = (key % (ts1 + 1)).astype(np.int32)
    pc.job_need_off = np.searchsorted(key // (ts1 + 1), np.arange(nj + 1)).astype(np.int32)
    # producer-side input layout: per top slot [y', I_bot(parent chain), one per dc entry]
    nt = ts1 - ts0
    cnt = np.zeros(nt, dtype=np.int64)
    for t in range(ts0, ts1):
        cnt[t - ts0] = 1 + (pc.slot_pchain[t] >= 0) + (pc.slot_dc_off[t + 1] - pc.slot_dc_off[t])
    uoff = np.zeros(nt + 1, dtype=np.int32)
    np.cumsum(cnt, out=uoff[1:])
    slot_uy = uoff[:-1].copy()
    chain_uit = np.full(pc.n_chains, -1, dtype=np.int32)
    chain_uib = np.full(pc.n_chains, -1, dtype=np.int32)
    job_root_u = np.full(nj, -1, dtype=np.int32)
    job_root_dc = np.full(nj, -1, dtype=np.int32)
    root_job = {}
    for j in range(nj):
        lv0, lv1 = pc.job_lvl_off[j], pc.job_lvl_off[j + 1]
        if lv1 > lv0:
            for sl in range(pc.lvl_slot_off[lv0], pc.lvl_slot_off[lv0 + 1]):
                root_job[sl] = j
    for t in range(ts0, ts1):
        k = uoff[t - ts0] + 1
        if pc.slot_pchain[t] >= 0:
            chain_uib[pc.slot_pchain[t]] = k
            k += 1
        for i in range(pc.slot_dc_off[t], pc.slot_dc_off[t + 1]):
            c, lo = pc.slot_dc[i], pc.dc_lo[i]
            if 0 <= lo < ts0:  # a lower job's root: kappa J_root + I_top, after its levels
                j = root_job[int(lo)]
                assert job_root_u[j] < 0, "one root per job"
                job_root_u[j] = k
                job_root_dc[j] = i
            else:
                chain_uit[c] = k
            k += 1
    pc.top_uoff, pc.slot_uy = uoff, slot_uy.astype(np.int32)
    pc.chain_uit, pc.chain_uib = chain_uit, chain_uib
    pc.job_root_u, pc.job_root_dc = job_root_u, job_root_dc


def top_dense_multi_model(pc: TreePreconditioner, T: np.ndarray, Dj: np.ndarray):
    """Several ranks: (G_loc, KJ, w, rootc) of the dense top with coarse roots held at 0
    (k_pc_gbuild with KJ, k_pc_wroot): z_top = G_loc a + w * zc[rootc], J_root = KJ a."""
    ts0, ts1 = int(pc.top_lvl_off[0]), int(pc.top_lvl_off[-1])
    nt = ts1 - ts0
    G = np.zeros((nt, nt))
    KJ = np.zeros((nt, nt))
    lv = pc.top_lvl_off
    for s in range(nt):
        J = np.zeros(nt)
        J[s] = 1.0
        t = ts0 + s
        while pc.slot_parent[t] >= ts0:
            p = pc.slot_parent[t]
            J[p - ts0] += J[t - ts0] / T[pc.slot_pchain[t]] / Dj[t]
            t = p
        if pc.slot_cidx[t] >= 0:
            KJ[t - ts0, s] = J[t - ts0]
        z = np.zeros(nt)
        for li in range(lv.size - 1):
            for u in range(lv[li], lv[li + 1]):
                p = pc.slot_parent[u]
                if p < ts0 and pc.slot_cidx[u] >= 0:
                    z[u - ts0] = 0.0
                    continue
                num = J[u - ts0] + (z[p - ts0] / T[pc.slot_pchain[u]] if p >= ts0 else 0.0)
                z[u - ts0] = num / Dj[u]
        G[:, s] = z
    w = np.zeros(nt)
    rootc = np.full(nt, -1)
    for li in range(lv.size - 1):
        for t in range(lv[li], lv[li + 1]):
            p = pc.slot_parent[t]
            if p < ts0:
                rootc[t - ts0] = pc.slot_cidx[t]
                w[t - ts0] = 1.0 if pc.slot_cidx[t] >= 0 else 0.0
            else:
                rootc[t - ts0] = rootc[p - ts0]
                w[t - ts0] = w[p - ts0] / T[pc.slot_pchain[t]] / Dj[t]
    return G, KJ, w, rootc


def top_inverse_model(pc: TreePreconditioner, T: np.ndarray, Dj: np.ndarray) -> np.ndarray:
    """G (n_top x n_top): column s = the top part's response to a unit J at top slot s
    (J up the ancestors with kappa = g_up / D, then the root-to-leaf back-substitution),
    i.e. the inverse of the top tree Schur matrix (k_pc_gbuild)."""
    ts0, ts1 = int(pc.top_lvl_off[0]), int(pc.top_lvl_off[-1])
    nt = ts1 - ts0
    G = np.zeros((nt, nt))
    lv = pc.top_lvl_off
    for s in range(nt):
        J = np.zeros(nt)
        J[s] = 1.0
        t = ts0 + s
        while pc.slot_parent[t] >= ts0:  # ancestors inside the top part
            p = pc.slot_parent[t]
            J[p - ts0] += J[t - ts0] / T[pc.slot_pchain[t]] / Dj[t]
            t = p
        z = np.zeros(nt)
        for li in range(lv.size - 1):
            for u in range(lv[li], lv[li + 1]):
                p = pc.slot_parent[u]
                num = J[u - ts0] + (z[p - ts0] / T[pc.slot_pchain[u]] if p >= ts0 else 0.0)
                z[u - ts0] = num / Dj[u]
        G[:, s] = z
    return G


# ----------------------------------------------------------------------------- model
def lumped_mass(Ab, lp) -> np.ndarray:
    """Lumped flux mass per edge, ``(E, N+1)``, from the assembled build-layout matrix."""
    N, per = lp.N, 2 * lp.N + 1
    E = lp.edges.size
    rows = (np.arange(E)[:, None] * per + 2 * np.arange(N + 1)[None, :]).ravel()
    sub = Ab[rows]
    d = np.zeros(rows.size)
    for i, r in enumerate(rows):
        s, e = sub.indptr[i], sub.indptr[i + 1]
        cols = sub.indices[s:e]
        vals = sub.data[s:e]
        mask = (cols < E * per) & ((cols % per) % 2 == 0)  # flux columns
        d[i] = np.abs(vals[mask]).sum()
    return d.reshape(E, N + 1)


def mass_tinv(N: int) -> np.ndarray:
    """``T^{-1}`` for the P1 mass of one edge, ``M_e = (R h / 6) T``, ``T = tridiag(1, 4, 1)``
    of size N+1 with 2 at both ends (``assembly.py:253`` on N equal cells)."""
    T = (np.diag(np.r_[2.0, np.full(N - 1, 4.0), 2.0]) if N > 0 else np.eye(1))
    T += np.diag(np.ones(N), 1) + np.diag(np.ones(N), -1)
    Ti = np.linalg.inv(T)
    return 0.5 * (Ti + Ti.T)


def apply_model(pc: TreePreconditioner, lp, dq: np.ndarray, r: np.ndarray,
                exact: bool = True) -> np.ndarray:
    """numpy model of the device application ``z = P^{-1} r`` on one rank (no coarse
    exchange: with several ranks use :func:`pc_up_model` / :func:`pc_finish_model` around
    a sum of the partials over ranks). ``exact``: consistent flux mass (the device
    default), else the lumped one."""
    st = pc_up_model(pc, lp, dq, r)
    return pc_finish_model(pc, lp, dq, st, st["partial"], exact=exact)


def _chain_dofs(pc, dq, c):
    N, per = pc.N, 2 * pc.N + 1
    e = pc.chain_edge[c]
    base = e * per
    cells = base + 2 * np.arange(N) + 1
    qs = base + 2 * np.arange(N + 1)
    rho = dq[e].copy()
    if pc.chain_flip[c]:
        cells, qs, rho = cells[::-1], qs[::-1], rho[::-1]
    return cells, qs, rho


def pc_up_model(pc: TreePreconditioner, lp, dq: np.ndarray, r: np.ndarray) -> dict:
    """Chain condensation and junction elimination (k_pc_up + the top elimination);
    returns the state and this rank's coarse partial ``[D | J | G]`` (length 3 nC)."""
    N = pc.N
    n_col = lp.n_own + lp.n_ghost
    rr = np.zeros(n_col)
    rr[:r.size] = r
    T = np.zeros(pc.n_chains)
    It = np.zeros(pc.n_chains)
    Ib = np.zeros(pc.n_chains)
    for c in range(pc.n_chains):
        cells, qs, rho = _chain_dofs(pc, dq, c)
        Dk = np.cumsum(rho)[:N]
        T[c] = rho.sum()
        rp = rr[cells]
        It[c] = np.sum(rp * (T[c] - Dk)) / T[c]
        Ib[c] = np.sum(rp * Dk) / T[c]
    Dj = np.zeros(pc.n_slots)
    Jj = np.zeros(pc.n_slots)

    def eliminate(j):
        pcn = pc.slot_pchain[j]
        D = 1.0 / T[pcn] if pcn >= 0 else 0.0
        J = rr[pc.slot_lam[j]] + (Ib[pcn] if pcn >= 0 else 0.0)
        for c in pc.slot_dc[pc.slot_dc_off[j]:pc.slot_dc_off[j + 1]]:
            g = 1.0 / T[c]
            J += It[c]
            lo = pc.chain_lo[c]
            if lo >= 0:
                D += g * (1.0 - g / Dj[lo])
                J += g * Jj[lo] / Dj[lo]
            else:
                D += g
        Dj[j], Jj[j] = D, J

    # lower jobs bottom-up, then top levels bottom-up
    for jb in range(pc.n_jobs):
        lv0, lv1 = pc.job_lvl_off[jb], pc.job_lvl_off[jb + 1]
        for lv in range(lv1 - 1, lv0 - 1, -1):
            for j in range(pc.lvl_slot_off[lv], pc.lvl_slot_off[lv + 1]):
                eliminate(j)
    tl = pc.top_lvl_off
    for lv in range(tl.size - 2, -1, -1):
        for j in range(tl[lv], tl[lv + 1]):
            eliminate(j)
    nC = pc.n_coarse
    partial = np.zeros(3 * nC)
    for j in np.flatnonzero(pc.slot_cidx >= 0) if nC else []:
        k = pc.slot_cidx[j]
        partial[k] += Dj[j]
        partial[nC + k] += Jj[j]
    for c, t, b in zip(pc.cc_chain, pc.cc_top, pc.cc_bot):
        g = 1.0 / T[c]
        partial[t] += g
        partial[b] += g
        partial[nC + t] += It[c]
        partial[nC + b] += Ib[c]
        partial[2 * nC + b] = g
    return dict(r=rr, T=T, Dj=Dj, Jj=Jj, partial=partial)


def coarse_solve_model(pc: TreePreconditioner, total: np.ndarray) -> np.ndarray:
    """Tree elimination on the coarse forest from the summed partials (k_pc_coarse)."""
    nC = pc.n_coarse
    D = total[:nC].copy()
    J = total[nC:2 * nC].copy()
    G = total[2 * nC:3 * nC]
    lo = pc.c_lvl_off
    for lv in range(lo.size - 2, -1, -1):
        for j in range(lo[lv], lo[lv + 1]):
            for k in pc.c_child[pc.c_child_off[j]:pc.c_child_off[j + 1]]:
                D[j] -= G[k] * G[k] / D[k]
                J[j] += G[k] * J[k] / D[k]
    zc = np.zeros(nC)
    for lv in range(lo.size - 1):
        for j in range(lo[lv], lo[lv + 1]):
            p = pc.c_parent[j]
            zc[j] = (J[j] + (G[j] * zc[p] if p >= 0 else 0.0)) / D[j]
    return zc


def pc_finish_model(pc: TreePreconditioner, lp, dq: np.ndarray, st: dict,
                    total: np.ndarray, exact: bool = True) -> np.ndarray:
    """Coarse solve, back-substitution and chain cells (k_pc_coarse / top + k_pc_down).
    Returns z on the owned DoFs. ``exact``: the consistent-mass variant (module doc)."""
    N = pc.N
    Ti = mass_tinv(N) if exact else None
    rr, T, Dj, Jj = st["r"], st["T"], st["Dj"], st["Jj"]
    z = np.zeros_like(rr)
    zc = coarse_solve_model(pc, total) if pc.n_coarse else np.zeros(0)
    zj = np.zeros(pc.n_slots)

    def back(j):
        p = pc.slot_parent[j]
        if pc.n_coarse and pc.slot_cidx[j] >= 0:
            zj[j] = zc[pc.slot_cidx[j]]
        elif p < 0:
            zj[j] = Jj[j] / Dj[j]
        else:
            zj[j] = (Jj[j] + zj[p] / T[pc.slot_pchain[j]]) / Dj[j]
        z[pc.slot_lam[j]] = zj[j]

    tl = pc.top_lvl_off
    for lv in range(tl.size - 1):
        for j in range(tl[lv], tl[lv + 1]):
            back(j)
    for jb in range(pc.n_jobs):
        lv0, lv1 = pc.job_lvl_off[jb], pc.job_lvl_off[jb + 1]
        for lv in range(lv0, lv1):
            for j in range(pc.lvl_slot_off[lv], pc.lvl_slot_off[lv + 1]):
                back(j)
    for c in range(pc.n_chains):
        cells, qs, rho = _chain_dofs(pc, dq, c)
        Dk = np.cumsum(rho)[:N]
        Tc = T[c]
        rp = rr[cells]
        zt = zj[pc.chain_up[c]] if pc.chain_up[c] >= 0 else 0.0
        zb = zj[pc.chain_lo[c]] if pc.chain_lo[c] >= 0 else 0.0
        a = (Tc - Dk) * rp  # suffix sums j >= k
        suf = np.cumsum(a[::-1])[::-1]
        b = Dk * rp  # prefix sums j < k
        pre = np.concatenate([[0.0], np.cumsum(b)[:-1]])
        z[cells] = zt * (Tc - Dk) / Tc + zb * Dk / Tc + (Dk / Tc) * suf + ((Tc - Dk) / Tc) * pre
        if exact:
            mo = rho[0] / 3.0  # R h / 6
            z[cells] -= mo * rp
            z[qs] = (Ti @ rr[qs]) / mo
        else:
            z[qs] = rr[qs] / rho
    return z[:lp.n_own]
