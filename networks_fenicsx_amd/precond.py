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
are processed by extra chain-only jobs in the same kernels.

Graphs that are not trees, and ranks of a partitioned problem, use the same machinery on
a spanning forest: a chain that would close a cycle, or whose far end is a junction owned
by another rank, is grounded at that end. ``P`` stays SPD (a grounded Laplacian block);
only its quality drops.
"""

from __future__ import annotations

from collections import deque
from dataclasses import dataclass

import numpy as np

__all__ = ["TreePreconditioner", "build_tree_preconditioner", "apply_model"]


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
    # jobs: lower subtrees first (chains + junction levels), then chain-only jobs
    job_chain_off: np.ndarray  # n_jobs + 1
    job_lvl_off: np.ndarray  # n_jobs + 1, offsets into lvl_slot_off
    lvl_slot_off: np.ndarray  # slot offsets of every level (per job, root level first)
    # top part (one workgroup): junction slots [top_slot0, top_slot1), levels
    top_lvl_off: np.ndarray  # slot offsets of the top levels (root level first)
    n_jobs: int
    n_slots: int

    @property
    def n_chains(self) -> int:
        return int(self.chain_edge.size)


def build_tree_preconditioner(lp, src: np.ndarray, dst: np.ndarray, degree: np.ndarray,
                              target_jobs: int = 256, max_top: int = 1024) -> TreePreconditioner:
    """Decompose the rank-local problem ``lp`` (:class:`layout.LocalProblem`).

    ``src``/``dst`` are the global node ids of all edges, ``degree`` the global degrees.
    """
    N = lp.N
    E = lp.edges.size
    es, ed = src[lp.edges], dst[lp.edges]
    # owned junctions: node -> slot candidate
    owned = {int(v): i for i, v in enumerate(lp.lm_nodes)}
    lam_of = {int(v): lp.n_edge_dofs + i for i, v in enumerate(lp.lm_nodes)}
    is_j = lambda v: v in owned  # noqa: E731
    # junction adjacency through local edges
    adj: dict[int, list[tuple[int, int]]] = {v: [] for v in owned}
    for e in range(E):
        a, b = int(es[e]), int(ed[e])
        if is_j(a):
            adj[a].append((e, b))
        if is_j(b):
            adj[b].append((e, a))

    # spanning forest: BFS from junctions touching ground first (they become roots)
    depth = {}
    parent_j = {}
    pchain = {}
    tree_edge = np.zeros(E, dtype=bool)
    ground_touch = [v for v in lp.lm_nodes.tolist() if any(not is_j(w) for _, w in adj[v])]
    order_roots = ground_touch + lp.lm_nodes.tolist()
    for r in order_roots:
        r = int(r)
        if r in depth:
            continue
        depth[r] = 0
        parent_j[r] = -1
        pchain[r] = -1
        q = deque([r])
        while q:
            u = q.popleft()
            for e, w in adj[u]:
                if is_j(w) and w not in depth:
                    depth[w] = depth[u] + 1
                    parent_j[w] = u
                    pchain[w] = e
                    tree_edge[e] = True
                    q.append(w)

    # chain ends: top = parent side (junction or ground), bottom = other
    chain_up_node = np.full(E, -1, dtype=np.int64)
    chain_lo_node = np.full(E, -1, dtype=np.int64)
    flip = np.zeros(E, dtype=np.int8)
    for e in range(E):
        a, b = int(es[e]), int(ed[e])
        ja, jb = is_j(a), is_j(b)
        if tree_edge[e]:
            # the child is the endpoint whose parent chain is e
            if jb and pchain.get(b) == e:
                up, lo = a, b
            else:
                up, lo = b, a
        elif ja and jb:  # closes a cycle: hang from the shallower end, ground the other
            up, lo = (a, -1) if depth[a] <= depth[b] else (b, -1)
        elif ja:
            up, lo = a, -1
        elif jb:
            up, lo = b, -1
        else:
            up, lo = -1, -1
        chain_up_node[e] = up
        chain_lo_node[e] = lo
        flip[e] = 1 if (up == b and up != -1) or (up == -1 and lo == a and lo != -1) else 0

    # cut depth: lower subtrees rooted at depth L
    dvals = np.array([depth[int(v)] for v in lp.lm_nodes], dtype=np.int64)
    maxd = int(dvals.max()) if dvals.size else -1
    counts = np.bincount(dvals, minlength=maxd + 1) if dvals.size else np.zeros(0, np.int64)
    L = maxd + 1  # default: everything in the top part
    for cand in range(maxd + 1):
        if counts[cand] >= target_jobs or counts[:cand].sum() + counts[cand] > max_top:
            L = cand
            break
    if dvals.size and counts[:L].sum() > max_top:
        L = max(0, L)

    children: dict[int, list[int]] = {v: [] for v in owned}
    for v in lp.lm_nodes.tolist():
        p = parent_j[v]
        if p != -1:
            children[p].append(v)

    # slots: lower subtrees (level order inside), then top levels
    slots: list[int] = []
    job_lvl_off = [0]
    lvl_slot_off = [0]
    job_roots = [v for v in lp.lm_nodes.tolist() if depth[v] == L]
    for r in job_roots:
        level = [r]
        while level:
            slots.extend(level)
            lvl_slot_off.append(len(slots))
            level = [c for u in level for c in children[u]]
        job_lvl_off.append(len(lvl_slot_off) - 1)
    n_lower_slots = len(slots)
    top_lvl_off = [n_lower_slots]
    for dlev in range(L):
        level = [v for v in lp.lm_nodes.tolist() if depth[v] == dlev]
        # keep siblings together (parents' order) for locality
        slots.extend(level)
        top_lvl_off.append(len(slots))
    assert len(slots) == len(lp.lm_nodes)
    slot_of = {v: i for i, v in enumerate(slots)}

    # chains: per lower job, the parent chains of its junctions + chains hanging from them
    # (grounded / cycle-closing); then chain-only jobs for the rest (top part chains)
    job_of_slot = np.full(len(slots), -1, dtype=np.int64)
    for j in range(len(job_roots)):
        a = lvl_slot_off[job_lvl_off[j]]
        b = lvl_slot_off[job_lvl_off[j + 1]]
        job_of_slot[a:b] = j
    chain_job = np.full(E, -1, dtype=np.int64)
    for e in range(E):
        lo, up = chain_lo_node[e], chain_up_node[e]
        if lo != -1 and job_of_slot[slot_of[lo]] >= 0:
            chain_job[e] = job_of_slot[slot_of[lo]]
        elif lo == -1 and up != -1 and job_of_slot[slot_of[up]] >= 0:
            chain_job[e] = job_of_slot[slot_of[up]]
    n_lower = len(job_roots)
    rest = np.flatnonzero(chain_job < 0)
    per_job = max(1, int(np.ceil(E / max(1, target_jobs)))) if E else 1
    per_job = max(per_job, 16)
    for i, e in enumerate(rest):
        chain_job[e] = n_lower + i // per_job
    n_jobs = n_lower + (int(np.ceil(rest.size / per_job)) if rest.size else 0)
    order = np.lexsort((np.arange(E), chain_job))
    job_chain_off = np.searchsorted(chain_job[order], np.arange(n_jobs + 1)).astype(np.int32)
    # chain-only jobs have no levels
    while len(job_lvl_off) < n_jobs + 1:
        job_lvl_off.append(job_lvl_off[-1])

    chain_index = np.empty(E, dtype=np.int64)
    chain_index[order] = np.arange(E)
    to_slot = lambda v: slot_of[int(v)] if v != -1 else -1  # noqa: E731
    c_up = np.array([to_slot(chain_up_node[e]) for e in order], dtype=np.int32)
    c_lo = np.array([to_slot(chain_lo_node[e]) for e in order], dtype=np.int32)

    n_slots = len(slots)
    slot_lam = np.array([lam_of[v] for v in slots], dtype=np.int32)
    slot_pchain = np.array([chain_index[pchain[v]] if pchain[v] != -1 else -1 for v in slots],
                           dtype=np.int32)
    slot_parent = np.array([slot_of[parent_j[v]] if parent_j[v] != -1 else -1 for v in slots],
                           dtype=np.int32)
    down = [[] for _ in range(n_slots)]
    for c in range(E):
        if c_up[c] != -1:
            down[c_up[c]].append(c)
    slot_dc_off = np.zeros(n_slots + 1, dtype=np.int32)
    np.cumsum([len(d) for d in down], out=slot_dc_off[1:])
    slot_dc = np.array([c for d in down for c in d], dtype=np.int32)
    dc_lo = c_lo[slot_dc] if slot_dc.size else np.zeros(0, np.int32)
    slot_plam = np.where(slot_parent >= 0, slot_lam[np.maximum(slot_parent, 0)], -1).astype(np.int32)
    return TreePreconditioner(
        N=N, chain_edge=order.astype(np.int32), chain_flip=flip[order].astype(np.int32),
        chain_up=c_up, chain_lo=c_lo, slot_lam=slot_lam, slot_pchain=slot_pchain,
        slot_parent=slot_parent, slot_dc_off=slot_dc_off, slot_dc=slot_dc,
        dc_lo=dc_lo.astype(np.int32), slot_plam=slot_plam,
        job_chain_off=job_chain_off, job_lvl_off=np.asarray(job_lvl_off, dtype=np.int32),
        lvl_slot_off=np.asarray(lvl_slot_off, dtype=np.int32),
        top_lvl_off=np.asarray(top_lvl_off, dtype=np.int32), n_jobs=int(n_jobs),
        n_slots=n_slots)


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


def apply_model(pc: TreePreconditioner, lp, dq: np.ndarray, r: np.ndarray) -> np.ndarray:
    """numpy model of the device application ``z = P^{-1} r`` (same decomposition)."""
    N, per = pc.N, 2 * pc.N + 1
    z = np.zeros_like(r)
    T = np.zeros(pc.n_chains)
    It = np.zeros(pc.n_chains)
    Ib = np.zeros(pc.n_chains)
    Dc = np.zeros(pc.n_chains * N)

    def chain_dofs(c):
        e = pc.chain_edge[c]
        base = e * per
        cells = base + 2 * np.arange(N) + 1
        qs = base + 2 * np.arange(N + 1)
        rho = dq[e].copy()
        if pc.chain_flip[c]:
            cells, qs, rho = cells[::-1], qs[::-1], rho[::-1]
        return cells, qs, rho

    for c in range(pc.n_chains):
        cells, qs, rho = chain_dofs(c)
        Dk = np.cumsum(rho)[:N]
        T[c] = rho.sum()
        rp = r[cells]
        It[c] = np.sum(rp * (T[c] - Dk)) / T[c]
        Ib[c] = np.sum(rp * Dk) / T[c]
    Dj = np.zeros(pc.n_slots)
    Jj = np.zeros(pc.n_slots)

    def eliminate(j):
        pcn = pc.slot_pchain[j]
        D = 1.0 / T[pcn] if pcn >= 0 else 0.0
        J = r[pc.slot_lam[j]] + (Ib[pcn] if pcn >= 0 else 0.0)
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
    zj = np.zeros(pc.n_slots)

    def back(j):
        p = pc.slot_parent[j]
        if p < 0:
            zj[j] = Jj[j] / Dj[j]
        else:
            zj[j] = (Jj[j] + zj[p] / T[pc.slot_pchain[j]]) / Dj[j]
        z[pc.slot_lam[j]] = zj[j]

    for lv in range(tl.size - 1):
        for j in range(tl[lv], tl[lv + 1]):
            back(j)
    for jb in range(pc.n_jobs):
        lv0, lv1 = pc.job_lvl_off[jb], pc.job_lvl_off[jb + 1]
        for lv in range(lv0, lv1):
            for j in range(pc.lvl_slot_off[lv], pc.lvl_slot_off[lv + 1]):
                back(j)
    for c in range(pc.n_chains):
        cells, qs, rho = chain_dofs(c)
        Dk = np.cumsum(rho)[:N]
        Tc = T[c]
        rp = r[cells]
        zt = zj[pc.chain_up[c]] if pc.chain_up[c] >= 0 else 0.0
        zb = zj[pc.chain_lo[c]] if pc.chain_lo[c] >= 0 else 0.0
        a = (Tc - Dk) * rp  # suffix sums j >= k
        suf = np.cumsum(a[::-1])[::-1]
        b = Dk * rp  # prefix sums j < k
        pre = np.concatenate([[0.0], np.cumsum(b)[:-1]])
        z[cells] = zt * (Tc - Dk) / Tc + zb * Dk / Tc + (Dk / Tc) * suf + ((Tc - Dk) / Tc) * pre
        z[qs] = r[qs] / rho
    return z
