"""Preconditioner host decomposition and its numpy model (CPU)."""

from __future__ import annotations

import numpy as np
import pytest

from cases import CASES, lattice_graph
from networks_fenicsx_amd import NetworkMesh
from networks_fenicsx_amd import network_generation as ng
from networks_fenicsx_amd.layout import build_local_problem
from networks_fenicsx_amd.precond import (apply_model, build_tree_preconditioner, coarse_solve_model,
                                          lumped_mass, pc_finish_model, pc_up_model,
                                          top_dense_multi_model, top_inverse_model)
from oracle import nx_oracle as O


def _problem(G, N, strategy=None):
    m = NetworkMesh(G, N=N, color_strategy=strategy)
    src, dst = m.edges
    P = O.build_problem(m.node_coordinates, src, dst, N, m.edge_colors)
    A, b = O.assemble_reference(P, lambda x: x[1])
    Ab, bb, perm, sign = O.to_build_layout(P, A, b)
    lp = build_local_problem(m.node_coordinates, src, dst, m.degrees, N)
    return m, Ab, lp


@pytest.mark.parametrize("case", ["depth6_N40", "arterial5_N40", "tree6_2d_N70", "Y_N4"])
@pytest.mark.parametrize("jobs", [4, 16, 256])
@pytest.mark.parametrize("exact", [False, True])
def test_exact_schur_solve_on_trees(case, jobs, exact):
    """P^{-1} from the decomposition equals a direct solve of blockdiag(D, G^T D^-1 G)
    (lumped) or of blockdiag(M, G^T M^-1 G) (consistent mass, the exact Schur complement)."""
    make, N, strategy, _ = CASES[case]
    m, Ab, lp = _problem(make(), N, strategy)
    src, dst = m.edges
    pc = build_tree_preconditioner(lp, src, dst, m.degrees, target_jobs=jobs)
    dq = lumped_mass(Ab, lp)
    n = Ab.shape[0]
    per = 2 * N + 1
    E = lp.edges.size
    qrows = (np.arange(E)[:, None] * per + 2 * np.arange(N + 1)[None, :]).ravel()
    other = np.setdiff1d(np.arange(n), qrows)
    Dq = dq.ravel()
    Gm = Ab[qrows][:, other].toarray()
    r = np.random.default_rng(3).standard_normal(n)
    z = apply_model(pc, lp, dq, r, exact=exact)
    if exact:
        M = Ab[qrows][:, qrows].toarray()
        S = Gm.T @ np.linalg.solve(M, Gm)
        zq = np.linalg.solve(M, r[qrows])
        assert np.linalg.norm(z[qrows] - zq) <= 1e-12 * np.linalg.norm(zq)
    else:
        S = Gm.T @ (Gm / Dq[:, None])
        np.testing.assert_allclose(z[qrows], r[qrows] / Dq, rtol=1e-13)
    zs = np.linalg.solve(S, r[other])
    assert np.linalg.norm(z[other] - zs) <= 1e-11 * np.linalg.norm(zs)


@pytest.mark.parametrize("case", ["depth6_N40", "arterial5_N40", "Y_N4"])
def test_exact_preconditioner_three_iterations(case):
    """With the consistent-mass Schur complement, P^{-1} A has three distinct eigenvalues
    (Murphy-Golub-Wathen): preconditioned MINRES reaches the direct solution in 3 steps."""
    import scipy.sparse.linalg as spla

    make, N, strategy, _ = CASES[case]
    m, Ab, lp = _problem(make(), N, strategy)
    src, dst = m.edges
    pc = build_tree_preconditioner(lp, src, dst, m.degrees, target_jobs=16)
    dq = lumped_mass(Ab, lp)
    n = Ab.shape[0]
    b = np.random.default_rng(5).standard_normal(n)
    x_direct = spla.spsolve(Ab.tocsc(), b)
    its = [0]

    def count(_x):
        its[0] += 1

    P = spla.LinearOperator((n, n), matvec=lambda r: apply_model(pc, lp, dq, r, exact=True))
    x, info = spla.minres(Ab, b, M=P, rtol=1e-12, maxiter=50, callback=count)
    assert info == 0 and its[0] <= 4
    assert np.linalg.norm(x - x_direct) <= 1e-10 * np.linalg.norm(x_direct)


@pytest.mark.parametrize("depth,jobs", [(6, 8), (8, 16), (9, 64)])
def test_dense_top_inverse_matches_back_substitution(depth, jobs):
    """z of the top slots = G a (k_pc_down's dense top) with a_s = J_s minus the top
    children's eliminated contributions."""
    m, Ab, lp = _problem(ng.make_tree(depth, depth, depth), 7)
    src, dst = m.edges
    pc = build_tree_preconditioner(lp, src, dst, m.degrees, target_jobs=jobs)
    dq = lumped_mass(Ab, lp)
    ts0, ts1 = int(pc.top_lvl_off[0]), int(pc.top_lvl_off[-1])
    assert ts1 > ts0 and pc.n_jobs > 0
    r = np.random.default_rng(1).standard_normal(lp.n_own)
    st = pc_up_model(pc, lp, dq, r)
    z = pc_finish_model(pc, lp, dq, st, st["partial"])
    T, Dj, Jj = st["T"], st["Dj"], st["Jj"]
    a = Jj[ts0:ts1].copy()
    for t in range(ts0, ts1):
        p = pc.slot_parent[t]
        if p >= ts0:
            a[p - ts0] -= Jj[t] / T[pc.slot_pchain[t]] / Dj[t]
    G = top_inverse_model(pc, T, Dj)
    zt = G @ a
    np.testing.assert_allclose(zt, z[pc.slot_lam[ts0:ts1]], rtol=1e-12, atol=1e-14)
    # every job's needed list covers its root's parent, its chain ends and its own slots
    for j in range(pc.n_jobs):
        need = set(pc.job_need[pc.job_need_off[j]:pc.job_need_off[j + 1]].tolist())
        own = pc.job_tslot[pc.job_tslot_off[j]:pc.job_tslot_off[j + 1]].tolist()
        assert set(own) <= need
        for c in range(pc.job_chain_off[j], pc.job_chain_off[j + 1]):
            for e in (pc.chain_up[c], pc.chain_lo[c]):
                assert e < ts0 or e in need
    assert sorted(pc.job_tslot.tolist()) == list(range(ts0, ts1))
    # producer-side input layout reproduces a_s
    u = np.zeros(int(pc.top_uoff[-1]))
    rr = st["r"]
    for t in range(ts0, ts1):
        u[pc.slot_uy[t - ts0]] = rr[pc.slot_lam[t]]
    It = np.zeros(pc.n_chains)
    Ib = np.zeros(pc.n_chains)
    N = pc.N
    for c in range(pc.n_chains):  # recompute the chain currents of the model
        e = pc.chain_edge[c]
        cells = e * (2 * N + 1) + 2 * np.arange(N) + 1
        rho = dq[e][::-1] if pc.chain_flip[c] else dq[e]
        cells = cells[::-1] if pc.chain_flip[c] else cells
        Dk = np.cumsum(rho)[:N]
        Ib[c] = np.sum(rr[cells] * Dk) / T[c]
        It[c] = np.sum(rr[cells] * (T[c] - Dk)) / T[c]
        if pc.chain_uit[c] >= 0:
            u[pc.chain_uit[c]] = It[c]
        if pc.chain_uib[c] >= 0:
            u[pc.chain_uib[c]] = Ib[c]
    for j in range(pc.n_jobs):
        if pc.job_root_u[j] >= 0:
            i = pc.job_root_dc[j]
            root = pc.dc_lo[i]
            c = pc.slot_dc[i]
            u[pc.job_root_u[j]] = It[c] + Jj[root] / T[c] / Dj[root]
    a_u = np.add.reduceat(u, pc.top_uoff[:-1]) if u.size else u
    np.testing.assert_allclose(a_u, a, rtol=1e-12, atol=1e-14)


@pytest.mark.parametrize("case,P", [("depth6_N40", 2), ("depth6_N40", 4), ("arterial5_N40", 3)])
def test_dense_top_several_ranks(case, P):
    """Several ranks: coarse partial J = KJ a, top values = G_loc a + w zc[root] against
    the exact multi-rank back-substitution of the model."""
    make, N, strategy, _ = CASES[case]
    m, Ab, lp1 = _problem(make(), N, strategy)
    src, dst = m.edges
    dqg = lumped_mass(Ab, lp1)
    lps = [build_local_problem(m.node_coordinates, src, dst, m.degrees, N, r, P) for r in range(P)]
    pcs = [build_tree_preconditioner(lp, src, dst, m.degrees) for lp in lps]
    rng = np.random.default_rng(5)
    sts = []
    for lp, pc in zip(lps, pcs):
        sts.append(pc_up_model(pc, lp, dqg[lp.edges], rng.standard_normal(lp.n_own)))
    total = sum(st["partial"] for st in sts)
    zc = coarse_solve_model(pcs[0], total)
    for lp, pc, st in zip(lps, pcs, sts):
        z = pc_finish_model(pc, lp, dqg[lp.edges], st, total)
        T, Dj, Jj = st["T"], st["Dj"], st["Jj"]
        ts0, ts1 = int(pc.top_lvl_off[0]), int(pc.top_lvl_off[-1])
        a = Jj[ts0:ts1].copy()
        for t in range(ts0, ts1):
            p = pc.slot_parent[t]
            if p >= ts0:
                a[p - ts0] -= Jj[t] / T[pc.slot_pchain[t]] / Dj[t]
        G, KJ, w, rootc = top_dense_multi_model(pc, T, Dj)
        roots = [t - ts0 for t in range(ts0, ts1)
                 if pc.slot_parent[t] < ts0 and pc.slot_cidx[t] >= 0]
        assert roots
        np.testing.assert_allclose((KJ @ a)[roots], Jj[ts0:ts1][roots], rtol=1e-12, atol=1e-13)
        zt = G @ a + np.where(rootc >= 0, w * zc[np.maximum(rootc, 0)], 0.0)
        zfull = np.zeros(lp.n_own + lp.n_ghost)
        zfull[:lp.n_own] = z
        own = pc.slot_lam[ts0:ts1] < lp.n_own
        np.testing.assert_allclose(zt[own], zfull[pc.slot_lam[ts0:ts1]][own], rtol=1e-11,
                                   atol=1e-13)


def _decomposition(levels, N, P, jobs):
    G = ng.make_tree(levels, levels, levels)
    mesh = NetworkMesh(G, N=N, color_strategy=None)
    src, dst = mesh.edges
    out = []
    for r in range(P):
        lp = build_local_problem(mesh.node_coordinates, src, dst, mesh.degrees, N, r, P)
        out.append(build_tree_preconditioner(lp, src, dst, mesh.degrees, target_jobs=jobs))
    return out


def test_single_rank_depth_cut_unchanged():
    """One rank, uniform binary tree: every job is one depth-L subtree of equal size."""
    (pc,) = _decomposition(9, 4, 1, 32)
    assert pc.n_jobs == 32
    assert np.unique(np.diff(pc.job_chain_off)).size <= 2  # top chains ride round-robin


@pytest.mark.parametrize("P", [4, 8])
def test_several_ranks_balanced_jobs(P):
    """Several ranks: the local forest's pieces differ in height; the largest-first split
    keeps every rank at <= target_jobs jobs (one workgroup per CU) -- the depth cut gave
    1.5x the target on some ranks and, at the 8-GPU bench size, a job over the LDS chain
    cap on half the ranks (those then ran a different kernel schedule: ranks diverged)."""
    jobs = 32
    for pc in _decomposition(12, 3, P, jobs):
        assert 0 < pc.n_jobs <= jobs
        cpj = np.diff(pc.job_chain_off)
        assert cpj.max() <= 512


def test_split_job_roots_promotes_over_cap():
    from networks_fenicsx_amd.precond import _CAP_CHAINS, _split_job_roots

    # root 0 with two children; 600 chains hang below child 1 -> root 0 is over the cap.
    # Subtree sizes (chains, slots, down-chain entries): chains whose bottom (else top)
    # end is the junction, plus the children's
    children = {0: [1, 2], 1: [], 2: []}
    s_ch = np.array([1 + 601 + 98, 601, 98])
    s_sl = np.array([3, 1, 1])
    s_dc = np.array([2 + 600 + 97, 600, 97])
    res = _split_job_roots([0], children.__getitem__, (s_ch, s_sl, s_dc), n_top=0,
                           max_top=1024)
    assert res.promoted == [0] and res.roots == [1, 2]
    assert 601 > _CAP_CHAINS  # child 1 stays over the cap: a leaf junction cannot split


def direct_model(pc, lp, dq, Ab, b):
    """The device's direct tree solve (csrc/nxhip.hip k_dir_*), restated with the
    preconditioner model: y = M^{-1} b_q, x_s = S^{-1}(K^T y - b_s), x_q = M^{-1}(b_q - K x_s)."""
    per = 2 * lp.N + 1
    rows = np.arange(Ab.shape[0])
    flux = (rows < lp.n_edge_dofs) & (rows % per % 2 == 0)
    y = apply_model(pc, lp, dq, np.where(flux, b, 0.0), exact=True)
    w = np.where(flux, 0.0, Ab @ np.where(flux, y, 0.0) - b)
    xs = apply_model(pc, lp, dq, w, exact=True)
    t = np.where(flux, b - Ab @ np.where(flux, 0.0, xs), 0.0)
    xq = apply_model(pc, lp, dq, t, exact=True)
    return np.where(flux, xq, xs)


@pytest.mark.parametrize("case", ["depth6_N40", "arterial5_N40", "tree6_2d_N70", "Y_N4",
                                  "demo_tree_N1", "linear_alt_N3", "edge_info_N10"])
def test_direct_tree_solve_model(case):
    """Block LU with the exact Schur complement: equals the sparse direct solve on trees
    (tree_exact); the cycle graph's decomposition grounds a chain (not tree_exact) and the
    same formula is only approximate there, so the device runs MINRES for it."""
    import scipy.sparse.linalg as spla

    make, N, strategy, _ = CASES[case]
    m, Ab, lp = _problem(make(), N, strategy)
    src, dst = m.edges
    pc = build_tree_preconditioner(lp, src, dst, m.degrees, target_jobs=16)
    is_tree = m.num_edges == m.num_nodes - 1
    assert pc.tree_exact == is_tree
    dq = lumped_mass(Ab, lp)
    b = np.random.default_rng(7).standard_normal(Ab.shape[0])
    x_ref = spla.spsolve(Ab.tocsc(), b)
    x = direct_model(pc, lp, dq, Ab, b)
    err = np.linalg.norm(x - x_ref) / np.linalg.norm(x_ref)
    if is_tree:
        assert err <= 1e-11, err
    else:
        assert err > 1e-6, err


@pytest.mark.parametrize("case,n_term", [("depth6_N40", 1), ("depth6_N40", 3),
                                         ("arterial5_N40", 2)])
def test_forced_coarse_terminals_one_rank(case, n_term):
    """coarse_structure(terminals=...) on one rank: the coarse set is the Steiner closure of
    the forced junctions (one terminal: itself; several: the paths between them), and the
    decomposition rooted at them keeps P^{-1} exact -- the coarse model (partials, coarse
    forest solve, back-substitution) equals the single-rank application."""
    from networks_fenicsx_amd.precond import coarse_structure

    make, N, strategy, _ = CASES[case]
    m, Ab, lp = _problem(make(), N, strategy)
    src, dst = m.edges
    bif = np.asarray(m.bifurcation_values)
    terms = bif[np.linspace(0, bif.size - 1, n_term).astype(np.int64)]
    cs = coarse_structure(src, dst, m.degrees, np.zeros(src.size, np.int64), 1, terminals=terms)
    assert set(terms.tolist()) <= set(cs.node.tolist())
    if n_term == 1:
        assert cs.n == 1
    # the coarse set is connected through coarse junctions only (Steiner closure): its
    # forest has one root
    assert int((cs.parent < 0).sum()) == 1
    pc = build_tree_preconditioner(lp, src, dst, m.degrees, coarse=cs)
    assert pc.n_coarse == cs.n
    dq = lumped_mass(Ab, lp)
    r = np.random.default_rng(5).standard_normal(Ab.shape[0])
    st = pc_up_model(pc, lp, dq, r)
    z = pc_finish_model(pc, lp, dq, st, st["partial"])
    pc1 = build_tree_preconditioner(lp, src, dst, m.degrees)
    z1 = apply_model(pc1, lp, dq, r)
    assert np.linalg.norm(z - z1) <= 1e-12 * np.linalg.norm(z1)


CYCLIC = {"edge_info_N10": (CASES["edge_info_N10"][0], 10),
          "lattice4x5_N6": (lambda: lattice_graph(4, 5), 6),
          "lattice6x6_N3": (lambda: lattice_graph(6, 6), 3),
          # 342 cycle chains: past round 5's 128-chain cap (the capacitance matrix is inverted
          # on the device since round 6)
          "lattice19x20_N2": (lambda: lattice_graph(19, 20), 2)}


# (the 342-chain lattice is the GPU tests' -- its dense CPU model takes minutes)
@pytest.mark.parametrize("case", sorted(c for c in CYCLIC if c != "lattice19x20_N2"))
def test_cycle_rows_and_woodbury(case):
    """Graphs with cycles (nx_set_cycles): the decomposition lists, per cycle-closing chain,
    the (flux end, multiplier) pair its grounded end drops -- a +-1 coupling of A. Without
    those pairs the system A_g is exactly what the tree solve inverts (the direct model equals
    a sparse solve of A_g), and the rank-2k Woodbury correction the device applies recovers
    A^{-1} b (the reference's MUMPS LU, solver.py:58-65) to 1e-12."""
    import scipy.sparse as sp
    import scipy.sparse.linalg as spla

    make, N = CYCLIC[case]
    m, Ab, lp = _problem(make(), N)
    src, dst = m.edges
    pc = build_tree_preconditioner(lp, src, dst, m.degrees, target_jobs=16)
    k = m.num_edges - m.num_nodes + 1  # independent cycles (one connected component)
    assert not pc.tree_exact and pc.cyc_rows.shape == (k, 2)
    q, lam = pc.cyc_rows[:, 0].astype(np.int64), pc.cyc_rows[:, 1].astype(np.int64)
    Ad = Ab.toarray()
    per = 2 * N + 1
    assert np.all(q < lp.n_edge_dofs) and np.all(q % per % (2 * N) == 0)  # flux end rows
    assert np.all(lam >= lp.n_edge_dofs)  # multiplier rows
    a = Ad[q, lam]
    assert np.all(np.abs(a) == 1.0) and np.array_equal(a, Ad[lam, q])
    Ag = Ad.copy()
    Ag[q, lam] = 0.0
    Ag[lam, q] = 0.0
    Ags = sp.csr_matrix(Ag)
    dq = lumped_mass(Ab, lp)
    b = np.random.default_rng(11).standard_normal(Ab.shape[0])
    xg = direct_model(pc, lp, dq, Ags, b)
    xg_ref = spla.spsolve(Ags.tocsc(), b)
    assert np.linalg.norm(xg - xg_ref) <= 1e-11 * np.linalg.norm(xg_ref)
    # Woodbury, as k_cyc_*: Z = A_g^{-1} U, Cinv = (C^{-1} + U^T Z)^{-1}
    rows = pc.cyc_rows.reshape(-1).astype(np.int64)
    mm = rows.size
    Z = np.stack([direct_model(pc, lp, dq, Ags, np.eye(Ab.shape[0])[r]) for r in rows], axis=1)
    cap = Z[rows]
    for i in range(k):
        cap[2 * i, 2 * i + 1] += 1.0 / a[i]
        cap[2 * i + 1, 2 * i] += 1.0 / a[i]
    w = np.linalg.solve(cap, xg[rows])
    x = xg - Z @ w
    x_ref = spla.spsolve(Ab.tocsc(), b)
    assert np.linalg.norm(x - x_ref) <= 1e-12 * np.linalg.norm(x_ref)
    assert mm == 2 * k


@pytest.mark.parametrize("case,P", [("edge_info_N10", 2), ("edge_info_N10", 3),
                                    ("lattice4x5_N6", 2), ("lattice4x5_N6", 3),
                                    ("lattice6x6_N3", 4)])
def test_multi_rank_cycle_rows_and_woodbury(case, P):
    """Several ranks, graphs with cycles (nx_set_cycles_team): each rank's decomposition lists
    the couplings its grounded chain ends drop -- chains closing a cycle inside the rank and
    coarse chains closing a cycle of the coarse graph (their multiplier can be another rank's
    row, a ghost column here). Without all ranks' pairs the system A_g is exactly what the
    multi-rank direct solve inverts (each rank's sweeps, one sum of the coarse partials, the
    coarse forest), and the rank-2k Woodbury correction recovers A^{-1} b to 1e-12."""
    import scipy.sparse as sp
    import scipy.sparse.linalg as spla

    import distributed_model as DM
    from networks_fenicsx_amd.precond import lumped_mass, pc_finish_model, pc_up_model

    make, N = CYCLIC[case]
    m, Ab, lp1 = _problem(make(), N)
    src, dst = m.edges
    bif = m.bifurcation_index
    dq_global = lumped_mass(Ab, lp1)
    lps = [build_local_problem(m.node_coordinates, src, dst, m.degrees, N, r, P)
           for r in range(P)]
    pcs = [build_tree_preconditioner(lp, src, dst, m.degrees, target_jobs=16) for lp in lps]
    rows = [DM.global_rows(lp, m.num_edges, bif) for lp in lps]
    # every rank's dropped couplings in global numbering
    pairs = []
    for lp, pc, rw in zip(lps, pcs, rows):
        for q, lam in pc.cyc_rows:
            gl = rw[lam] if lam < lp.n_own else lp.ghost_global[lam - lp.n_own]
            pairs.append((int(rw[q]), int(gl)))
    k = m.num_edges - m.num_nodes + 1
    assert len(pairs) == k, (len(pairs), k)
    q = np.array([p[0] for p in pairs])
    lam = np.array([p[1] for p in pairs])
    Ad = Ab.toarray()
    a = Ad[q, lam]
    assert np.all(np.abs(a) == 1.0) and np.array_equal(a, Ad[lam, q])
    Ag = Ad.copy()
    Ag[q, lam] = 0.0
    Ag[lam, q] = 0.0
    Ags = sp.csr_matrix(Ag)

    def apply_all(r):  # P^{-1} over the ranks: sweeps, the partials summed, coarse forest
        sts = [pc_up_model(pc, lp, dq_global[lp.edges], r[rw])
               for lp, pc, rw in zip(lps, pcs, rows)]
        tot = sum(st["partial"] for st in sts)
        z = np.zeros_like(r)
        for lp, pc, rw, st in zip(lps, pcs, rows, sts):
            z[rw] = pc_finish_model(pc, lp, dq_global[lp.edges], st, tot)
        return z

    per = 2 * N + 1
    rid = np.arange(Ab.shape[0])
    flux = (rid < m.num_edges * per) & (rid % per % 2 == 0)

    def direct_multi(b):
        y = apply_all(np.where(flux, b, 0.0))
        w = np.where(flux, 0.0, Ags @ np.where(flux, y, 0.0) - b)
        xs = apply_all(w)
        t = np.where(flux, b - Ags @ np.where(flux, 0.0, xs), 0.0)
        return np.where(flux, apply_all(t), xs)

    b = np.random.default_rng(5).standard_normal(Ab.shape[0])
    xg = direct_multi(b)
    xg_ref = spla.spsolve(Ags.tocsc(), b)
    assert np.linalg.norm(xg - xg_ref) <= 1e-11 * np.linalg.norm(xg_ref)
    U = np.stack([q, lam], axis=1).reshape(-1)
    Z = np.stack([direct_multi(np.eye(Ab.shape[0])[r]) for r in U], axis=1)
    cap = Z[U]
    for i in range(k):
        cap[2 * i, 2 * i + 1] += 1.0 / a[i]
        cap[2 * i + 1, 2 * i] += 1.0 / a[i]
    x = xg - Z @ np.linalg.solve(cap, xg[U])
    x_ref = spla.spsolve(Ab.tocsc(), b)
    assert np.linalg.norm(x - x_ref) <= 1e-12 * np.linalg.norm(x_ref)


@pytest.mark.parametrize("case,P", [("edge_info_N10", 2), ("lattice4x5_N6", 3),
                                    ("lattice6x6_N3", 4)])
def test_team_cycle_tables(case, P):
    """nx_set_cycles_team's per-rank arrays (layout.team_cycle_tables): every column of U has
    exactly one owning rank whose row is that global row; every pair's chain -- its flux end
    row and multiplier column, in that rank's numbering -- is on exactly one rank."""
    from networks_fenicsx_amd.layout import cycle_pairs_global, global_row_ids, team_cycle_tables

    make, N = CYCLIC[case]
    m, Ab, lp1 = _problem(make(), N)
    src, dst = m.edges
    bif = m.bifurcation_index
    lps = [build_local_problem(m.node_coordinates, src, dst, m.degrees, N, r, P)
           for r in range(P)]
    pcs = [build_tree_preconditioner(lp, src, dst, m.degrees, target_jobs=16) for lp in lps]
    pairs = [p for lp, pc in zip(lps, pcs)
             for p in cycle_pairs_global(lp, pc.cyc_rows, m.num_edges, bif)]
    K = len(pairs)
    assert K == m.num_edges - m.num_nodes + 1
    order = sorted(pairs)
    tabs = [team_cycle_tables(lp, pc.cyc_rows, pairs, m.num_edges, bif)
            for lp, pc in zip(lps, pcs)]
    for i in range(2 * K):
        g = order[i // 2][i % 2]
        owners = [r for r, t in enumerate(tabs) if t[0][i] >= 0]
        assert len(owners) == 1, (i, owners)
        r = owners[0]
        assert global_row_ids(lps[r], m.num_edges, bif)[tabs[r][0][i]] == g
    for k in range(K):
        holders = [r for r, t in enumerate(tabs) if t[1][k] >= 0]
        assert len(holders) == 1, (k, holders)
        r = holders[0]
        ids = global_row_ids(lps[r], m.num_edges, bif)
        assert (ids[tabs[r][1][k]], ids[tabs[r][2][k]]) == order[k]
