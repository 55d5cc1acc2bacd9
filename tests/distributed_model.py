"""CPU model of the device's multi-rank path (test infrastructure).

It runs the same MINRES kernel schedule as ``nx_solve`` (``csrc/nxhip.hip``:
k_mr_spmv -> alpha all-reduce -> k_mr_lanczos -> beta all-reduce + rotation), on each
rank's local CSR rows with ghost columns, and with the halo exchange driven by the
``LocalProblem`` plan. The local matrices are cut out of the oracle's global
build-layout matrix, so a wrong column map or halo plan shows up as a wrong answer.
"""

from __future__ import annotations

import numpy as np

from networks_fenicsx_amd.layout import LocalProblem


def global_rows(lp: LocalProblem, n_edges_global: int, bif_index: np.ndarray) -> np.ndarray:
    """Global (single-rank layout) index of every owned row, in local order."""
    per = 2 * lp.N + 1
    rows = (lp.edges[:, None] * per + np.arange(per)[None, :]).ravel()
    lam = n_edges_global * per + bif_index[lp.lm_nodes]
    return np.concatenate([rows, lam]).astype(np.int64)


def local_matrix(Ab, lp: LocalProblem, n_edges_global: int, bif_index: np.ndarray):
    rows = global_rows(lp, n_edges_global, bif_index)
    cols = np.concatenate([rows, lp.ghost_global])
    return Ab[rows][:, cols].tocsr(), rows


def halo_exchange_local(lps, xs):
    """Fill the ghost slots of every rank's vector from the owners (one process)."""
    out = []
    for r, lp in enumerate(lps):
        v = xs[r].copy()
        for j, p in enumerate(lp.peers):
            peer = lps[p]
            k = list(peer.peers).index(r)
            idx = peer.send_idx[peer.send_off[k]:peer.send_off[k + 1]]
            v[lp.n_own + lp.recv_off[j]: lp.n_own + lp.recv_off[j + 1]] = xs[p][idx]
        out.append(v)
    return out


def minres(A_local, b_local, n_own: int, halo, allreduce, rtol=1e-12, maxit=5000):
    """Unpreconditioned MINRES in the device's kernel order.

    ``halo(v)`` fills ``v[n_own:]`` in place; ``allreduce(x) -> float`` sums over ranks.
    Returns ``(x_owned, iterations, relres)``.
    """
    n_col = A_local.shape[1]
    vb = [np.zeros(n_col), np.zeros(n_col)]
    vb[0][:n_own] = b_local
    vb[1][:n_own] = b_local
    wb = [np.zeros(n_own), np.zeros(n_own)]
    x = np.zeros(n_own)
    beta1 = np.sqrt(allreduce(float(b_local @ b_local)))
    st = dict(beta=beta1, oldb=0.0, dbar=0.0, epsln=0.0, phibar=beta1, cs=-1.0, sn=0.0)
    if beta1 == 0:
        return x, 0, 0.0
    pend = None
    it = 0
    relres = 1.0
    while True:
        k = it + 1
        r1, r2 = vb[(k - 1) & 1], vb[k & 1]
        w1, w2 = wb[k & 1], wb[(k - 1) & 1]
        halo(r2)
        s = 1.0 / st["beta"]
        c1 = st["beta"] / st["oldb"] if it > 0 else 0.0
        Ay = A_local @ r2
        r1v = r1[:n_own].copy()
        y = s * Ay - c1 * r1v
        alfa_loc = float((s * r2[:n_own]) @ y)
        r1[:n_own] = y
        if pend is not None:
            vk = r1v / st["oldb"]
            wn = (vk - pend[0] * w1 - pend[1] * w2) * pend[2]
            w1[:] = wn
            x += pend[3] * wn
        alfa = allreduce(alfa_loc)
        y = r1[:n_own] - (alfa / st["beta"]) * r2[:n_own]
        r1[:n_own] = y
        b2 = allreduce(float(y @ y))
        oldb = st["beta"]
        beta = np.sqrt(b2)
        st["oldb"], st["beta"] = oldb, beta
        oldeps = st["epsln"]
        delta = st["cs"] * st["dbar"] + st["sn"] * alfa
        gbar = st["sn"] * st["dbar"] - st["cs"] * alfa
        st["epsln"] = st["sn"] * beta
        st["dbar"] = -st["cs"] * beta
        gamma = max(np.hypot(gbar, beta), 2.220446049250313e-16)
        st["cs"], st["sn"] = gbar / gamma, beta / gamma
        phi = st["cs"] * st["phibar"]
        st["phibar"] = st["sn"] * st["phibar"]
        pend = (oldeps, delta, 1.0 / gamma, phi)
        it += 1
        relres = st["phibar"] / beta1
        if relres <= rtol or beta == 0.0 or it >= maxit:
            break
    # finalize: pending update of the last iteration
    k = it + 1
    r1 = vb[(k - 1) & 1]
    w1, w2 = wb[k & 1], wb[(k - 1) & 1]
    vk = r1[:n_own] / st["oldb"]
    wn = (vk - pend[0] * w1 - pend[1] * w2) * pend[2]
    x += pend[3] * wn
    return x, it, relres


def minres_pc(A_local, b_local, n_own: int, halo, allreduce, apply_pc, rtol=1e-12, maxit=5000,
              linear: bool = False):
    """Preconditioned MINRES (scipy's statement order) with a rank-local SPD
    preconditioner ``apply_pc(r_owned) -> z_owned``; ``halo`` fills ghost slots of the
    gathered vector (z), as the device does before each SpMV. ``linear`` models the
    device's multi-rank form: the preconditioner is applied to y before alpha is known
    and z' = P^{-1}y - (alpha/beta) z (csrc/nxhip.hip, PcArgs::lin)."""
    n_col = A_local.shape[1]
    r1 = b_local.copy()
    r2 = b_local.copy()
    z = np.zeros(n_col)
    z[:n_own] = apply_pc(r1)
    beta1 = np.sqrt(allreduce(float(r1 @ z[:n_own])))
    x = np.zeros(n_own)
    w = np.zeros(n_own)
    w2 = np.zeros(n_own)
    oldb, beta, dbar, epsln, phibar, cs, sn = 0.0, beta1, 0.0, 0.0, beta1, -1.0, 0.0
    it = 0
    while it < maxit:
        it += 1
        s = 1.0 / beta
        halo(z)
        v = s * z[:n_own]
        y = s * (A_local @ z)
        if it >= 2:
            y = y - (beta / oldb) * r1
        if linear:
            py = apply_pc(y)  # before alpha (its partial travels with the coarse exchange)
        alfa = allreduce(float(v @ y))
        y = y - (alfa / beta) * r2
        r1, r2 = r2, y
        z_old = z[:n_own].copy()
        z = np.zeros(n_col)
        z[:n_own] = py - (alfa / beta) * z_old if linear else apply_pc(r2)
        oldb, beta = beta, np.sqrt(allreduce(float(r2 @ z[:n_own])))
        oldeps = epsln
        delta = cs * dbar + sn * alfa
        gbar = sn * dbar - cs * alfa
        epsln = sn * beta
        dbar = -cs * beta
        gamma = max(np.hypot(gbar, beta), 2.220446049250313e-16)
        cs, sn = gbar / gamma, beta / gamma
        phi = cs * phibar
        phibar = sn * phibar
        w1, w2 = w2, w
        w = (v - oldeps * w1 - delta * w2) / gamma
        x = x + phi * w
        if phibar / beta1 <= rtol:
            break
    return x, it, phibar / beta1
