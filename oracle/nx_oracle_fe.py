"""CPU ORACLE for general element degrees -- test infrastructure only.

Same rules as :mod:`oracle.nx_oracle`: only ``tests/``, ``__graft_entry__.smoke()`` and
``bench.py``'s ``cpu_baseline`` leg may import it, and only as the checker.

What it restates
----------------
``HydraulicNetworkAssembler(mesh, flux_degree=k, pressure_degree=m)``
(reference ``assembly.py:121-146``): per graph edge a Lagrange P_k flux space with the
*equispaced* variant (``assembly.py:126-131``), one pressure space on the whole network
mesh -- ``DG0`` when ``m == 0``, continuous Lagrange P_m otherwise (``assembly.py:135-145``;
continuous means shared at every mesh vertex, graph nodes included) -- and DG0
multipliers at the bifurcations. The forms are the ones of ``compute_forms``
(``assembly.py:253-277``), now with degree-k / degree-m element tensors:

* mass       ``R q v dx``          -> ``R h Mref[i, j]``,  ``Mref = int_0^1 phi_i phi_j``
* divergence ``phi dq/ds dx``      -> ``Dref[a, j] = int_0^1 psi_a phi_j'`` (no h)
* gradient   ``-p dv/ds dx``       -> ``-Dref[a, j]`` at (flux j, pressure a)
* source     ``f phi dx``          -> ``f h wref[a]``, ``wref = int_0^1 psi_a``
* boundary / junction terms act on the edge end values (Lagrange nodes at both ends),
  exactly as for P1 (``assembly.py:258-277``).

The element tensors come from basix's equispaced Lagrange basis on [0, 1] (nodes
``j / k``), a third-party dependency that is absent here; it is restated as the Lagrange
interpolation polynomials through those nodes, integrated with Gauss-Legendre rules exact
for the polynomial degree (FFCx likewise integrates these forms exactly).

Layout (the reference's block order, ``assembly.py:317-321``): flux colour blocks (the
``kN+1`` values of each edge along the edge, source -> target), then pressure, then the
multipliers. Pressure DoF order: ``m == 0`` -- ``N`` cell values per edge, edge-major;
``m >= 1`` -- first one value per graph node that has an edge (ascending node id), then
the ``mN-1`` interior values of every edge along the edge, edge-major. (DOLFINx permutes
its DoFs; the permutation is not observable through the reference's tests.)

Parity pinning
--------------
No reference output exists for degrees other than the default (P1/DG0): the reference's
tests and demos only use ``flux_degree=1, pressure_degree=0`` (``demo_perf.py:107``,
``demo_arterial_tree.py:20``). The restatement is pinned (a) by reducing to
:func:`oracle.nx_oracle.assemble_reference` bit-for-bit structure at ``k=1, m=0`` (test
``tests/test_oracle_fe.py``) and (b) analytically: for ``f = 0`` and edgewise-constant R the
exact solution (q constant, p linear per edge) lies in the discrete spaces whenever
``m >= 1``, so the discrete solution must equal the resistor-network answer
(:func:`resistor_network_solution_fe`). ``k >= 2, m == 0`` has no closed form: parity
for it is "pinned structurally" only (same assembler, analytic cases cover the tensors).
"""

from __future__ import annotations

from dataclasses import dataclass

import numpy as np
import scipy.sparse as sp

from .nx_oracle import _nodal, cell_geometry, resistor_network_solution  # noqa: F401

__all__ = ["reference_tensors", "FeProblem", "build_problem_fe", "assemble_reference_fe",
           "resistor_network_solution_fe", "pressure_positions"]


def _lagrange(nodes: np.ndarray, x: np.ndarray):
    """Values and derivatives of the Lagrange basis through ``nodes`` at ``x``.

    Returns ``(phi, dphi)`` of shape ``(len(nodes), len(x))``.
    """
    n = nodes.size
    phi = np.ones((n, x.size))
    dphi = np.zeros((n, x.size))
    for j in range(n):
        others = [i for i in range(n) if i != j]
        den = np.prod([nodes[j] - nodes[i] for i in others]) if others else 1.0
        num = np.ones_like(x)
        for i in others:
            num = num * (x - nodes[i])
        phi[j] = num / den
        # derivative: sum over the dropped factor
        d = np.zeros_like(x)
        for l in others:
            t = np.ones_like(x)
            for i in others:
                if i != l:
                    t = t * (x - nodes[i])
            d = d + t
        dphi[j] = d / den
    return phi, dphi


def reference_tensors(k: int, m: int):
    """``(Mref, Dref, wref)`` on the unit interval for flux P_k and pressure degree m.

    ``Mref[i, j] = int phi_i phi_j`` ((k+1)^2), ``Dref[a, j] = int psi_a phi_j'``
    ((m+1) x (k+1)), ``wref[a] = int psi_a``. Basis functions are ordered by node position
    ``0, 1/k, ..., 1`` (``psi = 1`` for m = 0).
    """
    if k < 1 or m < 0:
        raise ValueError("flux degree >= 1 and pressure degree >= 0 required")
    nq = max(k, m) + 2
    g, gw = np.polynomial.legendre.leggauss(nq)
    x = 0.5 * (g + 1.0)
    w = 0.5 * gw
    phi, dphi = _lagrange(np.arange(k + 1) / k, x)
    if m == 0:
        psi = np.ones((1, x.size))
    else:
        psi, _ = _lagrange(np.arange(m + 1) / m, x)
    Mref = (phi * w) @ phi.T
    Dref = (psi * w) @ dphi.T
    wref = psi @ w
    return Mref, Dref, wref


@dataclass
class FeProblem:
    base: object  # oracle.nx_oracle.OracleProblem-like topology (pos3, src, dst, N, ...)
    k: int
    m: int
    flux_offset: np.ndarray  # (E,) first flux DoF of each edge (kN+1 along the edge)
    color_offset: np.ndarray
    p_offset: int
    n_p: int
    p_nodes: np.ndarray  # graph nodes carrying a pressure DoF (m >= 1), ascending
    lm_offset: int
    n_dofs: int

    @property
    def N(self) -> int:
        return self.base.N


def build_problem_fe(pos, src, dst, N: int, k: int, m: int, colors=None) -> FeProblem:
    from .nx_oracle import build_problem

    base = build_problem(pos, src, dst, N, colors)
    E = base.src.size
    nf = k * N + 1
    flux_offset = np.zeros(E, dtype=np.int64)
    color_offset = np.zeros(base.n_colors + 1, dtype=np.int64)
    cursor = 0
    for c in range(base.n_colors):
        color_offset[c] = cursor
        members = np.flatnonzero(base.colors == c)
        flux_offset[members] = cursor + np.arange(members.size) * nf
        cursor += members.size * nf
    color_offset[base.n_colors] = cursor
    p_offset = cursor
    if m == 0:
        p_nodes = np.zeros(0, dtype=np.int64)
        n_p = E * N
    else:
        p_nodes = np.flatnonzero(base.degree > 0)
        n_p = p_nodes.size + E * (m * N - 1)
    lm_offset = p_offset + n_p
    n_dofs = lm_offset + base.bifurcations.size
    return FeProblem(base, k, m, flux_offset, color_offset, p_offset, n_p, p_nodes,
                     lm_offset, n_dofs)


def _pressure_dof(prob: FeProblem, e: np.ndarray, pos: np.ndarray) -> np.ndarray:
    """Global pressure DoF of position ``pos`` (0..mN) along edge ``e`` (m >= 1)."""
    b = prob.base
    N, m = b.N, prob.m
    node_slot = np.full(b.pos3.shape[0], -1, dtype=np.int64)
    node_slot[prob.p_nodes] = np.arange(prob.p_nodes.size)
    out = prob.p_offset + prob.p_nodes.size + e * (m * N - 1) + pos - 1
    out = np.where(pos == 0, prob.p_offset + node_slot[b.src[e]], out)
    out = np.where(pos == m * N, prob.p_offset + node_slot[b.dst[e]], out)
    return out


def assemble_reference_fe(prob: FeProblem, p_bc, f: float = 0.0, R=1.0):
    """Assemble ``(A, b)`` of the reference forms at degrees (k, m), non-symmetric as
    the reference assembles it. Sorted CSR with duplicates summed, and the rhs."""
    b_ = prob.base
    E, N, k, m = b_.src.size, b_.N, prob.k, prob.m
    _, h = cell_geometry(b_)  # (E, N)
    Mref, Dref, wref = reference_tensors(k, m)
    Re = np.broadcast_to(np.asarray(R, dtype=np.float64), (E,))[:, None]
    e_idx = np.broadcast_to(np.arange(E)[:, None], (E, N))
    c_idx = np.broadcast_to(np.arange(N)[None, :], (E, N))
    q = [prob.flux_offset[:, None] + c_idx * k + i for i in range(k + 1)]  # (E, N) each
    if m == 0:
        p = [prob.p_offset + e_idx * N + c_idx]
    else:
        p = [_pressure_dof(prob, e_idx, c_idx * m + a) for a in range(m + 1)]
    rows, cols, vals = [], [], []
    for i in range(k + 1):
        for j in range(k + 1):
            rows.append(q[i]); cols.append(q[j]); vals.append(Re * h * Mref[i, j])
    one = np.ones((E, N))
    for a in range(len(p)):
        for j in range(k + 1):
            rows.append(p[a]); cols.append(q[j]); vals.append(Dref[a, j] * one)
            rows.append(q[j]); cols.append(p[a]); vals.append(-Dref[a, j] * one)
    lm_of = np.full(b_.pos3.shape[0], -1, dtype=np.int64)
    lm_of[b_.bifurcations] = prob.lm_offset + np.arange(b_.bifurcations.size)
    e_in = np.flatnonzero(lm_of[b_.dst] >= 0)
    e_out = np.flatnonzero(lm_of[b_.src] >= 0)
    q_end = prob.flux_offset[e_in] + k * N
    q_start = prob.flux_offset[e_out]
    lam_in = lm_of[b_.dst[e_in]]
    lam_out = lm_of[b_.src[e_out]]
    rows += [lam_in, q_end, lam_out, q_start]
    cols += [q_end, lam_in, q_start, lam_out]
    vals += [np.ones(e_in.size), np.ones(e_in.size), -np.ones(e_out.size), -np.ones(e_out.size)]
    r = np.concatenate([np.asarray(a).ravel() for a in rows])
    c = np.concatenate([np.asarray(a).ravel() for a in cols])
    v = np.concatenate([np.asarray(a, dtype=np.float64).ravel() for a in vals])
    A = sp.coo_matrix((v, (r, c)), shape=(prob.n_dofs, prob.n_dofs)).tocsr()
    A.sum_duplicates()
    A.sort_indices()

    rhs = np.zeros(prob.n_dofs)
    pb = _nodal(p_bc, b_.pos3)
    is_leaf = np.zeros(b_.pos3.shape[0], dtype=bool)
    is_leaf[b_.leaf_in] = True
    is_root = np.zeros(b_.pos3.shape[0], dtype=bool)
    is_root[b_.root_out] = True
    e_leaf = np.flatnonzero(is_leaf[b_.dst])
    e_root = np.flatnonzero(is_root[b_.src])
    rhs[prob.flux_offset[e_leaf] + k * N] += pb[b_.dst[e_leaf]]
    rhs[prob.flux_offset[e_root]] -= pb[b_.src[e_root]]
    fe = np.broadcast_to(np.asarray(f, dtype=np.float64), (E,))[:, None]  # constant or per edge
    for a in range(len(p)):
        np.add.at(rhs, p[a].ravel(), (fe * h * wref[a]).ravel())
    return A, rhs


def pressure_positions(prob: FeProblem) -> np.ndarray:
    """Arc-length position ``s`` (from the edge's source) and edge of every pressure DoF:
    returns ``(edge, s)`` arrays over the pressure block (node DoFs: an incident edge)."""
    b_ = prob.base
    E, N, m = b_.src.size, b_.N, prob.m
    _, h = cell_geometry(b_)
    L = h.sum(axis=1)
    if m == 0:
        s = (np.cumsum(h, axis=1) - 0.5 * h).ravel()
        return np.repeat(np.arange(E), N), s
    pos = np.arange(1, m * N)
    e_in = np.repeat(np.arange(E), m * N - 1)
    s_in = (L[:, None] * pos[None, :] / (m * N)).ravel()
    return e_in, s_in


def resistor_network_solution_fe(prob: FeProblem, p_bc, R=1.0) -> np.ndarray:
    """Analytic answer for ``f = 0``, edgewise-constant R and ``m >= 1`` (the exact solution
    is in the discrete spaces): q constant per edge, p = P_u - R q s at every node."""
    if prob.m < 1:
        raise ValueError("closed form only for continuous pressure (m >= 1); "
                         "for m = 0 use oracle.nx_oracle.resistor_network_solution at k = 1")
    b_ = prob.base
    E, N, k, m = b_.src.size, b_.N, prob.k, prob.m
    x1 = resistor_network_solution(b_, p_bc, R)  # P1/DG0 answer in the P1 block layout
    Re = np.broadcast_to(np.asarray(R, dtype=np.float64), (E,))
    qe = x1[b_.flux_offset]  # constant flux per edge
    # nodal pressures: multipliers at bifurcations, -p_bc at boundary nodes
    n = b_.pos3.shape[0]
    P = np.zeros(n)
    pb = _nodal(p_bc, b_.pos3)
    P[b_.leaf_in] = -pb[b_.leaf_in]
    P[b_.root_out] = -pb[b_.root_out]
    P[b_.bifurcations] = x1[b_.lm_offset:]
    x = np.zeros(prob.n_dofs)
    for e in range(E):
        x[prob.flux_offset[e]: prob.flux_offset[e] + k * N + 1] = qe[e]
    x[prob.p_offset: prob.p_offset + prob.p_nodes.size] = P[prob.p_nodes]
    e_in, s_in = pressure_positions(prob)
    x[prob.p_offset + prob.p_nodes.size: prob.lm_offset] = P[b_.src[e_in]] - Re[e_in] * qe[e_in] * s_in
    x[prob.lm_offset:] = P[b_.bifurcations]
    return x
