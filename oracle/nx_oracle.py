"""CPU ORACLE -- test infrastructure only.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may
import this module, and only as the checker / CPU baseline. The product path
(``networks_fenicsx_amd``) never imports it and fails loudly without its HIP library.

What it restates
----------------
The reference assembles a mixed (M+2)x(M+2) block system with DOLFINx/FFCx and
solves it with PETSc/MUMPS. Neither is in this image, so this is a line-by-line
restatement of the *forms* in numpy, assembled cell by cell in the reference's
block layout and solved with SuperLU (``scipy.sparse.linalg.spsolve``, the
direct-solver stand-in for MUMPS, reference ``solver.py:58-65``):

* mass       ``R q v dx``                     -> ``R h/3, R h/6``   (``assembly.py:253``)
* divergence ``phi (grad q . t) dx``          -> ``[-1, +1]`` on (p_cell, q_up/q_down)
                                                                   (``assembly.py:254``)
* gradient   ``-p (grad v . t) dx``           -> ``[+1, -1]^T``     (``assembly.py:255``)
* boundary   ``p_bc v ds(in) - p_bc v ds(out)`` -> ``+p_bc`` at leaf end DoFs,
                                               ``-p_bc`` at root start DoFs (``:258-260``)
* source     ``f phi dx``                     -> ``f h``            (``assembly.py:262``)
* junctions  ``+-mu q ds``, ``+-lmbda v ds``  -> ``+1`` at in-edge ends, ``-1`` at out-edge
                                               starts, both blocks (``assembly.py:271-277``)

Geometry follows the reference mesh generator (``mesh.py:275-291``): interior points
``start * (1 - w) + end * w`` with ``w = linspace(0, 1, N, endpoint=False)[1:]``,
cell length = Euclidean norm of the cell's vertex difference, tangent source->target
(orientation semantics ``mesh.py:365-400``, pinned by ``tests/test_orientation.py`` of
the reference).

Block layout (the reference's function-space order, ``assembly.py:317-321``):
``[flux colour 0 | ... | flux colour M-1 | pressure (DG0, edge-major cells) |
multipliers (bifurcations ascending)]``; inside a colour block the edges of that colour
appear in ``graph.edges()`` order with ``N+1`` DoFs each, source -> target.
(DOLFINx permutes DoFs internally; that permutation is not observable through
the reference's tests and is not reproduced.)

Parity pinning
--------------
* Graph generation and topology: pinned by the reference's own generator outputs
  (``tests/golden/graphs.npz``) and its tests ``test_make_tree.py:21-24``,
  ``test_edge_info.py:36-55``, ``test_orientation.py:52-58``.
* Matrix / solution VALUES: no reference output exists (DOLFINx/PETSc/MUMPS are not
  installed and the reference tests check no values), so they are pinned by an
  analytic known answer instead: for ``f = 0`` and edgewise-constant ``R`` the discrete
  P1/DG0 solution equals the resistor-network solution (:func:`resistor_network_solution`),
  plus the closed-form ``demo_tree`` values. Solution parity against PETSc itself is
  therefore "pinned analytically", not by a reference run.
"""

from __future__ import annotations

from dataclasses import dataclass

import numpy as np
import scipy.sparse as sp
import scipy.sparse.linalg as spla

__all__ = [
    "OracleProblem",
    "build_problem",
    "assemble_reference",
    "solve_reference",
    "to_build_layout",
    "resistor_network_solution",
    "cell_geometry",
]


@dataclass
class OracleProblem:
    pos3: np.ndarray  # (n_nodes, 3)
    src: np.ndarray  # (E,)
    dst: np.ndarray  # (E,)
    N: int
    colors: np.ndarray  # (E,)
    n_colors: int
    degree: np.ndarray  # (n_nodes,)
    bifurcations: np.ndarray  # (B,) ascending node ids
    leaf_in: np.ndarray  # boundary nodes with an in-edge (in_marker)
    root_out: np.ndarray  # boundary nodes with an out-edge (out_marker)
    # reference block layout
    flux_offset: np.ndarray  # (E,) first DoF of edge e's flux in the global vector
    color_offset: np.ndarray  # (M+1,) start of each colour block
    p_offset: int
    lm_offset: int
    n_dofs: int


def build_problem(pos, src, dst, N: int, colors=None) -> OracleProblem:
    """Topology + reference block layout (reference ``mesh.py:175-225``, ``assembly.py:120-162``)."""
    pos = np.asarray(pos, dtype=np.float64)
    n_nodes = pos.shape[0]
    pos3 = np.zeros((n_nodes, 3))
    pos3[:, : pos.shape[1]] = pos
    src = np.asarray(src, dtype=np.int64)
    dst = np.asarray(dst, dtype=np.int64)
    E = src.size
    if colors is None:
        colors = np.arange(E)
    colors = np.asarray(colors, dtype=np.int64)
    n_colors = int(colors.max()) + 1 if E else 0
    degree = np.bincount(src, minlength=n_nodes) + np.bincount(dst, minlength=n_nodes)
    indeg = np.bincount(dst, minlength=n_nodes)
    bif = np.flatnonzero(degree > 1)
    bnd = np.flatnonzero(degree == 1)
    leaf_in = bnd[indeg[bnd] == 1]
    root_out = bnd[indeg[bnd] == 0]

    flux_offset = np.zeros(E, dtype=np.int64)
    color_offset = np.zeros(n_colors + 1, dtype=np.int64)
    cursor = 0
    for c in range(n_colors):
        color_offset[c] = cursor
        members = np.flatnonzero(colors == c)
        flux_offset[members] = cursor + np.arange(members.size) * (N + 1)
        cursor += members.size * (N + 1)
    color_offset[n_colors] = cursor
    p_offset = cursor
    lm_offset = p_offset + E * N
    n_dofs = lm_offset + bif.size
    return OracleProblem(pos3, src, dst, N, colors, n_colors, degree, bif, leaf_in, root_out,
                         flux_offset, color_offset, p_offset, lm_offset, n_dofs)


def cell_geometry(prob: OracleProblem):
    """Per-cell vertex coordinates and lengths, edge-major ``(E, N)``.

    Vertex k of edge e: ``x_u`` (k=0), ``x_v`` (k=N), else ``x_u (1-w_k) + x_v w_k``
    with the reference's ``np.linspace`` weights (``mesh.py:275, 290``).
    """
    N = prob.N
    start = prob.pos3[prob.src][:, None, :]
    end = prob.pos3[prob.dst][:, None, :]
    w = np.linspace(0, 1, N, endpoint=False)[1:][None, :, None]
    inner = start * (1 - w) + end * w  # (E, N-1, 3)
    verts = np.concatenate([start, inner, end], axis=1)  # (E, N+1, 3)
    d = verts[:, 1:, :] - verts[:, :-1, :]
    h = np.sqrt(d[..., 0] * d[..., 0] + d[..., 1] * d[..., 1] + d[..., 2] * d[..., 2])
    return verts, h


def _nodal(values_or_fn, pos3: np.ndarray) -> np.ndarray:
    """p_bc at the graph nodes. Callables get DOLFINx-style ``x`` of shape (3, n)."""
    if callable(values_or_fn):
        return np.asarray(values_or_fn(pos3.T.copy()), dtype=np.float64).reshape(-1)
    return np.asarray(values_or_fn, dtype=np.float64).reshape(-1)


def assemble_reference(prob: OracleProblem, p_bc, f: float = 0.0, R=1.0):
    """Assemble ``(A, b)`` exactly as the reference forms define them (non-symmetric).

    ``R`` and ``f`` are constants or one value per edge. Returns a CSR matrix with sorted
    column indices and duplicate contributions summed, and the rhs vector.
    """
    E, N = prob.src.size, prob.N
    _, h = cell_geometry(prob)
    Re = np.broadcast_to(np.asarray(R, dtype=np.float64), (E,))[:, None]
    k = np.arange(N)[None, :]
    q_up = prob.flux_offset[:, None] + k  # (E, N) upstream vertex DoF of each cell
    q_dn = q_up + 1
    pc = prob.p_offset + np.arange(E)[:, None] * N + k  # pressure DoF of each cell

    m_d = Re * h / 3.0
    m_o = Re * h / 6.0
    one = np.ones_like(h)
    rows = [q_up, q_up, q_dn, q_dn, pc, pc, q_up, q_dn]
    cols = [q_up, q_dn, q_up, q_dn, q_up, q_dn, pc, pc]
    vals = [m_d, m_o, m_o, m_d, -one, one, one, -one]

    # junction blocks (assembly.py:271-277)
    lm_of = np.full(prob.pos3.shape[0], -1, dtype=np.int64)
    lm_of[prob.bifurcations] = prob.lm_offset + np.arange(prob.bifurcations.size)
    e_in = np.flatnonzero(lm_of[prob.dst] >= 0)  # edges ending at a bifurcation
    e_out = np.flatnonzero(lm_of[prob.src] >= 0)  # edges starting at a bifurcation
    q_end = prob.flux_offset[e_in] + N
    q_start = prob.flux_offset[e_out]
    lam_in = lm_of[prob.dst[e_in]]
    lam_out = lm_of[prob.src[e_out]]
    rows += [lam_in, q_end, lam_out, q_start]
    cols += [q_end, lam_in, q_start, lam_out]
    vals += [np.ones(e_in.size), np.ones(e_in.size), -np.ones(e_out.size), -np.ones(e_out.size)]

    r = np.concatenate([np.asarray(a).ravel() for a in rows])
    c = np.concatenate([np.asarray(a).ravel() for a in cols])
    v = np.concatenate([np.asarray(a, dtype=np.float64).ravel() for a in vals])
    A = sp.coo_matrix((v, (r, c)), shape=(prob.n_dofs, prob.n_dofs)).tocsr()
    A.sum_duplicates()
    A.sort_indices()

    b = np.zeros(prob.n_dofs)
    pb = _nodal(p_bc, prob.pos3)
    is_leaf = np.zeros(prob.pos3.shape[0], dtype=bool)
    is_leaf[prob.leaf_in] = True
    is_root = np.zeros(prob.pos3.shape[0], dtype=bool)
    is_root[prob.root_out] = True
    e_leaf = np.flatnonzero(is_leaf[prob.dst])
    e_root = np.flatnonzero(is_root[prob.src])
    b[prob.flux_offset[e_leaf] + N] += pb[prob.dst[e_leaf]]
    b[prob.flux_offset[e_root]] -= pb[prob.src[e_root]]
    fe = np.broadcast_to(np.asarray(f, dtype=np.float64), (E,))[:, None]  # constant or per edge
    b[pc.ravel()] += (fe * h).ravel()
    return A, b


def solve_reference(A, b) -> np.ndarray:
    """Direct sparse solve (SuperLU standing in for MUMPS LU, ``solver.py:58-65``)."""
    return spla.spsolve(A.tocsc(), b)


def build_permutation(prob: OracleProblem, edge_order=None):
    """Map the device ("build") layout to the reference block layout.

    Build layout: edge-interleaved ``[q_0, p_0, q_1, p_1, ..., p_{N-1}, q_N]`` per edge
    (``2N+1`` DoFs) in ``edge_order``, then one multiplier per bifurcation ascending.
    Returns ``(perm, sign)`` with ``x_build = x_ref[perm]`` and ``sign = -1`` on the
    pressure rows (the build negates them to make the system symmetric).
    """
    E, N = prob.src.size, prob.N
    if edge_order is None:
        edge_order = np.arange(E)
    per = 2 * N + 1
    perm = np.empty(E * per + prob.bifurcations.size, dtype=np.int64)
    sign = np.ones(perm.size)
    loc = np.arange(per)
    for slot, e in enumerate(np.asarray(edge_order)):
        base = slot * per
        perm[base + loc[0::2]] = prob.flux_offset[e] + np.arange(N + 1)
        perm[base + loc[1::2]] = prob.p_offset + e * N + np.arange(N)
        sign[base + loc[1::2]] = -1.0
    perm[E * per :] = prob.lm_offset + np.arange(prob.bifurcations.size)
    return perm, sign


def to_build_layout(prob: OracleProblem, A, b, edge_order=None):
    """``(S P A P^T, S P b)``: the symmetric system the device assembles, as sorted CSR."""
    perm, sign = build_permutation(prob, edge_order)
    Ab = sp.diags(sign) @ A[perm][:, perm]
    Ab = Ab.tocsr()
    Ab.sum_duplicates()
    Ab.sort_indices()
    return Ab, sign * b[perm], perm, sign


def resistor_network_solution(prob: OracleProblem, p_bc, R=1.0):
    """Analytic known answer for ``f = 0`` and edgewise-constant ``R``.

    With ``f = 0`` the divergence rows force ``q`` constant per edge and the gradient
    rows force ``p`` linear, so the discrete solution is the resistor network with
    conductance ``g_e = 1 / (R_e L_e)`` and nodal pressure ``P`` where ``P = -p_bc`` on
    boundary nodes (sign from ``assembly.py:258-260``) and Kirchhoff's current law
    holds at every other node. Returns the solution in the reference block layout.
    """
    E, N = prob.src.size, prob.N
    verts, h = cell_geometry(prob)
    L = h.sum(axis=1)
    Re = np.broadcast_to(np.asarray(R, dtype=np.float64), (E,))
    g = 1.0 / (Re * L)
    n = prob.pos3.shape[0]
    Lap = sp.coo_matrix(
        (np.concatenate([g, g, -g, -g]),
         (np.concatenate([prob.src, prob.dst, prob.src, prob.dst]),
          np.concatenate([prob.src, prob.dst, prob.dst, prob.src]))),
        shape=(n, n)).tocsr()
    pb = _nodal(p_bc, prob.pos3)
    fixed = np.concatenate([prob.leaf_in, prob.root_out])
    free = np.setdiff1d(np.flatnonzero(prob.degree > 0), fixed)
    P = np.zeros(n)
    P[fixed] = -pb[fixed]
    if free.size:
        rhs = -Lap[free][:, fixed] @ P[fixed]
        P[free] = spla.spsolve(Lap[free][:, free].tocsc(), rhs)
    q = g * (P[prob.src] - P[prob.dst])
    x = np.zeros(prob.n_dofs)
    for e in range(E):
        x[prob.flux_offset[e] : prob.flux_offset[e] + N + 1] = q[e]
    # cell midpoints along the edge: P_u - R q s
    s_mid = np.cumsum(h, axis=1) - 0.5 * h
    x[prob.p_offset : prob.p_offset + E * N] = (P[prob.src][:, None]
                                                - Re[:, None] * q[:, None] * s_mid).ravel()
    x[prob.lm_offset :] = P[prob.bifurcations]
    return x
