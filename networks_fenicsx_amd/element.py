"""Reference element tensors for general flux / pressure degrees.

The reference builds its spaces with basix (``assembly.py:126-145``): equispaced Lagrange
P_k for the flux on every edge, DG0 (``pressure_degree == 0``) or continuous Lagrange P_m
for the pressure. FFCx then generates the element kernels for the forms of
``compute_forms`` (``assembly.py:253-262``). Every kernel is a constant reference tensor
times a per-cell factor, so they are tabulated once here, on the host, in closed form:
each basis function is expanded in monomials with rational coefficients and the
products are integrated exactly, then rounded once to double. The device gather
assembly (``k_assemble_fe``) multiplies them by ``R h`` / ``f h`` per cell.
"""

from __future__ import annotations

from fractions import Fraction

import numpy as np

__all__ = ["lagrange_monomials", "element_tensors", "stable_pair"]


def lagrange_monomials(degree: int) -> list[list[Fraction]]:
    """Exact monomial coefficients ``C[j][n]`` of the equispaced Lagrange basis on [0, 1]:
    ``phi_j(x) = sum_n C[j][n] x^n`` with ``phi_j(i / degree) = delta_ij`` (rational
    arithmetic: the tensors below are the correctly rounded exact integrals)."""
    if degree == 0:
        return [[Fraction(1)]]
    nodes = [Fraction(i, degree) for i in range(degree + 1)]
    out = []
    for j, xj in enumerate(nodes):
        coef = [Fraction(1)]  # running product, ascending powers
        for i, xi in enumerate(nodes):
            if i == j:
                continue
            # multiply by (x - xi) / (xj - xi)
            d = xj - xi
            nxt = [Fraction(0)] * (len(coef) + 1)
            for n, c in enumerate(coef):
                nxt[n + 1] += c / d
                nxt[n] -= c * xi / d
            coef = nxt
        out.append(coef)
    return out


def _integral_of_products(A, B) -> np.ndarray:
    """``int_0^1 a_i(x) b_j(x) dx`` for polynomials given by exact monomial coefficients."""
    out = np.empty((len(A), len(B)))
    for i, a in enumerate(A):
        for j, b in enumerate(B):
            s = Fraction(0)
            for p, ap in enumerate(a):
                for q, bq in enumerate(b):
                    s += ap * bq / (p + q + 1)
            out[i, j] = float(s)
    return out


def element_tensors(flux_degree: int, pressure_degree: int):
    """``(Mref, Dref, wref)`` for the unit cell.

    ``Mref[i, j] = int phi_i phi_j`` (flux mass), ``Dref[a, j] = int psi_a phi_j'`` (the
    divergence form ``phi dq/ds``; ``h`` cancels), ``wref[a] = int psi_a`` (source).
    Basis functions are ordered by node position along the cell (source side first).
    """
    k, m = int(flux_degree), int(pressure_degree)
    if k < 1 or m < 0:
        raise ValueError("flux_degree >= 1 and pressure_degree >= 0 required")
    Cq = lagrange_monomials(k)
    Cp = lagrange_monomials(m)
    dCq = [[c * n for n, c in enumerate(row)][1:] for row in Cq]  # derivatives
    Mref = _integral_of_products(Cq, Cq)
    Dref = _integral_of_products(Cp, dCq)
    wref = _integral_of_products(Cp, [[Fraction(1)]])[:, 0]
    return Mref, Dref, wref


def stable_pair(flux_degree: int, pressure_degree: int) -> bool:
    """Whether the discrete saddle-point system is nonsingular on every graph.

    DG0 pressure is stable with any flux degree. Continuous pressure of degree m needs
    flux degree k > m: for k <= m the pressure space holds a function orthogonal to every
    flux derivative (checked numerically on the reference's demo graphs: condition
    numbers ~1e16-1e18), and the reference's direct solve would fail on it.
    """
    return pressure_degree == 0 or flux_degree > pressure_degree


def condensed_flux_mass(flux_degree: int):
    """The P_k flux mass of one cell with its interior nodes condensed out, for DG0 pressure
    (whose divergence touches only the cell's two vertex values, so the interior fluxes
    appear in the flux rows alone): ``(alpha, beta, C, K, Mii_inv)`` with, for the cell mass
    ``R h Mref`` and the node order (left vertex, interior 1..k-1, right vertex),

    * ``R h [[alpha, beta], [beta, alpha]] = R h (M_vv - M_vi M_ii^{-1} M_iv)`` -- the
      vertex-only (Schur) mass, symmetric under the cell's reflection;
    * ``C = M_vi M_ii^{-1}`` (2 x (k-1)): the interior right-hand side's share moved onto
      the vertices, ``b_v -= C b_i`` (h and R cancel);
    * ``K = M_ii^{-1} M_iv`` ((k-1) x 2) and ``Mii_inv = M_ii^{-1}``: the interior values
      back from the vertex ones, ``x_i = Mii_inv b_i / (R h) - K x_v``.

    Exact rational arithmetic, rounded once (k = 1: alpha = 1/3, beta = 1/6, no interior)."""
    from fractions import Fraction as F

    k = int(flux_degree)
    Cq = lagrange_monomials(k)
    n = k + 1
    M = [[F(0)] * n for _ in range(n)]
    for i in range(n):
        for j in range(n):
            s = F(0)
            for p, ap in enumerate(Cq[i]):
                for q, bq in enumerate(Cq[j]):
                    s += ap * bq / (p + q + 1)
            M[i][j] = s
    vi = [0, k]
    ii = list(range(1, k))
    ni = len(ii)
    # exact inverse of M_ii (Gauss-Jordan over the rationals)
    A = [[M[r][c] for c in ii] + [F(int(r2 == r)) for r2 in ii] for r in ii]
    for col in range(ni):
        piv = next(r for r in range(col, ni) if A[r][col] != 0)
        A[col], A[piv] = A[piv], A[col]
        d = A[col][col]
        A[col] = [v / d for v in A[col]]
        for r in range(ni):
            if r != col and A[r][col] != 0:
                f = A[r][col]
                A[r] = [a - f * b for a, b in zip(A[r], A[col])]
    Minv = [row[ni:] for row in A]
    Mvi = [[M[v][c] for c in ii] for v in vi]
    C = [[sum(Mvi[a][t] * Minv[t][j] for t in range(ni)) for j in range(ni)] for a in range(2)]
    Kq = [[sum(Minv[i][t] * M[ii[t]][vi[b]] for t in range(ni)) for b in range(2)]
          for i in range(ni)]
    S = [[M[vi[a]][vi[b]] - sum(C[a][t] * M[ii[t]][vi[b]] for t in range(ni))
          for b in range(2)] for a in range(2)]
    assert S[0][0] == S[1][1] and S[0][1] == S[1][0]
    f64 = lambda X: np.array([[float(v) for v in row] for row in X], dtype=np.float64)  # noqa: E731
    return (float(S[0][0]), float(S[0][1]), f64(C).reshape(2, ni), f64(Kq).reshape(ni, 2),
            f64(Minv).reshape(ni, ni))


def _frac_inverse(A):
    """Exact inverse of a square matrix of Fractions (Gauss-Jordan, first nonzero pivot)."""
    from fractions import Fraction as F

    n = len(A)
    W = [list(row) + [F(int(i == j)) for j in range(n)] for i, row in enumerate(A)]
    for col in range(n):
        piv = next(r for r in range(col, n) if W[r][col] != 0)
        W[col], W[piv] = W[piv], W[col]
        d = W[col][col]
        W[col] = [v / d for v in W[col]]
        for r in range(n):
            if r != col and W[r][col] != 0:
                f = W[r][col]
                W[r] = [a - f * b for a, b in zip(W[r], W[col])]
    return [row[n:] for row in W]


def condensed_cell_blocks(flux_degree: int, pressure_degree: int):
    """One cell of continuous P_m pressure (m >= 1) and P_k flux with its interior nodes
    condensed out onto the vertex unknowns ``V = (q_L, p_L, q_R, p_R)`` -- the building block
    of the continuous-pressure direct solve (``nx_fe_set_cp``).

    The cell matrix with the negated pressure rows is ``A(s) = [[s Mref, -Dref^T], [-Dref, 0]]``
    (``s = R h``; ``element_tensors``), and ``A(s) = T A(1) T`` with ``T = diag(s^1/2`` on the
    flux nodes, ``s^-1/2`` on the pressure nodes). So with ``I`` the interior nodes (flux
    ``1..k-1``, then pressure ``1..m-1``) and ``Ah = A(1)``:

    * ``Kh = Ah_VV - Ah_VI Ah_II^-1 Ah_IV`` (4 x 4): the condensed cell matrix is
      ``s^(t_r + t_c) Kh[r, c]``;
    * ``Ch = Ah_VI Ah_II^-1`` (4 x nI): the vertices' rhs ``b_V - s^(t_r - t_c) Ch b_I``;
    * ``Eh = Ah_II^-1 Ah_IV`` (nI x 4), ``Fh = Ah_II^-1``: the interior values
      ``x_I = s^(-t_r - t_c) Fh b_I - s^(-t_r + t_c) Eh x_V``;

    with ``t = +1/2`` on flux and ``-1/2`` on pressure rows / columns (every exponent is -1,
    0 or 1). Exact rational arithmetic, rounded once. Returns ``(Kh, Ch, Eh, Fh, tI)``;
    ``tI``: the interior nodes' types (+1 flux, -1 pressure)."""
    from fractions import Fraction as F

    k, m = int(flux_degree), int(pressure_degree)
    if not (m >= 1 and k > m):
        raise ValueError("continuous pressure needs 1 <= pressure_degree < flux_degree")
    Cq, Cp = lagrange_monomials(k), lagrange_monomials(m)
    dCq = [[c * n for n, c in enumerate(row)][1:] for row in Cq]

    def integ(A, B):
        return [[sum((ap * bq / (p + q + 1) for p, ap in enumerate(a) for q, bq in enumerate(b)),
                     F(0)) for b in B] for a in A]

    M = integ(Cq, Cq)
    D = integ(Cp, dCq)  # (m+1) x (k+1)
    nq, npl = k + 1, m + 1
    n = nq + npl
    Ah = [[F(0)] * n for _ in range(n)]
    for i in range(nq):
        for j in range(nq):
            Ah[i][j] = M[i][j]
    for a in range(npl):
        for j in range(nq):
            Ah[nq + a][j] = -D[a][j]
            Ah[j][nq + a] = -D[a][j]
    V = [0, nq, k, nq + m]
    I = list(range(1, k)) + [nq + a for a in range(1, m)]
    tI = [1] * (k - 1) + [-1] * (m - 1)
    sub = lambda R, Cc: [[Ah[r][c] for c in Cc] for r in R]  # noqa: E731
    AVV, AVI, AIV, AII = sub(V, V), sub(V, I), sub(I, V), sub(I, I)
    nI = len(I)
    Fi = _frac_inverse(AII) if nI else []
    mm = lambda A, B: [[sum((A[i][t] * B[t][j] for t in range(len(B))), F(0))  # noqa: E731
                        for j in range(len(B[0]))] for i in range(len(A))]
    if nI:
        Ch = mm(AVI, Fi)
        Eh = mm(Fi, AIV)
        VIE = mm(AVI, Eh)
        Kh = [[AVV[r][c] - VIE[r][c] for c in range(4)] for r in range(4)]
    else:
        Ch, Eh, Kh = [[] for _ in range(4)], [], AVV
    f64 = lambda X, r, c: np.array([[float(v) for v in row] for row in X],  # noqa: E731
                                   dtype=np.float64).reshape(r, c)
    return (f64(Kh, 4, 4), f64(Ch, 4, nI), f64(Eh, nI, 4), f64(Fi, nI, nI),
            np.array(tI, dtype=np.int32))
