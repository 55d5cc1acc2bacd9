"""The reference's Python surface beyond assemble/solve, on the device path (``-m gpu``):

* ``bilinear_form(i, j)`` / ``linear_form(i)`` return block ``a[i][j]`` / ``L[i]``
  (reference ``assembly.py:378-398``) -- ``None`` exactly where the reference's block is
  None (``assembly.py:284-287``), and each block, extracted from the device-assembled
  system, equals the oracle's reference-form block bit for bit;
* ``Solver.solve`` output (``solver.py:107-135``): functions in the reference's order,
  filled by the device gather into pinned memory; buffers are reused only after the
  functions of a solve are dropped; given functions are filled in place;
* ``Solver.destroy`` (``solver.py:137-143``);
* deferred output: the functions of a solve read their device snapshot when first used.
"""

from __future__ import annotations

import gc

import numpy as np
import pytest

from cases import CASES
from networks_fenicsx_amd import HydraulicNetworkAssembler, NetworkMesh, Solver
from oracle import nx_oracle as O

pytestmark = pytest.mark.gpu


def _setup(case):
    make, N, strategy, pbc = CASES[case]
    mesh = NetworkMesh(make(), N=N, color_strategy=strategy)
    asm = HydraulicNetworkAssembler(mesh)
    asm.compute_forms(p_bc_ex=pbc)
    src, dst = mesh.edges
    P = O.build_problem(mesh.node_coordinates, src, dst, N, mesh.edge_colors)
    A, b = O.assemble_reference(P, pbc)
    return mesh, asm, P, A.tocsr(), b


def _bounds(P):
    return [*P.color_offset, P.lm_offset, P.n_dofs]


@pytest.mark.parametrize("case", ["Y_N4", "depth6_N40", "arterial5_N40", "edge_info_N10"])
def test_form_blocks_match_oracle(case):
    mesh, asm, P, A, b = _setup(case)
    asm.assemble()
    M = mesh.num_edge_colors
    n = M + 2
    bnd = _bounds(P)
    a = asm.bilinear_forms
    assert len(a) == n and all(len(r) == n for r in a)
    for i in range(n):
        for j in range(n):
            blk = asm.bilinear_form(i, j)
            ref = A[bnd[i]:bnd[i + 1], bnd[j]:bnd[j + 1]]
            expect_none = not (i == j < M or (i < M and j >= M) or (j < M and i >= M))
            if expect_none:
                assert blk is None, (i, j)
                assert ref.count_nonzero() == 0, (i, j)
                continue
            got = blk.assemble()
            assert got.shape == ref.shape
            np.testing.assert_array_equal(got.toarray(), ref.toarray())
    kinds = {(0, 0): "mass", (M, 0): "divergence", (0, M): "gradient", (M + 1, 0): "junction",
             (0, M + 1): "junction"}
    for (i, j), k in kinds.items():
        assert asm.bilinear_form(i, j).kind == k
    for i in range(n):
        got = asm.linear_form(i).assemble()
        np.testing.assert_array_equal(got, b[bnd[i]:bnd[i + 1]])
    assert asm.linear_form(M).kind == "source" and asm.linear_form(M + 1).kind == "zero"
    asm.close()


def test_solution_functions_order_and_pinned_reuse():
    mesh, asm, P, A, b = _setup("depth6_N40")
    x_ref = O.solve_reference(A, b)
    solver = Solver(asm)
    solver.assemble()
    sol = solver.solve()
    got = np.concatenate([f.x.array for f in sol])
    assert np.linalg.norm(got - x_ref) / np.linalg.norm(x_ref) <= 1e-10
    names = [f.name for f in sol]
    assert names == [f"flux_color_{c}" for c in range(mesh.num_edge_colors)] + [
        "pressure", "global_flux"]
    # the functions of one solve are views of one buffer
    base = sol[0].x.array.base
    assert all(f.x.array.base is base for f in sol)
    # while they are alive, a second solve uses another buffer
    keep = sol[1].x.array  # a view outlives its function
    before = keep.copy()
    del sol
    gc.collect()
    sol2 = solver.solve()
    assert sol2[0].x.array.base is not base
    np.testing.assert_array_equal(keep, before)
    # once every view of the first buffer is gone it is reused
    del keep, base
    gc.collect()
    sol3 = solver.solve()
    assert sol3[0].x.array.base is not sol2[0].x.array.base
    # given functions are filled in place
    for f in sol3:
        f.x.array[:] = 0.0
    arrays = [f.x.array for f in sol2]
    out = solver.solve(sol2)
    assert out is sol2 and all(f.x.array is a for f, a in zip(out, arrays))
    got = np.concatenate([f.x.array for f in out])
    assert np.linalg.norm(got - x_ref) / np.linalg.norm(x_ref) <= 1e-10
    solver.destroy()
    with pytest.raises(RuntimeError):
        solver.solve()
    # the functions survive the solver and the assembler
    asm.close()
    del solver
    gc.collect()
    got = np.concatenate([f.x.array for f in out])
    assert np.linalg.norm(got - x_ref) / np.linalg.norm(x_ref) <= 1e-10


def test_deferred_functions_keep_their_solve():
    """Functions returned by ``solve`` hold a device snapshot until first read
    (``nx_snapshot_solution``): later solves of a different problem do not change them,
    more unread solves than device slots are read in order, and ``close`` reads the rest."""
    mesh, asm, P, A, b = _setup("depth6_N40")
    x_ref = O.solve_reference(A, b)
    solver = Solver(asm)

    def solve_scaled(s):
        asm.compute_forms(p_bc_ex=lambda x, s=s: s * x[1])
        solver.assemble()
        return solver.solve()

    held = [solve_scaled(s) for s in range(1, 71)]  # 70 unread solves > 64 slots
    assert all(f.x._deferred is not None for f in held[-1])
    for s, sol in reversed(list(enumerate(held, start=1))):
        got = np.concatenate([f.x.array for f in sol])
        assert np.linalg.norm(got - s * x_ref) / np.linalg.norm(s * x_ref) <= 1e-10, s
    # the functions of one solve share one buffer after the read
    assert all(f.x.array.base is held[0][0].x.array.base for f in held[0])
    # unread functions survive the assembler's close
    last = solve_scaled(3)
    solver.destroy()
    asm.close()
    gc.collect()
    got = np.concatenate([f.x.array for f in last])
    assert np.linalg.norm(got - 3 * x_ref) / np.linalg.norm(3 * x_ref) <= 1e-10
    # eager read on request
    mesh, asm, P, A, b = _setup("Y_N4")
    solver = Solver(asm)
    solver.assemble()
    solver.solve()
    eager = asm.solution_functions(deferred=False)
    assert all(f.x._deferred is None for f in eager)
    asm.close()
