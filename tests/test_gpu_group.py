"""Multi-rank path on one GPU: the in-process rank group (``nx_group_*``) runs every rank's
handle -- partition, halo plan, preconditioner with the coarse step, the multi-rank kernel
variants and MINRES schedule of the RCCL path -- with device-copy transport.

Tolerances: the assembled per-rank CSR rows are bit-exact against the oracle's global
matrix cut to the rank (same formulas); the solution is within 1e-10 relative 2-norm of
the oracle's direct solve; with the preconditioner the iteration count stays within 2 of
the single-rank count (the coarse step makes P^{-1} the exact single-rank operator).
"""

from __future__ import annotations

import numpy as np
import pytest
import scipy.sparse as sp

import distributed_model as DM
from cases import CASES, CYCLIC, p_y
from networks_fenicsx_amd import HydraulicNetworkAssembler, NetworkMesh
from networks_fenicsx_amd import network_generation as ng
from networks_fenicsx_amd.group import RankGroup
from oracle import nx_oracle as O

pytestmark = pytest.mark.gpu

SOL_TOL = 1e-10


def _reference(case):
    make, N, strategy, pbc = CASES[case]
    G = make()
    mesh = NetworkMesh(G, N=N, color_strategy=strategy)
    src, dst = mesh.edges
    P = O.build_problem(mesh.node_coordinates, src, dst, N, mesh.edge_colors)
    A, b = O.assemble_reference(P, pbc)
    Ab, bb, perm, sign = O.to_build_layout(P, A, b)
    x_ref = O.solve_reference(A, b)[perm]
    return G, mesh, Ab, bb, x_ref


def _single_iterations(mesh, pbc, pc: bool) -> int:
    asm = HydraulicNetworkAssembler(mesh)
    asm.compute_forms(p_bc_ex=pbc)
    asm.assemble()
    asm.set_preconditioner(pc)
    it, _, conv = asm.handle.solve(1e-12, 50000, 32)
    assert conv
    asm.close()
    return it


@pytest.mark.parametrize("case,P,pc", [
    ("depth6_N40", 2, True), ("depth6_N40", 4, True), ("depth6_N40", 8, True),
    ("depth6_N40", 4, False), ("arterial5_N40", 3, True), ("edge_info_N10", 2, True),
    ("tree6_2d_N70", 5, True), ("linear_alt_N3", 3, True), ("double_Y_N5", 2, False),
    ("Y_N4", 2, True),
])
def test_group_solve_matches_direct(case, P, pc):
    make, N, strategy, pbc = CASES[case]
    G, mesh, Ab, bb, x_ref = _reference(case)
    grp = RankGroup(G, N, P, color_strategy=strategy)
    try:
        grp.compute_forms(p_bc_ex=pbc)
        grp.assemble()
        grp.set_preconditioner(pc)
        # per-rank CSR rows and rhs: the global build-layout matrix cut to the rank
        bif = mesh.bifurcation_index
        for a in grp.assemblers:
            lp = a.local_problem
            Al, rows = DM.local_matrix(Ab, lp, mesh.num_edges, bif)
            Al = Al.tocsr()
            Al.sort_indices()
            rp, col, val = a.handle.csr()
            Ad = sp.csr_matrix((val, col, rp), shape=Al.shape)
            Ad.sort_indices()
            np.testing.assert_array_equal(Ad.indptr, Al.indptr)
            np.testing.assert_array_equal(Ad.indices, Al.indices)
            np.testing.assert_array_equal(Ad.data, Al.data)
            np.testing.assert_array_equal(a.handle.rhs(), bb[rows])
        it, relres, conv = grp.solve(1e-12, 50000, 32)
        assert conv, (it, relres)
        x = np.zeros(Ab.shape[0])
        for a, xl in zip(grp.assemblers, grp.solutions()):
            x[DM.global_rows(a.local_problem, mesh.num_edges, bif)] = xl
        err = np.linalg.norm(x - x_ref) / np.linalg.norm(x_ref)
        assert err <= SOL_TOL, err
        if pc and mesh.num_edges == mesh.num_nodes - 1:  # trees: exact preconditioner
            it1 = _single_iterations(mesh, pbc, True)
            assert it <= it1 + 2 and it <= 4, (it, it1)
    finally:
        grp.close()


@pytest.mark.parametrize("env", [{}, {"NXHIP_PC_GLOBAL": "1"}])
def test_group_alternative_kernel_paths(env, monkeypatch):
    """The multi-rank MINRES with the LDS sweeps (linear form, fused coarse steps, dense top,
    beta^2 point-to-point) and with the global-memory preconditioner kernels
    (NXHIP_PC_GLOBAL=1: the fallback when a job exceeds the LDS caps -- alpha with its own
    all-reduce, separate k_pc_cpart / k_pc_coarse kernels, the per-iteration top kernel)."""
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    case, P = "depth6_N40", 4
    make, N, strategy, pbc = CASES[case]
    G, mesh, Ab, bb, x_ref = _reference(case)
    grp = RankGroup(G, N, P, color_strategy=strategy)
    try:
        grp.compute_forms(p_bc_ex=pbc)
        grp.assemble()
        it, relres, conv = grp.solve(1e-12, 50000, 32)
        assert conv
        x = np.zeros(Ab.shape[0])
        for a, xl in zip(grp.assemblers, grp.solutions()):
            x[DM.global_rows(a.local_problem, mesh.num_edges, mesh.bifurcation_index)] = xl
        assert np.linalg.norm(x - x_ref) / np.linalg.norm(x_ref) <= SOL_TOL
        assert it <= _single_iterations(mesh, pbc, True) + 2
    finally:
        grp.close()


@pytest.mark.parametrize("case,P", [("depth6_N40", 4), ("arterial5_N40", 3), ("tree6_2d_N70", 5)])
def test_group_lean_graph_matches_general_path(case, P):
    """One graph per solve (start, coefficients, iterations, published state) vs the
    general path (eager prologue, chunked iterations): same iterations and solution."""
    from networks_fenicsx_amd import _lib

    make, N, strategy, pbc = CASES[case]
    G, mesh, Ab, bb, x_ref = _reference(case)
    grp = RankGroup(G, N, P, color_strategy=strategy)
    try:
        grp.compute_forms(p_bc_ex=pbc)
        grp.assemble()
        out = {}
        for lean in (True, False):
            _lib.set_lean(lean)
            it, relres, conv = grp.solve(1e-12, 50000, 4)
            assert conv
            x = np.zeros(Ab.shape[0])
            for a, xl in zip(grp.assemblers, grp.solutions()):
                x[DM.global_rows(a.local_problem, mesh.num_edges, mesh.bifurcation_index)] = xl
            assert np.linalg.norm(x - x_ref) / np.linalg.norm(x_ref) <= SOL_TOL
            out[lean] = (it, x)
        assert out[True][0] == out[False][0]
        assert np.linalg.norm(out[True][1] - out[False][1]) <= 1e-12 * np.linalg.norm(x_ref)
    finally:
        _lib.set_lean(True)
        grp.close()


def test_group_large_tree_iterations_flat():
    """Depth-10 binary tree (N=15, ~61k DoF) on 8 ranks: same iteration count as 1 rank
    (block-Jacobi grounding of the cuts would need ~5x more)."""
    G = ng.make_tree(11, 11, 11)
    pbc = lambda x: x[1]  # noqa: E731
    mesh = NetworkMesh(G, N=15)
    it1 = _single_iterations(mesh, pbc, True)
    grp = RankGroup(G, 15, 8)
    try:
        grp.compute_forms(p_bc_ex=pbc)
        grp.assemble()
        it, relres, conv = grp.solve(1e-12, 50000, 32)
        assert conv
        assert it <= it1 + 2 and it <= 4, (it, it1)
    finally:
        grp.close()


@pytest.mark.parametrize("case,P", [("depth6_N40", 4), ("arterial5_N40", 3), ("Y_N4", 2)])
def test_group_direct_cut_rows_in_one_allreduce(case, P, monkeypatch):
    """The cut bifurcations' multiplier rows completed inside the residual's all-reduce
    (nx_set_cut, default) against the halo of x + all-reduce of two (NXHIP_DIR_CUT=0), and
    the coarse step inside the down sweeps (default) against k_pc_coarse
    (NXHIP_DIR_COARSE_DOWN=0): the same solution bit for bit, the same reported residual to
    its rounding, and a forced refinement pass (which starts from the stored cut rows' r and
    refines the top values in the down sweeps) converges to the true residual."""
    monkeypatch.setenv("NXHIP_DIR_XR", "0")  # the graph path's modes (the exchange step: below)
    make, N, strategy, pbc = CASES[case]
    G, mesh, Ab, bb, x_ref = _reference(case)
    grp = RankGroup(G, N, P, color_strategy=strategy)

    def gathered():
        x = np.zeros(Ab.shape[0])
        for a, xl in zip(grp.assemblers, grp.solutions()):
            x[DM.global_rows(a.local_problem, mesh.num_edges, mesh.bifurcation_index)] = xl
        return x

    try:
        assert grp.assemblers[0].local_problem.n_cut > 0
        grp.compute_forms(p_bc_ex=pbc)
        grp.set_direct(True)
        grp.assemble()
        it, rr, conv = grp.solve(1e-12, 50000, 4)
        assert conv and it == 1 and grp.solver_used == "direct"
        x1 = gathered()
        true1 = np.linalg.norm(bb - Ab @ x1) / np.linalg.norm(bb)
        assert abs(rr - true1) <= 0.05 * true1 + 5e-16, (rr, true1)
        monkeypatch.setenv("NXHIP_DIR_CUT", "0")  # (and so k_pc_coarse, see below)
        grp.assemble()
        it0, rr0, _ = grp.solve(1e-12, 50000, 4)
        np.testing.assert_array_equal(gathered(), x1)
        assert abs(rr0 - rr) <= 1e-6 * rr0 + 5e-16, (rr0, rr)
        monkeypatch.delenv("NXHIP_DIR_CUT")
        # the coarse step in every down workgroup (default) against the k_pc_coarse kernel
        monkeypatch.setenv("NXHIP_DIR_COARSE_DOWN", "0")
        grp.assemble()
        it0, rr0, _ = grp.solve(1e-12, 50000, 4)
        np.testing.assert_array_equal(gathered(), x1)
        # (the same x and the same reported residual bit for bit: the cut rows' sums skip the
        # ghost columns, whatever the halo run above left there)
        assert rr0 == rr, (rr0, rr)
        monkeypatch.delenv("NXHIP_DIR_COARSE_DOWN")
        if rr > 4e-15:  # room for a refinement step below the first pass's residual
            grp.assemble()
            it2, rr2, conv2 = grp.solve(rr / 2, 50000, 4)
            assert it2 == 2 and conv2 and grp.solver_used == "direct", (it2, rr2)
            x2 = gathered()
            true2 = np.linalg.norm(bb - Ab @ x2) / np.linalg.norm(bb)
            assert rr2 <= rr / 2 and abs(rr2 - true2) <= 0.05 * true2 + 5e-16, (rr2, true2)
            assert np.linalg.norm(x2 - x_ref) / np.linalg.norm(x_ref) <= SOL_TOL
    finally:
        grp.close()


@pytest.mark.parametrize("pc", [True, False])
def test_rccl_single_rank_communicator(pc):
    """A one-rank RCCL communicator drives the RCCL transport code (unique id, comm init,
    ncclAllReduce, grouped send/recv, eager launches, the multi-rank kernel variants) on
    one GPU; results must equal the single-handle solve."""
    from networks_fenicsx_amd import _lib

    make, N, strategy, pbc = CASES["depth6_N40"]
    G, mesh, Ab, bb, x_ref = _reference("depth6_N40")
    asm = HydraulicNetworkAssembler(mesh)
    try:
        lp = asm.local_problem
        asm.handle.comm_init(1, 0, _lib.comm_unique_id(), lp.peers, lp.send_off, lp.send_idx,
                             lp.recv_off)
        asm.set_preconditioner(pc)
        asm.compute_forms(p_bc_ex=pbc)
        asm.assemble()
        it, relres, conv = asm.handle.solve(1e-12, 50000, 32)
        assert conv
        x = asm.handle.solution()
        assert np.linalg.norm(x - x_ref) / np.linalg.norm(x_ref) <= SOL_TOL
        assert it <= _single_iterations(mesh, pbc, pc) + 2
        assert asm.handle.graph_mode()  # the RCCL iterations were captured as HIP graphs
        assert asm.handle.true_residual() < 1e-9
    finally:
        asm.close()


def _forced_coarse_direct(case: str, terminals, transport: str, then_lumped: bool = False):
    """One rank whose coarse set is forced (``coarse_structure(terminals=...)``: junctions
    kept out of the local eliminations exactly as interface junctions are), so the
    multi-rank direct schedule (``launch_direct_team``) runs on one GPU. ``transport``:
    ``"rccl"`` (a one-rank RCCL communicator) or ``"group"`` (a one-rank in-process group).
    ``then_lumped``: after the first solve switch the preconditioner to the lumped mass and
    solve again (the results are the second solve's).
    Returns (solution, iterations, relres, solver used, graph mode, true residual)."""
    from networks_fenicsx_amd import _lib
    from networks_fenicsx_amd.precond import build_tree_preconditioner, coarse_structure

    make, N, strategy, pbc = CASES[case]
    mesh = NetworkMesh(make(), N=N, color_strategy=strategy)
    src, dst = mesh.edges
    cs = coarse_structure(src, dst, mesh.degrees, np.zeros(src.size, np.int64), 1,
                          terminals=terminals)
    assert cs.n >= len(terminals)
    asm = HydraulicNetworkAssembler(mesh)
    grp = None
    try:
        lp = asm.local_problem
        h = asm.handle
        if transport == "rccl":
            h.comm_init(1, 0, _lib.comm_unique_id(), lp.peers, lp.send_off, lp.send_idx,
                        lp.recv_off)
        # no cut bifurcation on one rank: every multiplier row is this rank's own
        h.set_cut(0, np.full(lp.lm_nodes.size, -1, np.int32), np.zeros(1, np.int32),
                  np.zeros(0, np.int32), np.zeros(0))
        asm._pc = build_tree_preconditioner(lp, src, dst, mesh.degrees, coarse=cs)
        assert asm._pc.n_coarse == cs.n
        asm.set_preconditioner(True)
        asm.set_direct(True)
        asm.compute_forms(p_bc_ex=pbc)
        asm.assemble()
        if transport == "group":
            grp = _lib.Group([h])
        it, rr, conv = (h if grp is None else grp).solve(1e-12, 50000, 4)
        if then_lumped:
            assert h.solver()[1] == 1
            h.set_pc_exact(False)
            asm.assemble()
            it, rr, conv = (h if grp is None else grp).solve(1e-12, 50000, 4)
        assert conv, (it, rr)
        used = "direct" if h.solver()[1] == 1 else "minres"
        # (a group member's residual needs every rank's solution: RCCL only)
        out = (h.solution(), it, rr, used, h.graph_mode(),
               h.true_residual() if grp is None else None)
        if grp is not None:
            grp.close()
            grp = None
        return out
    finally:
        if grp is not None:
            grp.close()
        asm.close()


@pytest.mark.parametrize("case,n_term", [("depth6_N40", 1), ("depth6_N40", 3),
                                         ("arterial5_N40", 2)])
def test_rccl_direct_single_rank_communicator(case, n_term):
    """The RCCL direct solve -- the bench's default at P > 1 (launch_direct_team over a
    communicator: the schedule signature's all-reduce with direct_all, the coarse
    all-reduce, the cut rows' residual all-reduce, captured as one HIP graph) -- on a
    one-rank communicator with a forced coarse set: solver_used == "direct", the RCCL graph
    ran, the oracle's direct solution to 1e-10, and bit for bit the in-process group's
    result (same kernels and decomposition, device-copy transport). Replaces the reference's
    distributed solve (solver.py:127-132)."""
    G, mesh, Ab, bb, x_ref = _reference(case)
    bif = np.asarray(mesh.bifurcation_values)
    terms = bif[np.linspace(0, bif.size - 1, n_term).astype(np.int64)]
    x1, it1, rr1, used1, graph1, true1 = _forced_coarse_direct(case, terms, "rccl")
    assert used1 == "direct" and it1 in (1, 2), (used1, it1)
    assert graph1, "the RCCL direct solve was not captured as a HIP graph"
    assert np.linalg.norm(x1 - x_ref) / np.linalg.norm(x_ref) <= SOL_TOL
    assert rr1 <= 1e-12 and true1 <= 1e-12, (rr1, true1)
    x2, it2, rr2, used2, _, _ = _forced_coarse_direct(case, terms, "group")
    assert used2 == "direct" and it2 == it1
    np.testing.assert_array_equal(x1, x2)
    assert rr1 == rr2


def test_rccl_direct_follows_pc_mass_switch():
    """over RCCL the ranks' direct decision is cached with the schedule check;
    switching the preconditioner's mass to lumped (nx_set_pc_exact) after a direct solve
    must invalidate it, so the next solve runs MINRES (the direct solve needs the exact
    Schur complement)."""
    G, mesh, Ab, bb, x_ref = _reference("depth6_N40")
    terms = np.asarray(mesh.bifurcation_values)[:1]
    x, it, rr, used, _, _ = _forced_coarse_direct("depth6_N40", terms, "rccl", then_lumped=True)
    assert used == "minres"
    assert np.linalg.norm(x - x_ref) / np.linalg.norm(x_ref) <= SOL_TOL


def test_group_ranks_with_different_schedules_fail_loudly(monkeypatch):
    """A rank whose preconditioner runs another kernel schedule (here: the global-memory
    kernels on rank 1 only) must make the solve fail, not pair mismatched exchanges."""
    from networks_fenicsx_amd._lib import NxError

    make, N, strategy, pbc = CASES["depth6_N40"]
    grp = RankGroup(make(), N, 2, color_strategy=strategy)
    try:
        grp.compute_forms(p_bc_ex=pbc)
        grp.assemble()
        monkeypatch.setenv("NXHIP_PC_GLOBAL", "1")
        grp.assemblers[1].set_preconditioner(True)
        monkeypatch.delenv("NXHIP_PC_GLOBAL")
        with pytest.raises(NxError, match="different kernel schedules"):
            grp.solve(1e-12, 50000, 32)
        grp._close_group()
        grp.assemblers[1].set_preconditioner(True)  # same schedule again: solves
        it, _, conv = grp.solve(1e-12, 50000, 32)
        assert conv
    finally:
        grp.close()


def test_group_ranks_agree_on_sweep_kernels(monkeypatch):
    """A rank that cannot run the LDS sweeps (here forced: the global-memory kernels on rank 1
    only) makes every rank take the global-memory kernels (RankGroup._agree_kernels, over a
    communicator HydraulicNetworkAssembler.set_preconditioner's MIN all-reduce), so the
    solve runs -- MINRES, the direct solve needs the LDS sweeps across ranks -- instead of
    failing on mismatched schedules."""
    make, N, strategy, pbc = CASES["depth6_N40"]
    G, mesh, Ab, bb, x_ref = _reference("depth6_N40")
    grp = RankGroup(G, N, 2, color_strategy=strategy)
    try:
        grp.compute_forms(p_bc_ex=pbc)
        grp.assemble()
        monkeypatch.setenv("NXHIP_PC_GLOBAL", "1")
        grp.assemblers[1].set_preconditioner(True)
        monkeypatch.delenv("NXHIP_PC_GLOBAL")
        assert [a.handle.pc_lds() for a in grp.assemblers] == [True, False]
        grp._agree_kernels()
        assert [a.handle.pc_lds() for a in grp.assemblers] == [False, False]
        grp.set_direct(True)
        it, relres, conv = grp.solve(1e-12, 50000, 32)
        assert conv and grp.solver_used == "minres"
        x = np.zeros(Ab.shape[0])
        for a, xl in zip(grp.assemblers, grp.solutions()):
            x[DM.global_rows(a.local_problem, mesh.num_edges, mesh.bifurcation_index)] = xl
        assert np.linalg.norm(x - x_ref) / np.linalg.norm(x_ref) <= SOL_TOL
    finally:
        grp.close()


def test_group_rank_without_dense_top_fails_loudly(monkeypatch):
    """The dense top part is decided per rank (nx_set_pc_dense); it drives who packs the
    halo and beta^2 (fuse_pack). A rank without it must make the solve fail through the
    schedule check, never run with peers reading stale halo values."""
    from networks_fenicsx_amd._lib import NxError

    make, N, strategy, pbc = CASES["depth6_N40"]
    grp = RankGroup(make(), N, 2, color_strategy=strategy)
    try:
        grp.compute_forms(p_bc_ex=pbc)
        grp.assemble()
        import dataclasses

        a1 = grp.assemblers[1]  # its decomposition uploaded without the dense top's lists
        a1.handle.set_preconditioner(dataclasses.replace(
            a1.tree_preconditioner, job_tslot=np.zeros(0, np.int32)))
        with pytest.raises(NxError, match="different kernel schedules"):
            grp.solve(1e-12, 50000, 4)
        grp._close_group()
        grp.assemblers[1].set_preconditioner(True)
        it, _, conv = grp.solve(1e-12, 50000, 4)
        assert conv and it <= 4
    finally:
        grp.close()


def test_group_rehearsal_four_ranks_depth16():
    """4 ranks x make_tree(17) (1 M rows per rank): the size at which the depth-cut
    decomposition put a job over the LDS caps on some ranks and the ranks diverged
    (DESIGN.md section 6). Exact preconditioner: 3 iterations, analytic answer."""
    G = ng.make_tree(17, 17, 17)
    grp = RankGroup(G, 15, 4, color_strategy="smallest_last")
    try:
        grp.compute_forms(p_bc_ex=lambda x: x[1])
        grp.assemble()
        it, _, conv = grp.solve(1e-12, 50000, 4)
        assert conv and it == 3
        m0 = grp.meshes[0]
        src, dst = m0.edges
        P = O.build_problem(m0.node_coordinates, src, dst, 15)
        xa = O.resistor_network_solution(P, lambda x: x[1])[O.build_permutation(P)[0]]
        x = np.full(xa.size, np.nan)
        for a, xl in zip(grp.assemblers, grp.solutions()):
            x[DM.global_rows(a.local_problem, m0.num_edges, m0.bifurcation_index)] = xl
        assert np.linalg.norm(x - xa) / np.linalg.norm(xa) < 1e-10
    finally:
        grp.close()


@pytest.mark.parametrize("case,P", [("depth6_N40", 2), ("depth6_N40", 4), ("depth6_N40", 8),
                                    ("arterial5_N40", 3), ("tree6_2d_N70", 5),
                                    ("linear_alt_N3", 3), ("Y_N4", 2), ("edge_info_N10", 2)])
def test_group_direct_solve(case, P):
    """The direct tree solve across ranks (mode kModeDirect of the multi-rank sweeps, coarse
    all-reduce between the halves, halo of x, all-reduced true residual): the oracle's
    direct solution to 1e-10; graphs with a cycle too, through every rank's share of the
    Woodbury correction (nx_set_cycles_team)."""
    make, N, strategy, pbc = CASES[case]
    G, mesh, Ab, bb, x_ref = _reference(case)
    grp = RankGroup(G, N, P, color_strategy=strategy)
    try:
        grp.compute_forms(p_bc_ex=pbc)
        grp.set_direct(True)
        grp.assemble()  # (pending: both solves below take the same path -- the exchange step)
        it, relres, conv = grp.solve(1e-12, 50000, 4)
        assert conv, (it, relres)
        is_tree = mesh.num_edges == mesh.num_nodes - 1
        assert grp.solver_used == "direct"
        assert it in (1, 2) and relres <= 1e-12
        x = np.zeros(Ab.shape[0])
        for a, xl in zip(grp.assemblers, grp.solutions()):
            x[DM.global_rows(a.local_problem, mesh.num_edges, mesh.bifurcation_index)] = xl
        err = np.linalg.norm(x - x_ref) / np.linalg.norm(x_ref)
        assert err <= SOL_TOL, err
        # the reported residual (fused into the down sweeps; with cycles the CSR's after the
        # correction) is the true one
        true = np.linalg.norm(bb - Ab @ x) / np.linalg.norm(bb)
        assert abs(relres - true) <= 0.05 * true + 5e-16, (relres, true, is_tree)
        # again: the captured graphs are reused and the result does not move
        grp.assemble()
        grp.solve(1e-12, 50000, 4)
        x2 = np.zeros(Ab.shape[0])
        for a, xl in zip(grp.assemblers, grp.solutions()):
            x2[DM.global_rows(a.local_problem, mesh.num_edges, mesh.bifurcation_index)] = xl
        np.testing.assert_array_equal(x2, x)
    finally:
        grp.close()


def _gathered(grp, Ab, mesh):
    x = np.zeros(Ab.shape[0])
    for a, xl in zip(grp.assemblers, grp.solutions()):
        x[DM.global_rows(a.local_problem, mesh.num_edges, mesh.bifurcation_index)] = xl
    return x


@pytest.mark.parametrize("case,P", [("depth6_N40", 2), ("depth6_N40", 4), ("arterial5_N40", 3),
                                    ("Y_N4", 2), ("linear_alt_N3", 3), ("tree5_N15", 4)])
def test_group_exchange_step(case, P, monkeypatch):
    """The direct step of several ranks in ONE launch per rank (k_dir_xg: every rank's
    workgroups in one launch, exchanging the coarse partials and the residual's partials
    through device mailboxes instead of the two RCCL all-reduces): the oracle's solution to
    1e-10, the graph path's (NXHIP_DIR_XR=0) to its rounding, the reported residual the true
    one, the same bits on every repeated step, and the ranks' published residuals equal."""
    make, N, strategy, pbc = CASES[case]
    G, mesh, Ab, bb, x_ref = _reference(case)
    grp = RankGroup(G, N, P, color_strategy=strategy)
    try:
        grp.compute_forms(p_bc_ex=pbc)
        grp.set_direct(True)
        grp.assemble()
        it, rr, conv = grp.solve(1e-12, 50000, 4)
        assert conv and it == 1 and grp.solver_used == "direct"
        paths = {a.handle.direct_path() for a in grp.assemblers}
        assert paths == {"exchange"}, paths
        x1 = _gathered(grp, Ab, mesh)
        assert np.linalg.norm(x1 - x_ref) / np.linalg.norm(x_ref) <= SOL_TOL
        true1 = np.linalg.norm(bb - Ab @ x1) / np.linalg.norm(bb)
        assert abs(rr - true1) <= 0.05 * true1 + 5e-16, (rr, true1)
        for _ in range(20):  # the exchanges' tags move on; the bits do not
            grp.assemble()
            it2, rr2, _ = grp.solve(1e-12, 50000, 4)
            assert rr2 == rr and {a.handle.direct_path() for a in grp.assemblers} == {"exchange"}
            np.testing.assert_array_equal(_gathered(grp, Ab, mesh), x1)
        monkeypatch.setenv("NXHIP_DIR_XR", "0")  # the graph path (RCCL-shaped all-reduces)
        grp.assemble()
        it0, rr0, conv0 = grp.solve(1e-12, 50000, 4)
        assert conv0 and {a.handle.direct_path() for a in grp.assemblers} == {"launches"}
        x0 = _gathered(grp, Ab, mesh)
        assert np.linalg.norm(x0 - x1) <= 1e-14 * np.linalg.norm(x1)
        assert abs(rr0 - rr) <= 0.05 * rr0 + 5e-16, (rr0, rr)
    finally:
        grp.close()


@pytest.mark.parametrize("case,P", [("depth6_N40", 2), ("arterial5_N40", 3), ("tree5_N15", 4)])
def test_separate_launches_exchange(case, P):
    """The RCCL ranks' shape of the exchange step: every rank's k_dir_xr as its own launch on
    its own stream (one-handle teams: the exchange width is the rank count, not the team
    size), meeting only through the mailboxes -- the same bits as the group's one launch
    (k_dir_xg), the oracle to 1e-10, on every repeated step."""
    make, N, strategy, pbc = CASES[case]
    G, mesh, Ab, bb, x_ref = _reference(case)
    grp = RankGroup(G, N, P, color_strategy=strategy)
    try:
        grp.compute_forms(p_bc_ex=pbc)
        grp.set_direct(True)
        grp.assemble()
        it, rr, conv = grp.solve(1e-12, 50000, 4)
        assert conv and {a.handle.direct_path() for a in grp.assemblers} == {"exchange"}
        x1 = _gathered(grp, Ab, mesh)
        for _ in range(5):
            grp.assemble()
            rr2 = grp._group.xr_separate(1e-12)
            assert {a.handle.direct_path() for a in grp.assemblers} == {"exchange"}
            np.testing.assert_array_equal(_gathered(grp, Ab, mesh), x1)
            assert rr2 == rr, (rr2, rr)
        assert np.linalg.norm(x1 - x_ref) / np.linalg.norm(x_ref) <= SOL_TOL
        grp.assemble()  # and the group's launch again after them
        it, rr3, _ = grp.solve(1e-12, 50000, 4)
        assert rr3 == rr
        np.testing.assert_array_equal(_gathered(grp, Ab, mesh), x1)
    finally:
        grp.close()


def test_group_exchange_give_up_falls_back():
    """Every waiting workgroup gives up (a wait bound of 0 polls): no rank publishes, the host
    resets the hand-off counters and sequence numbers, and the same solve runs the graph
    path -- correct, and so is every later step."""
    case, P = "depth6_N40", 3
    make, N, strategy, pbc = CASES[case]
    G, mesh, Ab, bb, x_ref = _reference(case)
    grp = RankGroup(G, N, P, color_strategy=strategy)
    try:
        grp.compute_forms(p_bc_ex=pbc)
        grp.set_direct(True)
        for a in grp.assemblers:
            a.handle.set_wait_polls(0)
        for _ in range(3):
            grp.assemble()
            it, rr, conv = grp.solve(1e-12, 50000, 4)
            assert conv and grp.solver_used == "direct"
            assert {a.handle.direct_path() for a in grp.assemblers} == {"launches"}
            x = _gathered(grp, Ab, mesh)
            assert np.linalg.norm(x - x_ref) / np.linalg.norm(x_ref) <= SOL_TOL
    finally:
        grp.close()


@pytest.mark.parametrize("separate", [False, True])
def test_exchange_one_rank_gives_up_exchange2(separate):
    """One rank's exchange 2 gives up at once (nx_debug_xr_polls(1, 0): after its own slots
    and flags went out) while the others finish it -- in the group's one launch and as
    separate concurrent launches (the RCCL ranks' shape). The rank's host finishes exchange
    2 from its mailbox with the same bits, so every rank ends the step on the exchange path
    with the oracle's answer and the same residual; 5 further steps stay on it, bit for bit."""
    case, P = "depth6_N40", 3
    make, N, strategy, pbc = CASES[case]
    G, mesh, Ab, bb, x_ref = _reference(case)
    grp = RankGroup(G, N, P, color_strategy=strategy)
    try:
        grp.compute_forms(p_bc_ex=pbc)
        grp.set_direct(True)
        grp.assemble()
        _, rr, conv = grp.solve(1e-12, 50000, 4)
        assert conv and {a.handle.direct_path() for a in grp.assemblers} == {"exchange"}
        x1 = _gathered(grp, Ab, mesh)
        grp.assemblers[1].handle.xr_polls(1, 0)
        for k in range(6):
            grp.assemble()
            if separate:
                rr2 = grp._group.xr_separate(1e-12)
            else:
                _, rr2, _ = grp.solve(1e-12, 50000, 4)
            st = [a.handle.xr_status() for a in grp.assemblers]
            assert {a.handle.direct_path() for a in grp.assemblers} == {"exchange"}, (k, st)
            assert not any(s["off"] for s in st), st
            if k == 0:  # (the hook: given up, finished on the host)
                assert st[1]["why"] & 2, st
            else:
                assert all(s["why"] == 0 for s in st), (k, st)
            assert rr2 == rr
            np.testing.assert_array_equal(_gathered(grp, Ab, mesh), x1)
            if k == 0:
                grp.assemblers[1].handle.xr_polls(1, 1 << 20)  # (steps 1..5: no give-up)
        assert np.linalg.norm(x1 - x_ref) / np.linalg.norm(x_ref) <= SOL_TOL
    finally:
        grp.close()


@pytest.mark.parametrize("separate", [False, True])
def test_exchange_one_rank_gives_up_exchange1(separate):
    """One rank's exchange 1 gives up at once: that step cannot finish anywhere (the rank
    never sends its residual share), every rank's launch gives up -- the others on its
    abort word -- and every rank solves it and the 5 steps after it on the graph path: the
    same path on every rank, the oracle's answer every step."""
    case, P = "depth6_N40", 3
    make, N, strategy, pbc = CASES[case]
    G, mesh, Ab, bb, x_ref = _reference(case)
    grp = RankGroup(G, N, P, color_strategy=strategy)
    try:
        grp.compute_forms(p_bc_ex=pbc)
        grp.set_direct(True)
        grp.assemble()
        grp.solve(1e-12, 50000, 4)
        assert {a.handle.direct_path() for a in grp.assemblers} == {"exchange"}
        grp.assemblers[1].handle.xr_polls(0, 0)
        grp.assemble()
        if separate:
            rr = grp._group.xr_separate(1e-12)
        else:
            _, rr, conv = grp.solve(1e-12, 50000, 4)
            assert conv
        st = [a.handle.xr_status() for a in grp.assemblers]
        assert all(s["off"] and s["agreed"] == 1 for s in st), st
        assert st[1]["why"] & 1 and all(s["why"] & 4 for q, s in enumerate(st) if q != 1), st
        assert rr <= 1e-12
        for k in range(6):
            if k:
                grp.assemble()
                _, rr, conv = grp.solve(1e-12, 50000, 4)
                assert conv and rr <= 1e-12
            assert {a.handle.direct_path() for a in grp.assemblers} == {"launches"}, k
            x = _gathered(grp, Ab, mesh)
            assert np.linalg.norm(x - x_ref) / np.linalg.norm(x_ref) <= SOL_TOL, k
    finally:
        grp.close()



@pytest.mark.parametrize("case,P", [("edge_info_N10", 3), ("lattice4x5_N6", 2),
                                    ("lattice4x5_N6", 3), ("lattice6x6_N3", 4),
                                    ("lattice19x20_N2", 3)])
def test_group_direct_solve_cycles(case, P):
    """Graphs with cycles across ranks: cycle chains inside a rank and coarse chains closing a
    cycle between ranks are grounded by the decomposition; every rank holds its share of Z =
    A_g^{-1} U (2K team tree solves per assembled matrix) and the same capacitance inverse,
    and each solve sums U^T x over the ranks and corrects x: the oracle's LU to 1e-10, the
    reported residual the CSR's true one, the same bits on a second step, a new matrix (R
    changed) rebuilds the correction."""
    make, N = CYCLIC[case]
    G = make()
    mesh = NetworkMesh(G, N=N)
    src, dst = mesh.edges
    Pr = O.build_problem(mesh.node_coordinates, src, dst, N, mesh.edge_colors)
    A, b = O.assemble_reference(Pr, p_y)
    Ab, bb, perm, _ = O.to_build_layout(Pr, A, b)
    x_ref = O.solve_reference(A, b)[perm]
    grp = RankGroup(G, N, P)
    try:
        grp.compute_forms(p_bc_ex=p_y)
        grp.set_direct(True)
        grp.assemble()
        it, rr, conv = grp.solve(1e-12, 50000, 4)
        assert conv and grp.solver_used == "direct" and it in (1, 2), (it, rr)
        x = _gathered(grp, Ab, mesh)
        assert np.linalg.norm(x - x_ref) / np.linalg.norm(x_ref) <= SOL_TOL
        true = np.linalg.norm(bb - Ab @ x) / np.linalg.norm(bb)
        assert abs(rr - true) <= 0.05 * true + 5e-16, (rr, true)
        grp.assemble()
        it2, rr2, _ = grp.solve(1e-12, 50000, 4)
        np.testing.assert_array_equal(_gathered(grp, Ab, mesh), x)
        # another matrix: R = 2 everywhere (the correction is rebuilt for it)
        grp.compute_forms(p_bc_ex=p_y, R=2.0)
        grp.assemble()
        it3, rr3, conv3 = grp.solve(1e-12, 50000, 4)
        assert conv3 and grp.solver_used == "direct"
        A2, b2 = O.assemble_reference(Pr, p_y, R=2.0)
        x2_ref = O.solve_reference(A2, b2)[perm]
        x2 = _gathered(grp, Ab, mesh)
        assert np.linalg.norm(x2 - x2_ref) / np.linalg.norm(x2_ref) <= SOL_TOL
    finally:
        grp.close()
