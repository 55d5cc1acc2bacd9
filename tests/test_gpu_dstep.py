"""The fused direct step (``k_dir_step``, one rank): the deferred
assembly, the whole tree solve, the residual check and the published state in ONE launch of
one workgroup per job, with write-through hand-offs between the workgroups instead of
kernel boundaries.

Bar: what it assembles (CSR values, rhs, and through MINRES the lumped mass) is bit-exact
against the oracle and the assembly kernel; its solution equals the separate launches'
(``NXHIP_DIR_FUSED=0``: k_assemble_seg, up, down, publish) to 1e-14 relative 2-norm and the
oracle's direct solve to 1e-10; its reported residual is the true one to 5 %."""

from __future__ import annotations

import numpy as np
import pytest

from cases import CASES
from networks_fenicsx_amd import HydraulicNetworkAssembler, NetworkMesh
from networks_fenicsx_amd import network_generation as ng
from oracle import nx_oracle as O

pytestmark = pytest.mark.gpu

SOL_TOL = 1e-10
TREES = ["Y_N4", "demo_tree_N1", "demo_tree_N2", "double_Y_N5", "depth6_N40", "arterial5_N40",
         "tree6_2d_N70", "linear_alt_N3", "tree5_N15", "tree5_N16", "tree5_3d_N31"]


def _setup(case, **forms):
    make, N, strategy, pbc = CASES[case]
    mesh = NetworkMesh(make(), N=N, color_strategy=strategy)
    asm = HydraulicNetworkAssembler(mesh)
    asm.compute_forms(p_bc_ex=pbc, **forms)
    asm.set_direct(True)
    src, dst = mesh.edges
    P = O.build_problem(mesh.node_coordinates, src, dst, N, mesh.edge_colors)
    A, b = O.assemble_reference(P, pbc, **forms)
    return mesh, asm, P, A, b


@pytest.mark.parametrize("case", TREES)
def test_dstep_matches_oracle_and_launches(case, monkeypatch):
    mesh, asm, P, A, b = _setup(case)
    h = asm.handle
    asm.assemble()
    it, rr, conv = h.solve(1e-12, 100, 4)
    assert h.direct_path() == "fused" and h.solver() == (1, 1)
    assert conv and it == 1 and rr <= 1e-12
    x1 = h.solution()
    # what the fused kernel assembled: the oracle's CSR values and rhs, bit for bit
    Ab, bb, perm, _ = O.to_build_layout(P, A, b)
    rp, col, val = h.csr()
    np.testing.assert_array_equal(rp, Ab.indptr)
    np.testing.assert_array_equal(val, Ab.data)
    np.testing.assert_array_equal(h.rhs(), bb)
    x_ref = O.solve_reference(A, b)[perm]
    assert np.linalg.norm(x1 - x_ref) / np.linalg.norm(x_ref) <= SOL_TOL
    true1 = h.true_residual()
    assert abs(rr - true1) <= 0.05 * true1 + 5e-16, (rr, true1)
    # the separate launches: the same x to its rounding (same formulas; the compiler forms
    # other FMAs in the fused kernel, ~1 ulp on a few percent of the entries)
    monkeypatch.setenv("NXHIP_DIR_FUSED", "0")
    asm.assemble()
    it0, rr0, conv0 = h.solve(1e-12, 100, 4)
    assert h.direct_path() == "launches" and conv0 and it0 == 1
    x0 = h.solution()
    assert np.linalg.norm(x0 - x1) <= 1e-14 * np.linalg.norm(x1)
    assert abs(rr0 - rr) <= 0.05 * rr0 + 5e-16, (rr0, rr)
    asm.close()


@pytest.mark.parametrize("case", ["Y_N4", "depth6_N40", "arterial5_N40", "tree6_2d_N70",
                                  "tree5_3d_N31", "linear_alt_N3"])
def test_dstep_superposition_modes(case, monkeypatch):
    """Phase 2 by superposition (NXHIP_DIR_SUP): every slot's
    particular value and response and the chains' u-independent part are formed before the
    top values arrive (1: the top solver reloads and re-assembles its lanes after the top
    part; 5: it rebuilds them from their LDS copies), or not at all (0: phase 2 after the
    values). The three
    agree to rounding (the same solution, other orders of addition: |x_p| + |H u| ~ |x| on
    these graphs, so 1e-14 relative), each matches the oracle's direct solve, reports the
    residual of the x it stored, and repeats bit for bit."""
    mesh, asm, P, A, b = _setup(case)
    h = asm.handle
    Ab, bb, perm, _ = O.to_build_layout(P, A, b)
    x_ref = O.solve_reference(A, b)[perm]
    xs = {}
    for mode in ("0", "1", "5"):
        monkeypatch.setenv("NXHIP_DIR_SUP", mode)
        asm.assemble()
        it, rr, conv = h.solve(1e-12, 100, 4)
        assert h.direct_path() == "fused" and conv and it == 1, (mode, it, rr)
        x = h.solution()
        assert np.linalg.norm(x - x_ref) / np.linalg.norm(x_ref) <= SOL_TOL
        true = h.true_residual()
        assert abs(rr - true) <= 0.05 * true + 5e-16, (mode, rr, true)
        for _ in range(3):
            asm.assemble()
            it2, rr2, _ = h.solve(1e-12, 100, 4)
            assert rr2 == rr
            np.testing.assert_array_equal(h.solution(), x)
        np.testing.assert_array_equal(h.csr()[2], Ab.data)
        np.testing.assert_array_equal(h.rhs(), bb)
        xs[mode] = x
    np.testing.assert_array_equal(xs["1"], xs["5"])  # (the same lane values either way)
    assert np.linalg.norm(xs["1"] - xs["0"]) <= 1e-14 * np.linalg.norm(xs["0"])
    asm.close()


def test_dstep_lumped_mass_feeds_minres():
    """The lumped flux mass the fused kernel writes (the preconditioner's D block) is the
    assembly kernel's bit for bit: MINRES after a fused step and after the assembly kernel
    runs the same iterations to the same bits."""
    mesh, asm, P, A, b = _setup("arterial5_N40")
    h = asm.handle
    out = []
    for fused in ("1", "0"):
        import os
        os.environ["NXHIP_DIR_FUSED"] = fused
        try:
            asm.set_direct(True)
            asm.assemble()
            h.solve(1e-12, 100, 4)
            assert h.direct_path() == ("fused" if fused == "1" else "launches")
            asm.set_direct(False)  # MINRES on the assembled system, no new assembly
            it, rr, conv = h.solve(1e-12, 100, 4)
            assert conv and it <= 4
            out.append((it, h.solution()))
        finally:
            del os.environ["NXHIP_DIR_FUSED"]
    assert out[0][0] == out[1][0]
    np.testing.assert_array_equal(out[0][1], out[1][1])
    asm.close()


@pytest.mark.parametrize("case", ["depth6_N40", "tree6_2d_N70", "arterial5_N40"])
def test_dstep_refinement_step(case):
    """A residual above rtol after the fused pass: one refinement step (r = b - A x is formed
    first -- the fused kernel does not keep it) brings it under, reported truthfully."""
    mesh, asm, P, A, b = _setup(case)
    h = asm.handle
    asm.assemble()
    it, rr, conv = h.solve(1e-12, 100, 4)
    assert h.direct_path() == "fused"
    if rr <= 4e-15:
        pytest.skip(f"first pass already at {rr:.1e}: no room for a refinement step")
    asm.assemble()
    it2, rr2, conv2 = h.solve(rr / 2, 100, 4)
    assert it2 == 2 and conv2 and rr2 <= rr / 2, (it2, rr2)
    true2 = h.true_residual()
    assert abs(rr2 - true2) <= 0.05 * true2 + 5e-16, (rr2, true2)
    Ab, bb, perm, _ = O.to_build_layout(P, A, b)
    x_ref = O.solve_reference(A, b)[perm]
    assert np.linalg.norm(h.solution() - x_ref) / np.linalg.norm(x_ref) <= SOL_TOL
    asm.close()


def test_dstep_repeated_launches_and_new_coefficients():
    """Many launches in a row (the hand-off counters keep counting across launches) give the
    same bits; new coefficients (per-edge R and f) are assembled by the next launch."""
    mesh, asm, P, A, b = _setup("arterial5_N40")
    h = asm.handle
    asm.assemble()
    h.solve(1e-12, 100, 4)
    x1 = h.solution()
    for _ in range(40):
        asm.assemble()
        it, rr, conv = h.solve(1e-12, 100, 4)
        assert conv and h.direct_path() == "fused"
    np.testing.assert_array_equal(h.solution(), x1)
    R = 1.0 / mesh.edge_radius ** 4
    f = 0.1 + 0.02 * (np.arange(mesh.num_edges) % 5)
    asm.compute_forms(p_bc_ex=CASES["arterial5_N40"][3], f=f, R=R)
    asm.assemble()
    it, rr, conv = h.solve(1e-12, 100, 4)
    assert conv and h.direct_path() == "fused"
    A2, b2 = O.assemble_reference(P, CASES["arterial5_N40"][3], f=f, R=R)
    Ab2, bb2, perm, _ = O.to_build_layout(P, A2, b2)
    np.testing.assert_array_equal(h.csr()[2], Ab2.data)
    np.testing.assert_array_equal(h.rhs(), bb2)
    x_ref = O.solve_reference(A2, b2)[perm]
    assert np.linalg.norm(h.solution() - x_ref) / np.linalg.norm(x_ref) <= SOL_TOL
    asm.close()


@pytest.mark.parametrize("case", ["depth6_N40", "arterial5_N40"])
def test_dstep_give_up_falls_back_to_launches(case, monkeypatch):
    """The co-residency fallback: when the waiting workgroups give up
    (forced here with a wait bound of 0 polls), the launch publishes nothing; the host resets
    the hand-off counters and its published-state count, and the same solve runs the
    separate launches -- x bit-equal to NXHIP_DIR_FUSED=0 on the same matrix -- and keeps
    doing so, correctly, for the following steps."""
    mesh, asm, P, A, b = _setup(case)
    h = asm.handle
    Ab, bb, perm, _ = O.to_build_layout(P, A, b)
    x_ref = O.solve_reference(A, b)[perm]
    # the separate launches' answer on this matrix (the reference bits of the fallback)
    monkeypatch.setenv("NXHIP_DIR_FUSED", "0")
    asm.assemble()
    it0, rr0, conv0 = h.solve(1e-12, 100, 4)
    assert h.direct_path() == "launches" and conv0
    x_launch = h.solution()
    monkeypatch.delenv("NXHIP_DIR_FUSED")
    asm.assemble()
    h.solve(1e-12, 100, 4)
    assert h.direct_path() == "fused"
    # every waiting workgroup gives up at once: the step must still return the answer
    h.set_wait_polls(0)
    asm.assemble()
    it, rr, conv = h.solve(1e-12, 100, 4)
    assert h.direct_path() == "launches" and conv and it == 1 and rr == rr0
    np.testing.assert_array_equal(h.solution(), x_launch)
    h.set_wait_polls(1 << 20)
    for _ in range(10):  # the fallback is sticky and its published states stay in step
        asm.assemble()
        it, rr, conv = h.solve(1e-12, 100, 4)
        assert h.direct_path() == "launches" and conv and it == 1 and rr == rr0
        np.testing.assert_array_equal(h.solution(), x_launch)
    assert np.linalg.norm(x_launch - x_ref) / np.linalg.norm(x_ref) <= SOL_TOL
    np.testing.assert_array_equal(h.csr()[2], Ab.data)
    asm.close()


def test_dstep_c3_analytic():
    """C3 (make_tree(15), N = 15, 1,032,160 DoF, 256 jobs = one per CU): the fused step
    runs, the analytic answer to 1e-10, the CSR has the closed-form nnz and is symmetric."""
    mesh = NetworkMesh(ng.make_tree(15, 15, 15), N=15, color_strategy="smallest_last")
    asm = HydraulicNetworkAssembler(mesh)
    asm.compute_forms(p_bc_ex=lambda x: x[1])
    asm.set_direct(True)
    h = asm.handle
    asm.assemble()
    it, rr, conv = h.solve(1e-12, 100, 4)
    assert h.direct_path() == "fused" and conv and it == 1 and rr <= 1e-12
    src, dst = mesh.edges
    P = O.build_problem(mesh.node_coordinates, src, dst, 15)
    xa = O.resistor_network_solution(P, lambda x: x[1])[O.build_permutation(P)[0]]
    x = h.solution()
    assert np.linalg.norm(x - xa) / np.linalg.norm(xa) <= SOL_TOL
    assert h.true_residual() <= 1e-12
    # the hand-offs between the 256 workgroups (write-through stores + one agent-scope
    # counter, no release fence: DESIGN.md section 3c) give the same bits on every launch
    for _ in range(30):
        asm.assemble()
        it2, rr2, conv2 = h.solve(1e-12, 100, 4)
        assert h.direct_path() == "fused" and rr2 == rr
        np.testing.assert_array_equal(h.solution(), x)
    rp, col, val = h.csr()
    E, B = mesh.num_edges, len(mesh.bifurcation_values)
    assert rp[-1] == E * (7 * 15 + 1) + 6 * B
    import scipy.sparse as sp
    Ad = sp.csr_matrix((val, col, rp), shape=(h.n_rows, h.n_rows))
    assert abs(Ad - Ad.T).max() == 0.0
    asm.close()


def test_dstep_several_chain_passes_fresh_handle():
    """make_tree(16), N = 4: 65,535 edges over <= 256 jobs, so a job holds ~256 chains, more
    than one pass of its workgroup (1024 / 8 lanes = 128): phase 2 re-reads the chains' b and
    lumped mass, which the step then writes itself (dstep_multi) -- on a fresh handle no
    earlier assembly has left a lumped mass behind. The analytic answer to 1e-10."""
    mesh = NetworkMesh(ng.make_tree(16, 15, 15), N=4, color_strategy="smallest_last")
    asm = HydraulicNetworkAssembler(mesh)
    asm.compute_forms(p_bc_ex=lambda x: x[1])
    asm.set_direct(True)
    h = asm.handle
    assert int(np.diff(asm._pc.job_chain_off).max()) > 128
    asm.assemble()
    it, rr, conv = h.solve(1e-12, 100, 4)
    assert h.direct_path() == "fused" and conv and it == 1 and rr <= 1e-12
    src, dst = mesh.edges
    P = O.build_problem(mesh.node_coordinates, src, dst, 4)
    xa = O.resistor_network_solution(P, lambda x: x[1])[O.build_permutation(P)[0]]
    assert np.linalg.norm(h.solution() - xa) / np.linalg.norm(xa) <= SOL_TOL
    assert abs(rr - h.true_residual()) <= 0.05 * rr + 5e-16
    # MINRES on the same system after the step: the lumped mass is the assembly kernel's
    asm.set_direct(False)
    it2, rr2, conv2 = h.solve(1e-10, 200, 4)
    assert conv2 and np.linalg.norm(h.solution() - xa) / np.linalg.norm(xa) <= 1e-8
    asm.close()


def _edge_case_graphs():
    import networkx as nx

    one = nx.DiGraph()
    one.add_node(0, pos=np.array([0.0, 0.0, 0.0]))
    one.add_node(1, pos=np.array([0.3, 1.1, 0.0]))
    one.add_edge(0, 1)
    two = nx.DiGraph()  # a forest of two components, one of them a Y
    for i, p in enumerate([[0, 0, 0], [0, 1, 0], [2, 0, 0], [2, 1, 0], [1.5, 2, 0], [2.5, 2, 0]]):
        two.add_node(i, pos=np.array(p, dtype=float))
    two.add_edges_from([(0, 1), (2, 3), (3, 4), (3, 5)])
    return {"one_edge": one, "forest2": two}


@pytest.mark.parametrize("name", ["one_edge", "forest2"])
@pytest.mark.parametrize("N", [1, 7])
@pytest.mark.parametrize("direct", [True, False])
def test_small_graph_edge_cases(name, N, direct):
    """Edge cases of the job decomposition: a single edge (one job, no junction, no top
    part) and a forest of two components, N = 1 and 7, through the fused direct step and
    MINRES: the oracle's direct solve to 1e-10, the CSR bit-exact."""
    G = _edge_case_graphs()[name]
    mesh = NetworkMesh(G, N=N)
    asm = HydraulicNetworkAssembler(mesh)
    pbc = lambda x: x[1]  # noqa: E731
    asm.compute_forms(p_bc_ex=pbc)
    asm.set_direct(direct)
    h = asm.handle
    asm.assemble()
    it, rr, conv = h.solve(1e-12, 1000, 4)
    assert conv
    src, dst = mesh.edges
    P = O.build_problem(mesh.node_coordinates, src, dst, N, mesh.edge_colors)
    A, b = O.assemble_reference(P, pbc)
    Ab, bb, perm, _ = O.to_build_layout(P, A, b)
    np.testing.assert_array_equal(h.csr()[2], Ab.data)
    x_ref = O.solve_reference(A, b)[perm]
    assert np.linalg.norm(h.solution() - x_ref) / np.linalg.norm(x_ref) <= SOL_TOL
    asm.close()
