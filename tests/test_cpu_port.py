"""The all-cores CPU port (``oracle/nx_cpu.c``, bench.py's cpu_baseline leg) is pinned
against the oracle before it is used as a baseline: its CSR and rhs are bit-exact against
the oracle's symmetric build-layout system, and its preconditioned MINRES matches the direct
solve (<= 1e-10 rel. 2-norm) in the iteration count of the exact preconditioner (3)."""

from __future__ import annotations

import numpy as np
import pytest

from cases import CASES
from networks_fenicsx_amd import NetworkMesh
from networks_fenicsx_amd import network_generation as ng
from networks_fenicsx_amd.assembly import edge_boundary_rhs, evaluate_nodal
from networks_fenicsx_amd.layout import build_local_problem
from networks_fenicsx_amd.precond import build_tree_preconditioner
from oracle import nx_cpu
from oracle import nx_oracle as O


def _setup(G, N, strategy, pbc):
    m = NetworkMesh(G, N=N, color_strategy=strategy)
    src, dst = m.edges
    lp = build_local_problem(m.node_coordinates, src, dst, m.degrees, N)
    pc = build_tree_preconditioner(lp, src, dst, m.degrees)
    bc = edge_boundary_rhs(m, lp.edges, evaluate_nodal(pbc, m.node_coordinates))
    return m, lp, pc, nx_cpu.CpuStep(lp, pc, bc)


@pytest.mark.parametrize("case", ["Y_N4", "depth6_N40", "arterial5_N40", "tree5_N15",
                                  "edge_info_N10", "linear_alt_N3", "tree6_2d_N70"])
def test_cpu_port_matches_oracle(case):
    make, N, strategy, pbc = CASES[case]
    m, lp, pc, st = _setup(make(), N, strategy, pbc)
    src, dst = m.edges
    P = O.build_problem(m.node_coordinates, src, dst, N, m.edge_colors)
    A, b = O.assemble_reference(P, pbc)
    Ab, bb, perm, _ = O.to_build_layout(P, A, b)
    np.testing.assert_array_equal(st.rowptr, Ab.indptr)
    np.testing.assert_array_equal(st.col, Ab.indices)
    np.testing.assert_array_equal(st.val, Ab.data)
    np.testing.assert_array_equal(st.rhs, bb)
    it, rr = st.solve(1e-12)
    x_ref = O.solve_reference(A, b)[perm]
    err = np.linalg.norm(st.x - x_ref) / np.linalg.norm(x_ref)
    assert err <= 1e-10, err
    if m.num_edges == m.num_nodes - 1:  # trees: exact Schur-complement preconditioner
        assert it <= 4, it


def test_cpu_port_medium_tree_analytic():
    """make_tree(12) (depth 11, N=15, ~130k DoF): 3 iterations, analytic answer."""
    G = ng.make_tree(12, 12, 12)
    m, lp, pc, st = _setup(G, 15, "smallest_last", lambda x: x[1])
    st.assemble()
    it, rr = st.solve(1e-12)
    src, dst = m.edges
    P = O.build_problem(m.node_coordinates, src, dst, 15)
    xa = O.resistor_network_solution(P, lambda x: x[1])[O.build_permutation(P)[0]]
    assert it == 3
    assert np.linalg.norm(st.x - xa) / np.linalg.norm(xa) < 1e-10


@pytest.mark.parametrize("case", ["Y_N4", "depth6_N40", "arterial5_N40", "tree5_N15",
                                  "linear_alt_N3", "tree6_2d_N70", "demo_tree_N1"])
def test_cpu_direct_matches_oracle(case):
    """The host port of the GPU's direct tree solve (nxc_direct): the oracle's direct
    solution to 1e-10, true residual <= 1e-12 after at most one refinement step."""
    make, N, strategy, pbc = CASES[case]
    m, lp, pc, st = _setup(make(), N, strategy, pbc)
    assert pc.tree_exact
    src, dst = m.edges
    P = O.build_problem(m.node_coordinates, src, dst, N, m.edge_colors)
    A, b = O.assemble_reference(P, pbc)
    _, _, perm, _ = O.to_build_layout(P, A, b)
    passes, rr = st.solve_direct(1e-12)
    assert passes in (1, 2) and rr <= 1e-12, (passes, rr)
    x_ref = O.solve_reference(A, b)[perm]
    assert np.linalg.norm(st.x - x_ref) / np.linalg.norm(x_ref) <= 1e-10


def test_cpu_direct_medium_tree_analytic():
    G = ng.make_tree(12, 12, 12)
    m, lp, pc, st = _setup(G, 15, "smallest_last", lambda x: x[1])
    st.assemble()
    passes, rr = st.solve_direct(1e-12)
    src, dst = m.edges
    P = O.build_problem(m.node_coordinates, src, dst, 15)
    xa = O.resistor_network_solution(P, lambda x: x[1])[O.build_permutation(P)[0]]
    assert passes in (1, 2) and rr <= 1e-12
    assert np.linalg.norm(st.x - xa) / np.linalg.norm(xa) < 1e-10
