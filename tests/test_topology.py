"""Topology layer: the reference's own tests restated as known answers.

* tests/test_make_tree.py:21-24  -> cell / vertex counts
* tests/test_edge_info.py:36-55  -> bifurcations and in/out edge counts
* tests/test_orientation.py:52-58 -> integral of (1,0).tangent over the mesh
"""

import networkx as nx
import numpy as np
import pytest

from cases import edge_info_graph, linear_graph
from networks_fenicsx_amd import NetworkMesh, network_generation
from networks_fenicsx_amd.mesh import color_graph


@pytest.mark.parametrize("gdim", [2, 3])
@pytest.mark.parametrize("N", [1, 4, 10])
@pytest.mark.parametrize("n", [2, 5, 7])
@pytest.mark.parametrize("H", [1, 2])
def test_make_tree(n, H, gdim, N):
    G = network_generation.make_tree(n=n, H=H, W=1, dim=gdim)
    domain = NetworkMesh(G, N=N).mesh
    assert domain.topology.dim == 1
    assert domain.geometry.dim == gdim
    num_segments = sum(2**i for i in range(n))
    assert domain.topology.index_map(1).size_global == N * num_segments
    assert domain.topology.index_map(0).size_global == N + 1 + (num_segments - 1) * N


@pytest.mark.parametrize("N", [10, 50])
def test_edge_info(N):
    network_mesh = NetworkMesh(edge_info_graph(), N=N)
    assert len(network_mesh.bifurcation_values) == 6
    np.testing.assert_allclose([1, 2, 3, 4, 5, 7], network_mesh.bifurcation_values)
    expect = [(1, 1), (1, 1), (1, 1), (2, 1), (2, 1), (1, 3)]
    for i, (n_in, n_out) in enumerate(expect):
        assert len(network_mesh.in_edges(i)) == n_in
        assert len(network_mesh.out_edges(i)) == n_out


@pytest.mark.parametrize("order", ["in", "reverse", "alternating"])
@pytest.mark.parametrize("N", [1, 4, 8])
def test_orientation(order, N):
    n = 30
    ordered = {"in": lambda _: True, "reverse": lambda _: False,
               "alternating": lambda k: k % 2}[order]
    mesh = NetworkMesh(linear_graph(n, ordered=ordered), N=N)
    t = mesh.tangents()
    h = mesh.cell_lengths()
    val = float(np.sum(t[:, 0] * mesh.orientation.x.array * h))
    if order == "in":
        assert np.isclose(val, 1.0)
    elif order == "reverse":
        assert np.isclose(val, -1.0)
    else:
        edge_count = n - 1
        assert np.isclose(val, edge_count % 2 * -1 / edge_count)


def test_markers_and_boundaries():
    G = network_generation.make_tree(3, 1, 1)
    m = NetworkMesh(G, N=2)
    nn = G.number_of_nodes()
    assert m.in_marker == 3 * nn and m.out_marker == 5 * nn
    np.testing.assert_array_equal(m.boundary_out_nodes, [0])
    np.testing.assert_array_equal(m.boundary_in_nodes, [4, 5, 6, 7])
    np.testing.assert_array_equal(m.bifurcation_values, [1, 2, 3])
    tags = m.boundaries
    assert tags.values[tags.indices == 0][0] == m.out_marker
    assert np.all(tags.values[np.isin(tags.indices, [4, 5, 6, 7])] == m.in_marker)


@pytest.mark.parametrize("strategy", [None, "smallest_last", "largest_first",
                                      nx.coloring.strategy_largest_first])
def test_coloring_matches_networkx(strategy):
    G = network_generation.make_tree(6, 1, 1)
    c = color_graph(G, strategy)
    if strategy is None:
        assert c == {e: i for i, e in enumerate(G.edges)}
    else:
        ref = nx.coloring.greedy_color(nx.line_graph(G.to_undirected()), strategy=strategy)
        assert all(c[e] == ref[e] for e in G.edges)
        # proper edge colouring: edges sharing a node differ
        for v in G.nodes:
            cols = [c[e] for e in list(G.in_edges(v)) + list(G.out_edges(v))]
            assert len(cols) == len(set(cols))
    m = NetworkMesh(G, N=3, color_strategy=strategy)
    assert m.num_edge_colors == len(set(c.values()))
    assert sum(s.size for s in m.submeshes) == G.number_of_edges()


def test_geometry_matches_reference_formula():
    G = network_generation.make_arterial_tree(4)
    m = NetworkMesh(G, N=7)
    x = m.mesh.geometry.x
    src, dst = m.edges
    w = np.linspace(0, 1, 7, endpoint=False)[1:]
    e = 3
    start, end = x[src[e]], x[dst[e]]
    inner = start * (1 - w[:, None]) + end * w[:, None]
    first = G.number_of_nodes() + e * 6
    np.testing.assert_array_equal(x[first:first + 6], inner)
    np.testing.assert_array_equal(m.mesh.cells[e * 7], [src[e], first])
    np.testing.assert_array_equal(m.mesh.cells[e * 7 + 6], [first + 5, dst[e]])


def test_timers_registered():
    from networks_fenicsx_amd.timing import timing

    network_generation.make_tree(3, 1, 1)
    NetworkMesh(network_generation.make_tree(3, 1, 1), N=2, color_strategy="smallest_last")
    for name in ("nxfx:make_tree", "nxfx:NetworkMesh:build_mesh", "nxfx:color_graph"):
        count, total = timing(name)
        assert count >= 1 and total.total_seconds() >= 0
