"""The fast edge colouring (networks_fenicsx_amd/coloring.py) against networkx's own call
(reference mesh.py:29-42): identical colours and identical dict order."""

import random

import networkx as nx
import pytest

from networks_fenicsx_amd import network_generation as ng
from networks_fenicsx_amd.coloring import fast_edge_coloring, fast_path_available
from networks_fenicsx_amd.mesh import color_graph


def _nx(G, strategy):
    return nx.coloring.greedy_color(nx.line_graph(G.to_undirected()), strategy=strategy)


STRATS = ["smallest_last", "largest_first", nx.coloring.strategy_largest_first,
          nx.coloring.strategy_smallest_last]


@pytest.mark.parametrize("seed", range(24))
def test_random_graphs(seed):
    rnd = random.Random(seed)
    k = rnd.randint(2, 50)
    G = nx.gnm_random_graph(k, rnd.randint(1, 3 * k), seed=seed, directed=seed % 2 == 0)
    if seed % 3 == 0:  # non-contiguous labels: node order != label order
        G = nx.relabel_nodes(G, {v: (v * 7919) % 1009 for v in G})
    for s in STRATS:
        a, b = fast_edge_coloring(G, s), _nx(G, s)
        assert a == b and list(a) == list(b)


@pytest.mark.parametrize("levels", [2, 5, 9, 12])
def test_trees_and_arterial(levels):
    G = ng.make_tree(levels, levels, levels)
    for s in ("smallest_last", "largest_first"):
        a, b = fast_edge_coloring(G, s), _nx(G, s)
        assert a == b and list(a) == list(b)


def test_color_graph_dispatch():
    G = ng.make_tree(6, 6, 6)
    assert fast_path_available(G, "smallest_last")
    assert not fast_path_available(G, "DSATUR")
    assert not fast_path_available(nx.MultiGraph(G.to_undirected()), "smallest_last")
    want = {(u, v): _nx(G, "DSATUR").get((u, v), _nx(G, "DSATUR").get((v, u))) for u, v in G.edges}
    assert color_graph(G, "DSATUR") == want  # networkx path
    sl = _nx(G, "smallest_last")
    assert color_graph(G, "smallest_last") == {(u, v): sl.get((u, v), sl.get((v, u)))
                                               for u, v in G.edges}
    assert fast_edge_coloring(nx.DiGraph(), "smallest_last") == {}
