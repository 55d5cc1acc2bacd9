"""Shared test configurations (graphs + the oracle's view of them)."""

from __future__ import annotations

import networkx as nx
import numpy as np

from networks_fenicsx_amd import network_generation as ng


def p_y(x):
    return x[1]


def p_x(x):
    return x[0]


def edge_info_graph() -> nx.DiGraph:
    """The hand-built 8-node graph of the reference's tests/test_edge_info.py:8-35
    (pass-through nodes, a 3-way split and a cycle)."""
    G = nx.DiGraph()
    G.add_node(0, pos=np.zeros(3))
    G.add_node(1, pos=np.array([0.0, 0.0, 1.0]))
    G.add_node(2, pos=np.array([0.2, 0.2, 2.0]))
    G.add_node(3, pos=np.array([-0.2, 0.3, 2.0]))
    G.add_node(4, pos=np.array([0.0, 0.1, 2.1]))
    G.add_node(5, pos=np.array([0.1, -0.1, 3.0]))
    G.add_node(6, pos=np.array([-0.3, 0.4, 4.0]))
    G.add_node(7, pos=1.1 * G.nodes[1]["pos"])
    for e in [(0, 1), (1, 7), (7, 2), (2, 5), (7, 3), (3, 4), (4, 5), (7, 4), (5, 6)]:
        G.add_edge(*e)
    return G


def linear_graph(n: int, dim: int = 2, ordered=lambda _: True) -> nx.DiGraph:
    """Reference tests/test_orientation.py:10-25."""
    G = nx.DiGraph()
    G.add_nodes_from(range(n))
    for i in range(n - 1):
        if ordered(i):
            G.add_edge(i, i + 1)
        else:
            G.add_edge(i + 1, i)
    for i in range(n):
        pos = np.zeros(dim)
        pos[0] = i / (n - 1)
        G.nodes[i]["pos"] = pos
    return G


def lattice_graph(nx_: int, ny: int):
    """An nx_ x ny grid of pipes (many cycles: (nx_-1)(ny-1) of them), inlet/outlet at two
    corners through extra boundary edges -- an anastomosed network's worst case."""
    import networkx as nx

    G = nx.DiGraph()
    idx = lambda i, j: i * ny + j  # noqa: E731
    for i in range(nx_):
        for j in range(ny):
            G.add_node(idx(i, j), pos=np.array([float(i), float(j) + 0.1 * i, 0.0]))
    n = nx_ * ny
    G.add_node(n, pos=np.array([-1.0, 0.0, 0.0]))
    G.add_node(n + 1, pos=np.array([float(nx_), float(ny - 1) + 0.1 * (nx_ - 1), 0.0]))
    G.add_edge(n, idx(0, 0))
    for i in range(nx_):
        for j in range(ny):
            if i + 1 < nx_:
                G.add_edge(idx(i, j), idx(i + 1, j))
            if j + 1 < ny:
                G.add_edge(idx(i, j), idx(i, j + 1))
    G.add_edge(idx(nx_ - 1, ny - 1), n + 1)
    return G


# name -> (graph factory, N, colour strategy, p_bc)
CASES = {
    "Y_N4": (lambda: ng.make_tree(2, 1, 3), 4, None, p_y),
    "demo_tree_N2": (lambda: ng.make_tree(2, 1, 1), 2, None, p_y),
    "demo_tree_N1": (lambda: ng.make_tree(2, 1, 1), 1, None, p_y),
    "demo_tree_N4": (lambda: ng.make_tree(2, 1, 1), 4, None, p_y),
    "double_Y_N5": (lambda: ng.make_tree(2, 3.1, 7.3), 5, None, p_x),
    "depth6_N40": (lambda: ng.make_tree(7, 7, 7), 40, "smallest_last", p_y),
    "arterial5_N40": (lambda: ng.make_arterial_tree(5, direction=np.array([0.1, 1, 0])), 40,
                      nx.coloring.strategy_largest_first, p_y),
    "edge_info_N10": (edge_info_graph, 10, None, p_y),
    "tree6_2d_N70": (lambda: ng.make_tree(6, 2, 1, dim=2), 70, "smallest_last", p_y),
    "linear_alt_N3": (lambda: linear_graph(12, ordered=lambda k: k % 2), 3, None, p_x),
    # assembly layouts: 4 edges per wave (N < 16), 2 (N < 32), and the boundaries
    "tree5_N15": (lambda: ng.make_tree(5, 5, 5), 15, "smallest_last", p_y),
    "tree5_N16": (lambda: ng.make_tree(5, 5, 5), 16, "smallest_last", p_y),
    "tree5_3d_N31": (lambda: ng.make_tree(5, 2, 3), 31, "smallest_last", p_x),
}

# every configuration of tests/golden/systems.npz (tests/golden/make_golden.py)
GOLDEN_CASES = ["Y_N4", "demo_tree_N2", "demo_tree_N4", "double_Y_N5", "depth6_N40",
                "arterial5_N40"]


def graph_arrays(G):
    pos = np.asarray([G.nodes[v]["pos"] for v in G.nodes()], dtype=np.float64)
    edges = np.asarray(list(G.edges()), dtype=np.int64).reshape(-1, 2)
    return pos, edges

# graphs with cycles (the direct solve's Woodbury correction), name -> (factory, N)
CYCLIC = {"edge_info_N10": (edge_info_graph, 10),
          "lattice4x5_N6": (lambda: lattice_graph(4, 5), 6),
          "lattice6x6_N3": (lambda: lattice_graph(6, 6), 3),
          "lattice19x20_N2": (lambda: lattice_graph(19, 20), 2)}  # (342 cycle chains)
