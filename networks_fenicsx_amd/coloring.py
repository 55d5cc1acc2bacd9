"""Fast, result-identical edge colouring for ``NetworkMesh`` (host setup).

The reference colours the edges with ``nx.coloring.greedy_color(nx.line_graph(
graph.to_undirected()), strategy)`` (``src/networks_fenicsx/mesh.py:29-42``). On a
depth-18 tree (524 k edges) that call takes ~27 s, most of it in networkx's graph
classes: ``to_undirected`` deep-copies every attribute dict, ``line_graph`` and
``strategy_smallest_last``'s ``G.copy()`` go through ``add_edges_from`` one edge at a
time, and the bucket queue calls ``H.degree(v)`` through a view per neighbour.

This module replays the *same sequence of dict and set operations* on plain
dict-of-dicts, so every container ends in the same state as networkx's and the colouring
is identical, including the ties that ``set.pop()`` breaks (``strategy_smallest_last``
pops from per-degree sets; a set's pop order depends only on the hashes and on the
history of inserts and removals, which is replayed exactly). The algorithms restated:

* ``Graph.to_undirected`` (networkx 3.4 ``classes/digraph.py`` ``to_undirected``):
  nodes in node order, then ``add_edges_from`` over ``(u, v)`` for ``u`` in node order,
  ``v`` in successor order;
* ``_lg_undirected`` (``generators/line.py``): line-graph nodes are the end-node pairs
  sorted by node index; a clique per node is added to a Python ``set`` of canonical
  pairs, isolated nodes first, then ``add_edges_from(set)``;
* ``Graph.copy`` (node order, then ``add_edges_from`` over the adjacency), used by
  ``strategy_smallest_last``; ``strategy_largest_first`` is ``sorted(G, key=degree,
  reverse=True)``;
* ``greedy_color``: the first colour not used by an already-coloured neighbour.

Only the strategies ``"largest_first"`` and ``"smallest_last"`` (names or the networkx
functions) on simple (Di)Graphs take this path, and only for the networkx series it
was checked against (``tests/test_coloring.py`` compares it with networkx on random and
tree graphs); everything else calls networkx, as the reference does.
"""

from __future__ import annotations

from collections import defaultdict, deque
from itertools import count

import networkx as nx

__all__ = ["fast_edge_coloring", "fast_path_available"]

_CHECKED_SERIES = ("3.2", "3.3", "3.4", "3.5")


def _series() -> str:
    return ".".join(nx.__version__.split(".")[:2])


def _strategy_name(strategy) -> str | None:
    if strategy in ("largest_first", "smallest_last"):
        return strategy
    if strategy is nx.coloring.strategy_largest_first:
        return "largest_first"
    if strategy is nx.coloring.strategy_smallest_last:
        return "smallest_last"
    return None


def fast_path_available(graph, strategy) -> bool:
    return (_strategy_name(strategy) is not None and _series() in _CHECKED_SERIES
            and not graph.is_multigraph())


def _undirected(graph) -> dict:
    """``to_undirected``: nodes in node order, then ``add_edges_from`` (a dict per node;
    an existing key keeps its place)."""
    adj = {n: {} for n in graph}
    for u, nbrs in graph._adj.items():  # successors for a DiGraph, neighbours for a Graph
        au = adj[u]
        for v in nbrs:
            au[v] = None
            adj[v][u] = None
    return adj


def _line_graph(adj: dict) -> tuple[list, list]:
    """``_lg_undirected`` with integer ids: (line-graph nodes in L's node order, adjacency
    lists in L's adjacency order). Every canonical pair is in the set once, so appending
    reproduces ``add_edges_from``'s dict order."""
    # sorted(..., key=...) of two distinct items is "swap when the key is smaller"; the
    # pair keys are computed once per incident edge instead of inside every comparison
    index = {n: i for i, n in enumerate(adj)}
    nodes: list = []
    ids: dict = {}
    edges = set()
    add = edges.add
    for u, nbrs in adj.items():
        iu = index[u]
        pairs, keys = [], []
        for v in nbrs:
            iv = index[v]
            if iv < iu:
                pairs.append((v, u))
                keys.append((iv, iu))
            else:
                pairs.append((u, v))
                keys.append((iu, iv))
        if len(pairs) == 1 and pairs[0] not in ids:
            ids[pairs[0]] = len(nodes)
            nodes.append(pairs[0])
        m = len(pairs)
        for i in range(m - 1):  # set.update(list) == add() item by item, in order
            a, ka = pairs[i], keys[i]
            for j in range(i + 1, m):
                add((pairs[j], a) if keys[j] < ka else (a, pairs[j]))
    nbr: list = [[] for _ in nodes]
    for a, b in edges:
        ia = ids.get(a)
        if ia is None:
            ia = ids[a] = len(nodes)
            nodes.append(a)
            nbr.append([])
        ib = ids.get(b)
        if ib is None:
            ib = ids[b] = len(nodes)
            nodes.append(b)
            nbr.append([])
        nbr[ia].append(ib)
        nbr[ib].append(ia)
    return nodes, nbr


def _order_smallest_last(nodes: list, nbr: list) -> list:
    """``strategy_smallest_last`` on ``H = G.copy()``. The copy re-inserts the edges node
    by node, so ``H[x]`` lists x's neighbours placed before x (ascending), then the ones
    after x in ``G[x]``'s order; deleting a node keeps the others' order, so iterating
    the live neighbours of that list is iterating ``H[u]``. The per-degree buckets are
    the same sets of the same node objects with the same operations (``pop`` ties)."""
    n = len(nodes)
    H: list = [[] for _ in range(n)]
    for u in range(n):
        for v in nbr[u]:
            if v > u:
                H[u].append(v)
                H[v].append(u)
    deg = [len(h) for h in H]
    alive = [True] * n
    ids = {x: i for i, x in enumerate(nodes)}
    degrees = defaultdict(set)
    lbound = float("inf")
    for i in range(n):
        d = deg[i]
        degrees[d].add(nodes[i])
        if d < lbound:
            lbound = d
    result = []
    for _ in range(n):
        min_degree = next(d for d in count(lbound) if d in degrees)
        bucket = degrees[min_degree]
        x = bucket.pop()
        if not bucket:
            del degrees[min_degree]
        u = ids[x]
        result.append(u)
        alive[u] = False
        for v in H[u]:
            if alive[v]:
                d = deg[v]
                b = degrees[d]
                xv = nodes[v]
                b.remove(xv)
                if not b:
                    del degrees[d]
                degrees[d - 1].add(xv)
                deg[v] = d - 1
        lbound = min_degree - 1
    result.reverse()  # appendleft
    return result


def _order_largest_first(nodes: list, nbr: list) -> list:
    return sorted(range(len(nodes)), key=lambda i: len(nbr[i]), reverse=True)


def fast_edge_coloring(graph, strategy) -> dict:
    """Colour of every line-graph node (``(u, v)`` pair, node-index order), exactly as
    ``nx.coloring.greedy_color(nx.line_graph(graph.to_undirected()), strategy)``."""
    name = _strategy_name(strategy)
    if name is None:
        raise ValueError(f"no fast path for strategy {strategy!r}")
    nodes, nbr = _line_graph(_undirected(graph))
    if not nodes:
        return {}
    order = (_order_smallest_last if name == "smallest_last" else _order_largest_first)(
        nodes, nbr)
    color = [-1] * len(nodes)
    for u in order:
        used = {color[v] for v in nbr[u]}
        c = 0
        while c in used:
            c += 1
        color[u] = c
    return {nodes[u]: color[u] for u in order}
