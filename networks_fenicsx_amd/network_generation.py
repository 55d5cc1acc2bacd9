"""Host-side generators for the synthetic input graphs.

Restates the two generators of the reference
(``src/networks_fenicsx/network_generation.py``):

* :func:`make_tree` -- the symmetric binary tree (reference ``:41-100``), with the
  breadth-first edge order of ``tree_edges`` (``:18-38``) written in closed form:
  edge 0 is ``(0, 1)`` and every later node ``c`` hangs below node ``c // 2``.
* :func:`make_arterial_tree` -- the Murray's-law arterial tree (``:157-283``).

Both return a :class:`networkx.DiGraph` whose nodes carry ``"pos"`` and (arterial)
whose edges carry ``"radius"``, like the reference. Floating-point operations are
performed in the same order as the reference so that node coordinates are
bit-identical; this is pinned by ``tests/golden/graphs.npz`` (generated from the
reference module itself by ``tests/golden/make_golden.py``).
Generation is setup work and stays on the host.
"""

from __future__ import annotations

from typing import Callable

import networkx as nx
import numpy as np
import numpy.typing as npt

from .timing import timed

__all__ = ["make_tree", "make_arterial_tree", "tree_arrays"]


def tree_arrays(n: int, H: float, W: float, dim: int = 3):
    """Array form of :func:`make_tree`: ``(pos[n_nodes, dim], src[E], dst[E])``.

    This is what the device path consumes; :func:`make_tree` wraps it into a
    ``networkx.DiGraph``. Node ``c >= 2`` is a child of ``c // 2``; nodes of each
    generation are sorted by x (reference ``network_generation.py:77-95``).
    """
    assert n >= 1, "Number of generations must be at least 1"
    per_gen = [2**g for g in range(n)]
    n_nodes = 1 + sum(per_gen)
    n_last = 2 ** (n - 1)
    # Same expressions as the reference; n == 1 divides by zero there too.
    x_off = W / (2 * (n_last - 1))
    y_off = H / n

    xs = np.zeros(n_nodes, dtype=np.float64)
    ys = np.zeros(n_nodes, dtype=np.float64)
    ys[1] = y_off
    start = 2
    for gen in range(1, n):
        factor = 2 ** (n - gen)
        half = per_gen[gen] // 2
        step = x_off * factor
        # sequential accumulation x_{i+1} = x_i + step, as the reference's loop does
        seed = np.empty(half, dtype=np.float64)
        seed[0] = x_off * (factor / 2)
        seed[1:] = step
        right = np.cumsum(seed)
        row = np.sort(np.concatenate([right, -right]))
        xs[start : start + 2 * half] = row
        ys[start : start + 2 * half] = y_off * (gen + 1)
        start += 2 * half

    pos = np.zeros((n_nodes, dim), dtype=np.float64)
    pos[:, 0] = xs
    pos[:, 1] = ys
    dst = np.arange(1, n_nodes, dtype=np.int64)
    src = dst // 2
    src[0] = 0
    return pos, src, dst


@timed("nxfx:make_tree")
def make_tree(n: int, H: float, W: float, dim: int = 3) -> nx.DiGraph:
    """Symmetric binary tree with ``n`` generations, root edge ``(0, 1)`` at the origin.

    Args:
        n: number of generations of branches (``2**n - 1`` edges)
        H: height of the tree
        W: width of the tree at its largest extent
        dim: geometric dimension (2 or 3)
    """
    pos, src, dst = tree_arrays(n, H, W, dim)
    G = nx.DiGraph()
    G.add_nodes_from(range(pos.shape[0]))
    for i in range(pos.shape[0]):
        G.nodes[i]["pos"] = [float(c) for c in pos[i]]
    G.add_edges_from(zip(src.tolist(), dst.tolist()))
    return G


# --- arterial tree ---------------------------------------------------------------


def _default_normal(x: npt.NDArray[np.floating]) -> npt.NDArray[np.floating]:
    """Unit normal of the xy-plane (reference ``network_generation.py:103-107``)."""
    nrm = np.zeros_like(x)
    nrm[2] = 1
    return nrm


def _advance(p0, direction, length):
    """``p0 + length * direction / |direction|`` (reference ``:148-154``)."""
    assert len(p0) == len(direction)
    return p0 + length * direction / np.linalg.norm(direction, axis=-1)


def _daughter_endpoint(parent: np.ndarray, normal, angle_deg: float, length: float):
    """End point of a daughter vessel (reference ``:110-145``).

    The parent direction is projected onto the plane with normal ``normal`` and
    rotated about that normal by ``angle_deg`` (Rodrigues' formula).
    """
    tail, head = parent[0], parent[1]
    d = head - tail
    # projection onto the plane
    s = np.dot(d, normal) / np.linalg.norm(normal)
    d_plane = d - s * normal / np.linalg.norm(normal)
    # Rodrigues rotation about the (normalised) plane normal
    theta = np.radians(angle_deg)
    k = normal / np.linalg.norm(normal)
    K = np.array([[0, -k[2], k[1]], [k[2], 0, -k[0]], [-k[1], k[0], 0]])
    Rot = np.eye(3) + np.sin(theta) * K + (1 - np.cos(theta)) * np.dot(K, K)
    return _advance(head, np.dot(Rot, d_plane), length)


@timed("nxfx:make_arterial_tree")
def make_arterial_tree(
    N: int,
    p0: npt.NDArray[np.floating] = np.zeros(3, dtype=np.float64),
    direction: npt.NDArray[np.floating] = np.array([0, 1, 0], dtype=np.float64),
    D0: float = 2.0,
    lmbda: float = 8.0,
    gamma: float = 0.8,
    normal: Callable[[npt.NDArray[np.floating]], npt.NDArray[np.floating]] = _default_normal,
    random: bool = False,
) -> nx.DiGraph:
    """Arterial tree following Murray's law (``D0^3 = D1^3 + D2^3``, ``D1 = gamma D2``).

    Vessel length is ``lmbda * diameter``; bifurcation angles follow the
    minimum-energy relation. ``random=True`` draws the left/right choice from
    ``np.random`` exactly once per parent vessel, as the reference does.

    Raises:
        ValueError: if ``gamma > 1``.
    """
    if gamma > 1:
        raise ValueError("Please choose a gamma lower or equal to 1")

    G = nx.DiGraph()
    G.add_edge(0, 1)
    nx.set_node_attributes(G, p0, "pos")
    nx.set_edge_attributes(G, D0 / 2, "radius")
    G.nodes[1]["pos"] = _advance(p0, direction, D0 * lmbda)

    last = 1
    frontier = [(0, 1)]
    parent = np.empty((2, 3), dtype=p0.dtype)
    for _generation in range(1, N):
        nxt = []
        for e in frontier:
            parent[0, :] = G.nodes[e[0]]["pos"]
            parent[1, :] = G.nodes[e[1]]["pos"]
            Dp = G.edges[e]["radius"] * 2
            D2 = Dp * (gamma**3 + 1) ** (-1 / 3)
            D1 = gamma * D2
            L1, L2 = lmbda * D1, lmbda * D2
            c1 = (Dp**4 + D1**4 - (Dp**3 - D1**3) ** (4 / 3)) / (2 * Dp**2 * D1**2)
            c2 = (Dp**4 + D2**4 - (Dp**3 - D2**3) ** (4 / 3)) / (2 * Dp**2 * D2**2)
            a1 = np.degrees(np.arccos(c1))
            a2 = np.degrees(np.arccos(c2))
            s1 = 1 if not random else np.random.choice([-1, 1])
            for sign, ang, length, diam in ((s1, a1, L1, D1), (-s1, a2, L2, D2)):
                last += 1
                edge = (e[1], last)
                G.add_edge(*edge)
                G.nodes[last]["pos"] = _daughter_endpoint(
                    parent, normal(parent[1]), sign * ang, length
                )
                G.edges[edge]["radius"] = diam / 2
                nxt.append(edge)
        frontier = nxt
    return G
