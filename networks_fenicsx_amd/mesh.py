"""Graph -> 1-D network topology (host side).

Re-designs the reference's ``NetworkMesh`` (``src/networks_fenicsx/mesh.py:45-538``)
without DOLFINx. What the hot path needs from it is *topology*, not a general
finite-element mesh:

* the edge list in ``graph.edges()`` order and the node coordinates
  (``mesh.py:180, 274``);
* the edge colouring (``mesh.py:29-42``), which only decides how the solution is
  grouped into per-colour flux functions on output;
* node degrees -> ``bifurcation_values`` (degree > 1, ascending) and
  ``boundary_values`` (degree == 1) (``mesh.py:182-186``);
* per-bifurcation in/out colour lists (``mesh.py:189-209``);
* boundary nodes split into inlets/outlets with the ``in_marker = 3 * #nodes`` /
  ``out_marker = 5 * #nodes`` tags (``mesh.py:211-225, 402-408``).

The interval mesh itself (``N`` cells per edge, interior points
``x_u (1 - k/N) + x_v (k/N)``, ``mesh.py:269-322``) is kept as a light
:class:`IntervalMesh` built with vectorised numpy for tests and post-processing;
the device kernels regenerate the same points on the fly from the two edge end
points, so the mesh is never shipped to the GPU.

Cells are always stored source -> target, so the orientation field
(``mesh.py:365-400``) is identically +1 and the unit tangent of every cell is the
source -> target direction of its graph edge.
"""

from __future__ import annotations

from typing import Any, Callable, Iterable

import networkx as nx
import numpy as np
import numpy.typing as npt

from .coloring import fast_edge_coloring, fast_path_available
from .comm import Comm, SerialComm, as_comm
from .timing import timed

__all__ = ["NetworkMesh", "color_graph", "IntervalMesh", "AdjacencyList"]


@timed("nxfx:color_graph")
def color_graph(
    graph: nx.DiGraph,
    strategy: str | Callable[[nx.Graph, dict[int, int]], Iterable[int]] | None,
) -> dict[tuple[int, int], int]:
    """Greedy colouring of the line graph (reference ``mesh.py:29-42``).

    ``strategy=None`` gives every edge its own colour (edge index in
    ``graph.edges()`` order). Otherwise the colouring of the reference's networkx call,
    computed by :mod:`.coloring` for ``largest_first`` / ``smallest_last`` (the same
    operations without networkx's graph classes) and by networkx itself otherwise. The line graph of an undirected graph names each edge by its end
    nodes in node order; both spellings of an edge are accepted here.
    """
    if strategy is None:
        return {edge: i for i, edge in enumerate(graph.edges)}
    if fast_path_available(graph, strategy):  # same result, ~4x faster (coloring.py)
        colouring = fast_edge_coloring(graph, strategy)
    else:
        colouring = nx.coloring.greedy_color(nx.line_graph(graph.to_undirected()),
                                             strategy=strategy)
    out: dict[tuple[int, int], int] = {}
    for u, v in graph.edges:
        c = colouring.get((u, v))
        if c is None:
            c = colouring[(v, u)]
        out[(u, v)] = c
    return out


class AdjacencyList:
    """CSR adjacency (stand-in for ``dolfinx.graph.AdjacencyList``)."""

    def __init__(self, array: npt.NDArray[np.int32], offsets: npt.NDArray[np.int32]):
        self.array = np.asarray(array, dtype=np.int32)
        self.offsets = np.asarray(offsets, dtype=np.int32)

    def links(self, i: int) -> npt.NDArray[np.int32]:
        return self.array[self.offsets[i] : self.offsets[i + 1]]

    @property
    def num_nodes(self) -> int:
        return len(self.offsets) - 1


# --- light mesh objects ------------------------------------------------------------


class _IndexMap:
    def __init__(self, size: int):
        self.size_local = size
        self.size_global = size
        self.num_ghosts = 0


class _Topology:
    def __init__(self, dim: int, sizes: dict[int, int], cells: np.ndarray):
        self.dim = dim
        self._sizes = sizes
        self.cells = cells

    def index_map(self, d: int) -> _IndexMap:
        return _IndexMap(self._sizes[d])

    def create_connectivity(self, *_args) -> None:  # DOLFINx API no-op
        return None

    def create_entity_permutations(self) -> None:
        return None


class _Geometry:
    def __init__(self, x: np.ndarray, dim: int):
        self.x = x  # (num_points, 3), padded like DOLFINx
        self.dim = dim
        self.input_global_indices = np.arange(x.shape[0], dtype=np.int64)


class IntervalMesh:
    """Interval mesh of the network: ``N`` cells per graph edge, source -> target."""

    def __init__(self, comm: Comm, x: np.ndarray, cells: np.ndarray, gdim: int, tdim: int = 1,
                 network=None):
        self.comm = comm
        self.network = network  # the NetworkMesh this mesh discretises
        self.geometry = _Geometry(x, gdim)
        n_vertices = int(np.unique(cells).size) if cells.size else 0
        self.topology = _Topology(tdim, {0: n_vertices, tdim: cells.shape[0]}, cells)

    @property
    def cells(self) -> np.ndarray:
        return self.topology.cells

    def cell_lengths(self) -> np.ndarray:
        d = self.geometry.x[self.cells[:, 1]] - self.geometry.x[self.cells[:, 0]]
        return np.sqrt(d[:, 0] * d[:, 0] + d[:, 1] * d[:, 1] + d[:, 2] * d[:, 2])


class MeshTags:
    def __init__(self, dim: int, indices: np.ndarray, values: np.ndarray, name: str = ""):
        self.dim = dim
        self.indices = np.asarray(indices, dtype=np.int32)
        self.values = np.asarray(values, dtype=np.int32)
        self.name = name

    def find(self, value: int) -> np.ndarray:
        return self.indices[self.values == value]


class DG0Function:
    """A cellwise-constant field (``orientation``) with the DOLFINx ``x.array`` shape."""

    class _X:
        def __init__(self, a: np.ndarray):
            self.array = a

        def scatter_forward(self) -> None:
            return None

    def __init__(self, values: np.ndarray, name: str = ""):
        self.x = DG0Function._X(values)
        self.name = name


def interval_points(pos3: np.ndarray, src: np.ndarray, dst: np.ndarray, N: int) -> np.ndarray:
    """Interior points of every edge, exactly as the reference computes them.

    ``start * (1 - w) + end * w`` with ``w = np.linspace(0, 1, N, endpoint=False)[1:]``
    (reference ``mesh.py:275, 290``). Returns ``(E * (N - 1), 3)``.
    """
    w = np.linspace(0, 1, N, endpoint=False)[1:][None, :, None]  # (1, N-1, 1)
    start = pos3[src][:, None, :]
    end = pos3[dst][:, None, :]
    return (start * (1 - w) + end * w).reshape(-1, 3)


class NetworkMesh:
    """Host-side representation of a directed network graph.

    Args:
        graph: the directed networkx graph (nodes labelled ``0..n-1`` with ``"pos"``).
            Only needed on ``graph_rank``.
        N: number of cells per graph edge.
        color_strategy: networkx greedy-colouring strategy for the edges, or ``None``
            (one colour per edge).
        comm: communicator (``None`` = this process alone, or the initialised
            ``torch.distributed`` world).
        graph_rank: rank that holds ``graph``.
    """

    def __init__(
        self,
        graph: nx.DiGraph | None,
        N: int,
        color_strategy: str | Callable | None = None,
        comm: Any = None,
        graph_rank: int = 0,
    ):
        self._comm = as_comm(comm)
        self._N = int(N)
        if self._N < 1:
            raise ValueError("N must be >= 1")
        self._msh: IntervalMesh | None = None
        self._orientation: DG0Function | None = None
        self._subdomains: MeshTags | None = None
        self._facet_markers: MeshTags | None = None
        self._edge_meshes: list | None = None
        self._lm_mesh: Any = None
        self._build_mesh(graph, color_strategy, graph_rank)

    # ------------------------------------------------------------------ build
    @timed("nxfx:NetworkMesh:build_mesh")
    def _build_mesh(self, graph, color_strategy, graph_rank: int) -> None:
        comm = self._comm
        payload = None
        if comm.rank == graph_rank:
            assert isinstance(graph, nx.DiGraph), f"Directional graph not present on {graph_rank}"
            payload = self._analyse(graph, color_strategy)
        payload = comm.bcast(payload, root=graph_rank)
        (
            self._geom_dim,
            self._pos,
            self._src,
            self._dst,
            self._edge_color,
            self._num_edge_colors,
            self._degree,
            self._edge_radius,
            in_pairs,
            out_pairs,
        ) = payload

        n_nodes = self._pos.shape[0]
        deg = self._degree
        self._bifurcation_values = np.flatnonzero(deg > 1).astype(np.int32)
        self._boundary_values = np.flatnonzero(deg == 1).astype(np.int32)
        # inlets/outlets (reference mesh.py:211-225): a degree-1 node with an
        # in-edge is an outlet leaf (in_marker), with an out-edge a root (out_marker)
        indeg = np.bincount(self._dst, minlength=n_nodes)
        bnd = self._boundary_values
        self._boundary_in_nodes = bnd[indeg[bnd] == 1].astype(np.int32)
        self._boundary_out_nodes = bnd[indeg[bnd] == 0].astype(np.int32)
        self._in_marker = 3 * n_nodes
        self._out_marker = 5 * n_nodes

        # bifurcation index of every node (-1 if not a bifurcation)
        self._bif_index = np.full(n_nodes, -1, dtype=np.int64)
        self._bif_index[self._bifurcation_values] = np.arange(
            self._bifurcation_values.size, dtype=np.int64
        )
        self._bifurcation_in_color = self._pairs_to_adjacency(in_pairs)
        self._bifurcation_out_color = self._pairs_to_adjacency(out_pairs)

    def _pairs_to_adjacency(self, pairs: tuple[np.ndarray, np.ndarray]) -> AdjacencyList:
        """(node, colour) pairs in networkx adjacency order -> CSR over bifurcations."""
        nodes, colours = pairs
        bi = self._bif_index[nodes]
        keep = bi >= 0
        bi, colours = bi[keep], colours[keep]
        order = np.argsort(bi, kind="stable")  # keep networkx order inside a node
        counts = np.bincount(bi, minlength=self._bifurcation_values.size)
        offsets = np.zeros(counts.size + 1, dtype=np.int32)
        np.cumsum(counts, out=offsets[1:])
        return AdjacencyList(colours[order].astype(np.int32), offsets)

    @staticmethod
    def _analyse(graph: nx.DiGraph, color_strategy):
        """Graph -> plain arrays (runs on ``graph_rank`` only)."""
        gdim = len(graph.nodes[1]["pos"])
        coloring = color_graph(graph, color_strategy)
        n_colors = len(set(coloring.values()))
        n_nodes = graph.number_of_nodes()
        edges = np.asarray(list(graph.edges()), dtype=np.int64).reshape(-1, 2)
        src, dst = edges[:, 0].copy(), edges[:, 1].copy()
        pos = np.asarray([graph.nodes[v]["pos"] for v in graph.nodes()], dtype=np.float64)
        deg = np.full(n_nodes, -1, dtype=np.int32)
        for node, d in graph.degree():
            deg[node] = d
        ecol = np.fromiter((coloring[(u, v)] for u, v in zip(src.tolist(), dst.tolist())),
                           dtype=np.int32, count=src.size)
        radius = None
        if src.size and all("radius" in graph.edges[e] for e in graph.edges):
            radius = np.fromiter((graph.edges[e]["radius"] for e in graph.edges),
                                 dtype=np.float64, count=src.size)
        # in/out colours per node in networkx adjacency order (reference mesh.py:193-209)
        in_nodes, in_cols, out_nodes, out_cols = [], [], [], []
        for v, preds in graph.pred.items():
            for u in preds:
                in_nodes.append(v)
                in_cols.append(coloring[(u, v)])
        for u, succs in graph.succ.items():
            for v in succs:
                out_nodes.append(u)
                out_cols.append(coloring[(u, v)])
        in_pairs = (np.asarray(in_nodes, dtype=np.int64), np.asarray(in_cols, dtype=np.int32))
        out_pairs = (np.asarray(out_nodes, dtype=np.int64), np.asarray(out_cols, dtype=np.int32))
        return gdim, pos, src, dst, ecol, n_colors, deg, radius, in_pairs, out_pairs

    def with_comm(self, comm: Any) -> "NetworkMesh":
        """The same network seen through another communicator (shares the graph arrays).

        Every rank holds the whole graph after the broadcast, so e.g. ``with_comm(None)``
        on rank 0 gives the single-process problem of a partitioned run (``bench.py``'s
        same-workload one-GPU time) without analysing the graph again."""
        import copy

        m = copy.copy(self)
        m._comm = as_comm(comm) if comm is not None else SerialComm()
        m._msh = None
        return m

    # -------------------------------------------------------------- geometry
    @property
    def mesh(self) -> IntervalMesh:
        """The interval mesh (built lazily; not needed by the device path)."""
        if self._msh is None:
            self._msh = self._build_interval_mesh()
        return self._msh

    def _build_interval_mesh(self) -> IntervalMesh:
        N, E = self._N, self._src.size
        n_nodes = self._pos.shape[0]
        pos3 = np.zeros((n_nodes, 3), dtype=np.float64)
        pos3[:, : self._geom_dim] = self._pos
        if N == 1:
            x = pos3
            cells = np.stack([self._src, self._dst], axis=1).astype(np.int64)
        else:
            x = np.vstack([pos3, interval_points(pos3, self._src, self._dst, N)])
            first = n_nodes + np.arange(E, dtype=np.int64) * (N - 1)
            idx = np.empty((E, N + 1), dtype=np.int64)
            idx[:, 0] = self._src
            idx[:, 1:N] = first[:, None] + np.arange(N - 1, dtype=np.int64)[None, :]
            idx[:, N] = self._dst
            cells = np.stack([idx[:, :-1], idx[:, 1:]], axis=2).reshape(-1, 2)
        return IntervalMesh(self._comm, x, cells, self._geom_dim, network=self)

    def cell_lengths(self) -> np.ndarray:
        """Length of every cell, edge-major (``E * N``)."""
        return self.mesh.cell_lengths()

    def local_edges(self) -> np.ndarray:
        """Graph edges owned by this rank (the assembler's partition, ``layout.py``)."""
        from .layout import partition_edges

        if self._comm.size == 1:
            return np.arange(self._src.size, dtype=np.int64)
        owner = partition_edges(self._src, self._dst, self._pos.shape[0], self._comm.size)
        return np.flatnonzero(owner == self._comm.rank)

    def tangents(self) -> np.ndarray:
        """Unit tangent of every cell (``E * N x 3``), source -> target of its edge."""
        m = self.mesh
        d = m.geometry.x[m.cells[:, 1]] - m.geometry.x[m.cells[:, 0]]
        return d / m.cell_lengths()[:, None]

    # ------------------------------------------------------------- accessors
    @property
    def comm(self) -> Comm:
        return self._comm

    @property
    def N(self) -> int:
        return self._N

    @property
    def geometric_dimension(self) -> int:
        return self._geom_dim

    @property
    def node_coordinates(self) -> np.ndarray:
        return self._pos

    @property
    def edges(self) -> tuple[np.ndarray, np.ndarray]:
        """``(src, dst)`` node ids of every graph edge, in ``graph.edges()`` order."""
        return self._src, self._dst

    @property
    def num_edges(self) -> int:
        return int(self._src.size)

    @property
    def num_nodes(self) -> int:
        return int(self._pos.shape[0])

    @property
    def edge_colors(self) -> np.ndarray:
        return self._edge_color

    @property
    def edge_radius(self) -> np.ndarray | None:
        return self._edge_radius

    @property
    def degrees(self) -> np.ndarray:
        return self._degree

    @property
    def num_edge_colors(self) -> int:
        return self._num_edge_colors

    @property
    def bifurcation_values(self) -> npt.NDArray[np.int32]:
        return self._bifurcation_values

    @property
    def boundary_values(self) -> npt.NDArray[np.int32]:
        return self._boundary_values

    @property
    def boundary_in_nodes(self) -> npt.NDArray[np.int32]:
        return self._boundary_in_nodes

    @property
    def boundary_out_nodes(self) -> npt.NDArray[np.int32]:
        return self._boundary_out_nodes

    def in_edges(self, bifurcation_idx: int) -> npt.NDArray[np.int32]:
        """Colours of the in-edges of bifurcation ``bifurcation_idx`` (reference ``mesh.py:515-519``)."""
        assert bifurcation_idx < len(self.bifurcation_values)
        return self._bifurcation_in_color.links(int(bifurcation_idx))

    def out_edges(self, bifurcation_idx: int) -> npt.NDArray[np.int32]:
        """Colours of the out-edges of bifurcation ``bifurcation_idx`` (reference ``mesh.py:521-525``)."""
        assert bifurcation_idx < len(self.bifurcation_values)
        return self._bifurcation_out_color.links(int(bifurcation_idx))

    @property
    def in_marker(self) -> int:
        return self._in_marker

    @property
    def out_marker(self) -> int:
        return self._out_marker

    @property
    def orientation(self) -> DG0Function:
        """Cellwise +-1 such that ``orientation * J/|J|`` is the source -> target tangent.

        Cells are stored source -> target here, so this is +1 everywhere.
        """
        if self._orientation is None:
            self._orientation = DG0Function(
                np.ones(self.num_edges * self._N, dtype=np.float64), name="orientation"
            )
        return self._orientation

    @property
    def subdomains(self) -> MeshTags:
        """Cell tags = edge colour (reference ``mesh.py:353-363``)."""
        if self._subdomains is None:
            vals = np.repeat(self._edge_color, self._N)
            self._subdomains = MeshTags(1, np.arange(vals.size), vals, "subdomains")
        return self._subdomains

    @property
    def boundaries(self) -> MeshTags:
        """Vertex tags: node id, or in/out marker on boundary nodes (``mesh.py:402-420``)."""
        if self._facet_markers is None:
            used = np.flatnonzero(self._degree > 0)
            vals = used.astype(np.int64).copy()
            lookup = np.arange(self.num_nodes, dtype=np.int64)
            lookup[self._boundary_in_nodes] = self._in_marker
            lookup[self._boundary_out_nodes] = self._out_marker
            vals = lookup[used]
            self._facet_markers = MeshTags(0, used, vals, "bifurcations")
        return self._facet_markers

    @property
    def submeshes(self) -> list[np.ndarray]:
        """Per colour: the graph edges of that colour (the colour 'submesh')."""
        if self._edge_meshes is None:
            order = np.argsort(self._edge_color, kind="stable")
            cuts = np.searchsorted(self._edge_color[order], np.arange(self._num_edge_colors + 1))
            self._edge_meshes = [order[cuts[c]:cuts[c + 1]] for c in range(self._num_edge_colors)]
        return self._edge_meshes

    @property
    def lm_mesh(self) -> np.ndarray:
        """Point cloud of the bifurcation vertices (one multiplier each)."""
        return self._pos[self._bifurcation_values]

    @property
    def bifurcation_index(self) -> np.ndarray:
        """Node id -> position in ``bifurcation_values`` (``-1`` if not a bifurcation)."""
        return self._bif_index
