"""Post-processing of the solution functions.

Mirrors ``src/networks_fenicsx/post_processing.py``:

* :func:`extract_global_flux` (reference ``:19-52``): the per-colour P_k fluxes gathered
  into one discontinuous P_k ("DG_k") field on the whole network, ``k+1`` values per cell
  (its nodes, source side first), cells edge-major;
* :func:`export_functions` / :func:`export_submeshes` (reference ``:55-97``): the
  reference writes ADIOS2 ``.bp`` (VTXWriter) / XDMF files. ADIOS2 and DOLFINx IO are not
  available here; these write VTK XML files that ParaView opens the same way (``.vtu``: one
  per function, every cell with its own nodes so discontinuous fields stay exact; P_k
  flux as Lagrange curves) and XDMF with inline XML data for the submeshes, plus the raw
  arrays as ``.npz`` archives (one per function / colour).
"""

from __future__ import annotations

import base64

from pathlib import Path

import numpy as np

from .fem import Function, FunctionSpace
from .mesh import NetworkMesh

__all__ = ["extract_global_flux", "export_functions", "export_submeshes", "integrate_dg1",
           "write_vtu"]


def extract_global_flux(graph_mesh: NetworkMesh, functions: list[Function]) -> Function:
    """Global DG_k flux on the network mesh from ``[flux_0, ..., flux_{M-1}, p, lm]``.

    ``k`` is the flux degree (reference ``:31-33``); every cell gets the ``k+1`` node values
    of its edge's flux (source side first), cells edge-major."""
    flux_functions = functions[:-2]
    N = graph_mesh.N
    if not flux_functions:
        raise ValueError("no flux functions given")
    degree = flux_functions[0].function_space.element.basix_element.degree
    # edges present in this rank's functions, and their values per node
    edges = np.concatenate([f.function_space.edges for f in flux_functions])
    vals = np.concatenate([f.x.array.reshape(-1, degree * N + 1) for f in flux_functions])
    order = np.argsort(edges, kind="stable")
    edges, vals = edges[order], vals[order]
    V = FunctionSpace(graph_mesh, "global_flux", "DG", degree, True,
                      edges.size * (degree + 1) * N, edges)
    g = Function(V, name="Global_Flux")
    nodes = np.arange(N)[:, None] * degree + np.arange(degree + 1)[None, :]  # (N, k+1)
    g.x.array[:] = vals[:, nodes].ravel()
    return g


def integrate_dg1(graph_mesh: NetworkMesh, g: Function) -> tuple[float, float]:
    """``(integral of g, length)`` over the cells held in ``g`` (exact for the DG_k field
    :func:`extract_global_flux` returns; the name is kept from the P1 default)."""
    from .element import element_tensors

    N = graph_mesh.N
    degree = g.function_space.element.basix_element.degree
    weights = element_tensors(1, degree)[2]  # int_0^1 of the degree-k Lagrange basis
    h = graph_mesh.cell_lengths().reshape(-1, N)[g.function_space.edges]
    v = g.x.array.reshape(-1, N, degree + 1)
    return float(np.sum(h * (v @ weights))), float(np.sum(h))


_VTK_VERTEX, _VTK_LINE, _VTK_LAGRANGE_CURVE = 1, 3, 68


def write_vtu(path: Path | str, pts: np.ndarray, cell_type: int, point_data: dict | None = None,
              cell_data: dict | None = None) -> None:
    """VTK XML unstructured grid (ASCII) of ``pts`` (cells, nodes per cell, 3): every cell its
    own points (a Lagrange curve lists its two ends, then its interior nodes)."""
    pts = np.asarray(pts, dtype=np.float64)
    nc, npc = pts.shape[0], pts.shape[1]

    def arr(name, a, ncomp=1, kind="Float64"):
        a = np.asarray(a).ravel()
        if kind == "Float64" and not np.all(np.isfinite(a)):
            # (VTK's ASCII reader cannot parse 'nan' -- e.g. a node value another rank
            # owns: inline binary, base64 of a UInt32 byte count then the little-endian
            # doubles, which carries NaN as such)
            raw = np.ascontiguousarray(a, dtype="<f8").tobytes()
            body = base64.b64encode(np.uint32(len(raw)).astype("<u4").tobytes() + raw).decode()
            return (f'<DataArray type="Float64" Name="{name}" NumberOfComponents="{ncomp}" '
                    f'format="binary">{body}</DataArray>')
        body = " ".join(repr(float(v)) if kind == "Float64" else str(int(v)) for v in a)
        return (f'<DataArray type="{kind}" Name="{name}" NumberOfComponents="{ncomp}" '
                f'format="ascii">{body}</DataArray>')

    lines = ['<?xml version="1.0"?>',
             '<VTKFile type="UnstructuredGrid" version="1.0" byte_order="LittleEndian">',
             "<UnstructuredGrid>",
             f'<Piece NumberOfPoints="{nc * npc}" NumberOfCells="{nc}">',
             "<Points>", arr("Points", pts.reshape(-1, 3), 3), "</Points>",
             "<Cells>", arr("connectivity", np.arange(nc * npc), kind="Int64"),
             arr("offsets", npc * np.arange(1, nc + 1), kind="Int64"),
             arr("types", np.full(nc, cell_type), kind="UInt8"), "</Cells>"]
    if point_data:
        lines.append("<PointData>")
        lines += [arr(k, v) for k, v in point_data.items()]
        lines.append("</PointData>")
    if cell_data:
        lines.append("<CellData>")
        lines += [arr(k, v) for k, v in cell_data.items()]
        lines.append("</CellData>")
    lines += ["</Piece>", "</UnstructuredGrid>", "</VTKFile>"]
    Path(path).write_text("\n".join(lines) + "\n")


def _cell_points(mesh: NetworkMesh, edges: np.ndarray, npc: int) -> np.ndarray:
    """(edges x N cells, npc nodes, 3): the cells of ``edges`` with npc equispaced nodes each,
    in VTK's Lagrange-curve order (ends first, then the interior)."""
    N = mesh.N
    x = np.zeros((mesh.mesh.geometry.x.shape[0], 3))
    x[:, : mesh.mesh.geometry.x.shape[1]] = mesh.mesh.geometry.x
    cells = mesh.mesh.cells[(np.asarray(edges, dtype=np.int64)[:, None] * N
                             + np.arange(N)[None, :]).ravel()]
    t = np.arange(npc) / max(npc - 1, 1)
    t = np.concatenate([[0.0, 1.0], t[1:-1]]) if npc > 2 else t
    a, b = x[cells[:, 0]], x[cells[:, 1]]
    return a[:, None, :] + (b - a)[:, None, :] * t[None, :, None]


def _vtk_order(npc: int) -> np.ndarray:
    """Node order of a Lagrange curve: 0, last, then 1 .. last - 1."""
    return np.concatenate([[0, npc - 1], np.arange(1, npc - 1)]) if npc > 2 else np.arange(npc)


def _export_vtu(fn: Function, path: Path) -> None:
    V = fn.function_space
    mesh, N = V.mesh, V.mesh.N
    deg = V.element.basix_element.degree
    vals = np.asarray(fn.x.array)
    name = fn.name or V.kind
    if V.kind == "multiplier":  # one vertex per bifurcation
        nodes = np.asarray(V.nodes if V.nodes is not None else [], dtype=np.int64)
        pos = np.zeros((nodes.size, 3))
        c = np.asarray(mesh.node_coordinates)[nodes]
        pos[:, : c.shape[1]] = c
        write_vtu(path, pos[:, None, :], _VTK_VERTEX, point_data={name: vals})
        return
    edges = np.asarray(V.edges, dtype=np.int64)
    if V.element.basix_element.discontinuous and deg == 0:  # DG0: one value per cell
        write_vtu(path, _cell_points(mesh, edges, 2), _VTK_LINE, cell_data={name: vals})
        return
    if V.kind == "flux" or (V.kind == "global_flux"):
        if V.kind == "global_flux":  # DG_k: k + 1 values per cell
            per_cell = vals.reshape(-1, deg + 1)
        else:  # P_k per edge: kN + 1 nodes along the edge
            v = vals.reshape(edges.size, deg * N + 1)
            idx = np.arange(N)[:, None] * deg + np.arange(deg + 1)[None, :]
            per_cell = v[:, idx].reshape(-1, deg + 1)
    else:  # continuous P_m pressure: the shared node values, then the interiors per edge
        nodes = np.asarray(V.nodes, dtype=np.int64)
        src, dst = mesh.edges
        nv = np.full(int(max(nodes.max(initial=-1), src.max(), dst.max())) + 1, np.nan)
        nv[nodes] = vals[: nodes.size]  # (a node another rank owns stays NaN)
        inner = vals[nodes.size:].reshape(edges.size, deg * N - 1)
        full = np.concatenate([nv[src[edges]][:, None], inner, nv[dst[edges]][:, None]], axis=1)
        idx = np.arange(N)[:, None] * deg + np.arange(deg + 1)[None, :]
        per_cell = full[:, idx].reshape(-1, deg + 1)
    npc = deg + 1
    ctype = _VTK_LINE if npc == 2 else _VTK_LAGRANGE_CURVE
    write_vtu(path, _cell_points(mesh, edges, npc), ctype,
              point_data={name: per_cell[:, _vtk_order(npc)]})


def export_functions(functions: list[Function], outpath: Path | str) -> None:
    """Write ``flux_{i}``, ``pressure`` and ``lm`` as ``.vtu`` (in place of the reference's
    ``.bp``) and their raw arrays as ``.npz``. On several ranks every rank writes its own
    piece, ``<name>_r{rank}`` (the reference writes one collective file; ranks must not
    overwrite each other's)."""
    out = Path(outpath)
    out.mkdir(parents=True, exist_ok=True)
    comm = getattr(functions[-1].function_space.mesh, "comm", None)
    size = int(getattr(comm, "size", 1) or 1)
    sfx = f"_r{int(comm.rank)}" if size > 1 else ""
    for i, q in enumerate(functions[:-2]):
        _export_vtu(q, out / f"flux_{i}{sfx}.vtu")
    _export_vtu(functions[-2], out / f"pressure{sfx}.vtu")
    _export_vtu(functions[-1], out / f"lm{sfx}.vtu")
    for i, q in enumerate(functions[:-2]):
        np.savez(out / f"flux_{i}{sfx}.npz", values=q.x.array, edges=q.function_space.edges)
    np.savez(out / f"pressure{sfx}.npz", values=functions[-2].x.array,
             edges=functions[-2].function_space.edges)
    np.savez(out / f"lm{sfx}.npz", values=functions[-1].x.array)


def export_submeshes(network_mesh: NetworkMesh, outpath: str | Path) -> None:
    """Write every colour's submesh as XDMF with inline XML data (``submesh_{c}.xdmf``: its
    cells as a polyline topology, the network mesh's points) and as ``.npz``."""
    out = Path(outpath)
    out.mkdir(parents=True, exist_ok=True)
    m = network_mesh.mesh
    N = network_mesh.N
    x = np.zeros((m.geometry.x.shape[0], 3))
    x[:, : m.geometry.x.shape[1]] = m.geometry.x
    for c, edges in enumerate(network_mesh.submeshes):
        cells = m.cells[(edges[:, None] * N + np.arange(N)[None, :]).ravel()]
        np.savez(out / f"submesh_{c}.npz", x=m.geometry.x, cells=cells, edges=edges)
        topo = " ".join(str(int(v)) for v in cells.ravel())
        geo = " ".join(repr(float(v)) for v in x.ravel())
        (out / f"submesh_{c}.xdmf").write_text(
            '<?xml version="1.0"?>\n<Xdmf Version="3.0">\n<Domain>\n'
            f'<Grid Name="submesh_{c}" GridType="Uniform">\n'
            f'<Topology TopologyType="Polyline" NodesPerElement="2" '
            f'NumberOfElements="{cells.shape[0]}">\n'
            f'<DataItem Dimensions="{cells.shape[0]} 2" NumberType="Int" Format="XML">'
            f"{topo}</DataItem>\n</Topology>\n"
            f'<Geometry GeometryType="XYZ">\n<DataItem Dimensions="{x.shape[0]} 3" '
            f'NumberType="Float" Precision="8" Format="XML">{geo}</DataItem>\n</Geometry>\n'
            "</Grid>\n</Domain>\n</Xdmf>\n")
