"""Post-processing of the solution functions.

Mirrors ``src/networks_fenicsx/post_processing.py``:

* :func:`extract_global_flux` (reference ``:19-52``): the per-colour P1 fluxes gathered
  into one discontinuous P1 ("DG1") field on the whole network, two values per cell
  (its source-side and target-side vertex values), cells edge-major;
* :func:`export_functions` / :func:`export_submeshes` (reference ``:55-97``): the
  reference writes ADIOS2 ``.bp`` / XDMF files. ADIOS2 and DOLFINx IO are not
  available here; these write the same data as ``.npz`` archives (one per function /
  colour) so downstream scripts keep working.
"""

from __future__ import annotations

from pathlib import Path

import numpy as np

from .fem import Function, FunctionSpace
from .mesh import NetworkMesh

__all__ = ["extract_global_flux", "export_functions", "export_submeshes", "integrate_dg1"]


def extract_global_flux(graph_mesh: NetworkMesh, functions: list[Function]) -> Function:
    """Global DG1 flux on the network mesh from ``[flux_0, ..., flux_{M-1}, p, lm]``."""
    flux_functions = functions[:-2]
    N = graph_mesh.N
    if not flux_functions:
        raise ValueError("no flux functions given")
    # edges present in this rank's functions, and their values per vertex
    edges = np.concatenate([f.function_space.edges for f in flux_functions])
    vals = np.concatenate([f.x.array.reshape(-1, N + 1) for f in flux_functions])
    order = np.argsort(edges, kind="stable")
    edges, vals = edges[order], vals[order]
    degree = flux_functions[0].function_space.element.basix_element.degree
    V = FunctionSpace(graph_mesh, "global_flux", "DG", degree, True, edges.size * 2 * N, edges)
    g = Function(V, name="Global_Flux")
    dg = np.empty((edges.size, N, 2), dtype=np.float64)
    dg[:, :, 0] = vals[:, :-1]
    dg[:, :, 1] = vals[:, 1:]
    g.x.array[:] = dg.ravel()
    return g


def integrate_dg1(graph_mesh: NetworkMesh, g: Function) -> tuple[float, float]:
    """``(integral of g, length)`` over the cells held in ``g`` (exact for DG1)."""
    N = graph_mesh.N
    h = graph_mesh.cell_lengths().reshape(-1, N)[g.function_space.edges]
    v = g.x.array.reshape(-1, N, 2)
    return float(np.sum(h * 0.5 * (v[:, :, 0] + v[:, :, 1]))), float(np.sum(h))


def export_functions(functions: list[Function], outpath: Path | str) -> None:
    """Write ``flux_{i}``, ``pressure`` and ``lm`` arrays (``.npz`` instead of ``.bp``)."""
    out = Path(outpath)
    out.mkdir(parents=True, exist_ok=True)
    for i, q in enumerate(functions[:-2]):
        np.savez(out / f"flux_{i}.npz", values=q.x.array, edges=q.function_space.edges)
    np.savez(out / "pressure.npz", values=functions[-2].x.array,
             edges=functions[-2].function_space.edges)
    np.savez(out / "lm.npz", values=functions[-1].x.array)


def export_submeshes(network_mesh: NetworkMesh, outpath: str | Path) -> None:
    """Write every colour's cells and vertex markers (``.npz`` instead of XDMF)."""
    out = Path(outpath)
    out.mkdir(parents=True, exist_ok=True)
    m = network_mesh.mesh
    N = network_mesh.N
    for c, edges in enumerate(network_mesh.submeshes):
        cells = (edges[:, None] * N + np.arange(N)[None, :]).ravel()
        np.savez(out / f"submesh_{c}.npz", x=m.geometry.x, cells=m.cells[cells], edges=edges)
