"""Post-processing of the solution functions.

Mirrors ``src/networks_fenicsx/post_processing.py``:

* :func:`extract_global_flux` (reference ``:19-52``): the per-colour P_k fluxes gathered
  into one discontinuous P_k ("DG_k") field on the whole network, ``k+1`` values per cell
  (its nodes, source side first), cells edge-major;
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
