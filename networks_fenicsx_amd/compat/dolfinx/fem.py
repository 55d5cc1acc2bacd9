"""``dolfinx.fem`` subset used by the demos (``demos/demo_tree.py:66-71``).

``assemble_scalar(form(f * dx))`` integrates exactly over THIS rank's cells (reduce over
ranks with ``comm.allreduce(..., op=MPI.SUM)`` as the demos do):

* the solver's functions -- flux colour (P1 per edge), pressure (DG0), the global flux of
  ``extract_global_flux`` (DG1) -- integrate over the cells they hold;
* a ``Constant`` or a ``ufl`` coordinate expression integrates over the cells of the
  edges this rank owns (2-point Gauss: exact up to cubic expressions).
"""

from __future__ import annotations

import numbers

import numpy as np

from networks_fenicsx_amd.fem import Constant, Function, FunctionSpace  # noqa: F401
from networks_fenicsx_amd.mesh import IntervalMesh, NetworkMesh

__all__ = ["Constant", "Function", "FunctionSpace", "form", "assemble_scalar"]


def form(f, **_kwargs):
    """Forms are kept symbolic; ``jit_options`` etc. are accepted and ignored."""
    if isinstance(f, (list, tuple)):
        return type(f)(form(g) for g in f)
    return f


def _network_of(obj) -> NetworkMesh:
    if isinstance(obj, NetworkMesh):
        return obj
    if isinstance(obj, IntervalMesh) and obj.network is not None:
        return obj.network
    raise TypeError(f"cannot find the network mesh of {obj!r}")


def _edge_cells(net: NetworkMesh, edges: np.ndarray) -> np.ndarray:
    N = net.N
    return (np.asarray(edges, dtype=np.int64)[:, None] * N + np.arange(N)[None, :]).ravel()


def _integrate_function(g: Function) -> float:
    V = g.function_space
    net = _network_of(V.mesh)
    N = net.N
    h = net.cell_lengths().reshape(-1, N)[V.edges]
    v = g.x.array
    if V.kind == "global_flux":  # DG1: two values per cell
        v = v.reshape(-1, N, 2)
        return float(np.sum(h * 0.5 * (v[:, :, 0] + v[:, :, 1])))
    if V.kind == "flux":  # P1 per edge: N+1 vertex values
        v = v.reshape(-1, N + 1)
        return float(np.sum(h * 0.5 * (v[:, :-1] + v[:, 1:])))
    if V.kind == "pressure":  # DG0
        return float(np.sum(h * v.reshape(-1, N)))
    raise NotImplementedError(f"integral of a {V.kind} function")


def _integrate_expr(expr, net: NetworkMesh) -> float:
    m = net.mesh
    cells = m.cells[_edge_cells(net, net.local_edges())]
    a, b = m.geometry.x[cells[:, 0]], m.geometry.x[cells[:, 1]]
    h = np.linalg.norm(b - a, axis=1)
    g = 0.5 / np.sqrt(3.0)
    total = 0.0
    for w in (0.5 - g, 0.5 + g):
        x = (a * (1 - w) + b * w).T  # (3, n)
        total += 0.5 * float(np.sum(h * np.broadcast_to(expr.eval(x), h.shape)))
    return total


def assemble_scalar(f) -> float:
    """Integral of a (symbolic) form over this rank's cells."""
    forms = getattr(f, "forms", None)
    if forms is not None:
        return float(sum(assemble_scalar(g) for g in forms))
    integrand = getattr(f, "integrand", None)
    measure = getattr(f, "measure", None)
    if integrand is None or measure is None:
        raise TypeError("assemble_scalar expects `integrand * ufl.dx`")
    if measure.kind != "dx" or measure.subdomain_id is not None:
        raise NotImplementedError("only the whole-network cell integral (ufl.dx) is supported")
    if isinstance(integrand, Function):
        return _integrate_function(integrand)
    if isinstance(integrand, Constant):
        net = _network_of(integrand.domain)
        h = net.cell_lengths()[_edge_cells(net, net.local_edges())]
        return float(integrand.value) * float(np.sum(h))
    if isinstance(integrand, numbers.Number):
        raise TypeError("integrate a number through fem.Constant(mesh, value) * ufl.dx")
    if hasattr(integrand, "eval"):
        dom = getattr(integrand, "domain", None)
        if dom is None:
            raise TypeError("coordinate expression without a mesh: use SpatialCoordinate(mesh)")
        return _integrate_expr(integrand, _network_of(dom))
    raise NotImplementedError(f"integrand {integrand!r}")
