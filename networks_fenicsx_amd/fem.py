"""Light function-space / function objects returned by the solver.

The reference returns DOLFINx ``fem.Function`` objects
``[flux_color_0, ..., flux_color_{M-1}, pressure, global_flux]`` (``solver.py:120-135``).
These classes keep the attributes the reference's callers use
(``.x.array``, ``.name``, ``.function_space``, ``.function_space.mesh``,
``.function_space.element.basix_element.degree``) without DOLFINx.

DoF order inside each function (documented, since DOLFINx's internal permutation is
not reproduced):

* flux colour ``c``: the edges of colour ``c`` in ``graph.edges()`` order, ``kN+1``
  node values each (flux degree k; ``N+1`` vertex values for the default P1), source ->
  target;
* pressure: ``N`` cell values per edge, edge-major, source -> target (DG0); continuous
  P_m: one value per graph node with an edge (ascending id), then the ``mN-1`` interior
  node values of every edge, edge-major;
* multiplier: one value per bifurcation, ascending node id.

On a multi-rank run each rank's arrays hold the edges / bifurcations that rank
owns (in the same order), like the local part of a distributed DOLFINx function.
"""

from __future__ import annotations

from dataclasses import dataclass

import numpy as np

__all__ = ["FunctionSpace", "Function", "Constant", "Vector"]


@dataclass
class _BasixElement:
    degree: int
    family: str = "P"
    discontinuous: bool = False


class _Element:
    def __init__(self, family: str, degree: int, discontinuous: bool):
        self.basix_element = _BasixElement(degree, family, discontinuous)


class _IndexMap:
    def __init__(self, n: int):
        self.size_local = n
        self.size_global = n
        self.num_ghosts = 0


class _DofMap:
    def __init__(self, n: int):
        self.index_map = _IndexMap(n)
        self.index_map_bs = 1


class FunctionSpace:
    """A named block of the discrete system (flux colour / pressure / multiplier)."""

    def __init__(self, mesh, kind: str, family: str, degree: int, discontinuous: bool,
                 n_dofs: int, edges: np.ndarray | None = None, color: int | None = None):
        self.mesh = mesh
        self.kind = kind
        self.color = color
        self.edges = edges
        self.nodes = None  # graph nodes of a multiplier space / of P_m's shared node values
        self.element = _Element(family, degree, discontinuous)
        self.dofmap = _DofMap(n_dofs)
        self._n = n_dofs

    @property
    def num_dofs(self) -> int:
        return self._n

    def __repr__(self) -> str:
        return f"FunctionSpace({self.kind}, color={self.color}, dofs={self._n})"


class Vector:
    """``.x`` of a :class:`Function` (DOLFINx ``la.Vector`` subset).

    ``deferred=(source, lo, hi)``: the values are ``source.array()[lo:hi]``, read when
    ``array`` is first used (the solver's output stays on the device until then)."""

    def __init__(self, n: int, array: np.ndarray | None = None, deferred=None):
        if array is not None and array.shape != (n,):
            raise ValueError(f"array must have shape ({n},)")
        self._n = n
        self._deferred = deferred if array is None else None
        self._array = array if array is not None or deferred is not None else np.zeros(
            n, dtype=np.float64)

    @property
    def array(self) -> np.ndarray:
        if self._deferred is not None:
            src, lo, hi = self._deferred
            self._array = src.array()[lo:hi]
            self._deferred = None
        return self._array

    @array.setter
    def array(self, value: np.ndarray) -> None:
        self._deferred = None
        self._array = value

    def scatter_forward(self) -> None:
        return None

    def scatter_reverse(self, *_a) -> None:
        return None


class Function:
    """``array``: an existing float64 buffer to use as ``x.array``; ``deferred``: the
    solver's device-held output (see :class:`Vector`)."""

    def __init__(self, V: FunctionSpace, name: str | None = None,
                 array: np.ndarray | None = None, deferred=None):
        self.function_space = V
        self.name = name or "f"
        self.x = Vector(V.num_dofs, array, deferred)

    def __repr__(self) -> str:
        return f"Function({self.name!r}, {self.function_space!r})"


class Constant:
    """A spatially constant coefficient (stand-in for ``dolfinx.fem.Constant``)."""

    def __init__(self, domain, value):
        self.domain = domain
        self.value = np.asarray(value, dtype=np.float64)

    def __float__(self) -> float:
        return float(self.value)
