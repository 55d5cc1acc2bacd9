"""Stand-in for the ``ufl`` surface used by the networks_fenicsx demos.

* ``SpatialCoordinate(mesh)[i]`` and arithmetic on it -- the pressure boundary data of
  ``demos/demo_Y_bifurcation.py:21-23`` (``x[1]``) and ``demo_double_Y_bifurcation.py``
  (``x[0]``). Expressions evaluate on DOLFINx-style coordinates ``x`` of shape ``(3, n)``
  through ``.eval(x)``, the protocol :meth:`HydraulicNetworkAssembler.compute_forms`
  accepts (reference ``assembly.py:24-25``: ``PressureFunction.eval``).
* ``dx`` / ``ds`` measures: ``integrand * dx`` is a form for
  ``dolfinx.fem.assemble_scalar`` (``demos/demo_tree.py:66-68``).
"""

from __future__ import annotations

import math
import numbers

import numpy as np

__all__ = ["SpatialCoordinate", "Expr", "Form", "Measure", "dx", "ds", "sin", "cos", "exp",
           "sqrt", "ln", "pi"]

pi = math.pi


class Expr:
    """A scalar expression of the spatial coordinate."""

    domain = None  # the mesh of the SpatialCoordinate it is built from

    def eval(self, x: np.ndarray) -> np.ndarray:  # pragma: no cover - interface
        raise NotImplementedError

    # arithmetic
    def __add__(self, o):
        return _Bin(np.add, self, o)

    def __radd__(self, o):
        return _Bin(np.add, o, self)

    def __sub__(self, o):
        return _Bin(np.subtract, self, o)

    def __rsub__(self, o):
        return _Bin(np.subtract, o, self)

    def __mul__(self, o):
        if isinstance(o, Measure):
            return Form(self, o)
        return _Bin(np.multiply, self, o)

    def __rmul__(self, o):
        return _Bin(np.multiply, o, self)

    def __truediv__(self, o):
        return _Bin(np.divide, self, o)

    def __rtruediv__(self, o):
        return _Bin(np.divide, o, self)

    def __pow__(self, o):
        return _Bin(np.power, self, o)

    def __neg__(self):
        return _Un(np.negative, self)


def _value(a, x: np.ndarray):
    if isinstance(a, Expr):
        return a.eval(x)
    if isinstance(a, numbers.Number):
        return float(a)
    if hasattr(a, "value"):  # fem.Constant
        return float(np.asarray(a.value))
    raise TypeError(f"cannot evaluate {a!r} as a coordinate expression")


def _domain(*args):
    for a in args:
        d = getattr(a, "domain", None)
        if d is not None:
            return d
    return None


class _Bin(Expr):
    def __init__(self, op, a, b):
        self.op, self.a, self.b = op, a, b
        self.domain = _domain(a, b)

    def eval(self, x):
        return self.op(_value(self.a, x), _value(self.b, x))


class _Un(Expr):
    def __init__(self, op, a):
        self.op, self.a = op, a
        self.domain = _domain(a)

    def eval(self, x):
        return self.op(_value(self.a, x))


class _Component(Expr):
    def __init__(self, i: int, domain=None):
        self.i = int(i)
        self.domain = domain

    def eval(self, x):
        return np.asarray(x)[self.i]


class SpatialCoordinate(Expr):
    """``x = SpatialCoordinate(mesh)``; ``x[i]`` is the i-th coordinate."""

    def __init__(self, domain=None):
        self.domain = domain

    def __getitem__(self, i: int) -> Expr:
        return _Component(i, self.domain)

    def eval(self, x):
        return np.asarray(x)


def _fn(op):
    def f(a):
        return _Un(op, a) if isinstance(a, Expr) else op(a)

    return f


sin, cos, exp, sqrt, ln = _fn(np.sin), _fn(np.cos), _fn(np.exp), _fn(np.sqrt), _fn(np.log)


class Measure:
    def __init__(self, kind: str, subdomain_id=None):
        self.kind = kind
        self.subdomain_id = subdomain_id

    def __call__(self, subdomain_id=None, **_kw) -> "Measure":
        return Measure(self.kind, subdomain_id)

    def __rmul__(self, integrand) -> "Form":
        return Form(integrand, self)


class Form:
    """``integrand * measure`` (one integral)."""

    def __init__(self, integrand, measure: Measure):
        self.integrand = integrand
        self.measure = measure

    def __add__(self, o: "Form") -> "FormSum":
        return FormSum([self, o])


class FormSum:
    def __init__(self, forms):
        self.forms = list(forms)

    def __add__(self, o):
        return FormSum(self.forms + (o.forms if isinstance(o, FormSum) else [o]))


dx = Measure("dx")
ds = Measure("ds")
