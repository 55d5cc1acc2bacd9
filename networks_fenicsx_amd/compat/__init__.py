"""Run networks_fenicsx demo scripts unchanged on the MI355X path.

The reference demos (``demos/demo_tree.py``, ``demo_arterial_tree.py``,
``demo_Y_bifurcation.py``, ``demo_double_Y_bifurcation.py``) import ``networks_fenicsx``,
``dolfinx``, ``ufl`` and ``mpi4py``. This directory holds minimal stand-ins for exactly
the parts of those packages that the demos touch, implemented on top of
``networks_fenicsx_amd``:

* ``networks_fenicsx``  -- alias of this package (same classes, same module names);
* ``ufl``               -- ``SpatialCoordinate`` expressions (``x[1]``, arithmetic,
                           ``sin``/``cos``/``exp``/``sqrt``/``ln``), the ``dx``/``ds`` measures;
* ``dolfinx``           -- ``io.VTXWriter`` (writes ``.npz`` steps inside the ``.bp``
                           directory: ADIOS2 is not available), ``fem.form``,
                           ``fem.Constant``, ``fem.assemble_scalar`` (exact integrals of the
                           network functions over this rank's cells), ``common.timed`` /
                           ``timing`` / ``list_timings`` / ``Timer``;
* ``mpi4py``            -- ``MPI.COMM_WORLD`` (the host control plane of
                           :mod:`networks_fenicsx_amd.comm`) and the ``SUM``/``MAX``/``MIN`` ops.

They are NOT on ``sys.path`` by default (they would shadow real installations). Use

    python -m networks_fenicsx_amd.compat path/to/demo_tree.py [args]

or call :func:`install` before importing the demo's modules.
"""

from __future__ import annotations

import sys
from pathlib import Path

SHIM_DIR = Path(__file__).resolve().parent

__all__ = ["install", "SHIM_DIR"]


def install() -> None:
    """Put the stand-in packages first on ``sys.path`` (idempotent)."""
    p = str(SHIM_DIR)
    if p not in sys.path:
        sys.path.insert(0, p)
