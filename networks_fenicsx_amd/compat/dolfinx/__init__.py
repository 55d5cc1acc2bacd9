"""Stand-in for the ``dolfinx`` surface used by the networks_fenicsx demos
(``io.VTXWriter``, ``fem.form/Constant/assemble_scalar``, ``common.timed/timing``).
See :mod:`networks_fenicsx_amd.compat`."""

from . import common, fem, io  # noqa: F401

__version__ = "0.10.0+networks_fenicsx_amd.shim"
__all__ = ["common", "fem", "io"]
