"""Stand-in for the ``mpi4py`` surface used by the networks_fenicsx demos
(``demos/demo_tree.py:3,64-71``, ``demos/demo_perf.py:12,77``)."""

from . import MPI  # noqa: F401

__all__ = ["MPI"]
