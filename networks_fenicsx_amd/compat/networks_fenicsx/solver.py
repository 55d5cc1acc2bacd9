"""``networks_fenicsx.solver`` -> :mod:`networks_fenicsx_amd.solver`."""

from networks_fenicsx_amd.solver import *  # noqa: F401,F403
from networks_fenicsx_amd.solver import __all__  # noqa: F401
