"""``networks_fenicsx.mesh`` -> :mod:`networks_fenicsx_amd.mesh`."""

from networks_fenicsx_amd.mesh import *  # noqa: F401,F403
from networks_fenicsx_amd.mesh import __all__  # noqa: F401
