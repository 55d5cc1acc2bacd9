"""``networks_fenicsx.network_generation`` -> :mod:`networks_fenicsx_amd.network_generation`."""

from networks_fenicsx_amd.network_generation import *  # noqa: F401,F403
from networks_fenicsx_amd.network_generation import __all__  # noqa: F401
