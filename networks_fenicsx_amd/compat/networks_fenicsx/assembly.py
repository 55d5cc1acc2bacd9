"""``networks_fenicsx.assembly`` -> :mod:`networks_fenicsx_amd.assembly`."""

from networks_fenicsx_amd.assembly import *  # noqa: F401,F403
from networks_fenicsx_amd.assembly import __all__  # noqa: F401
