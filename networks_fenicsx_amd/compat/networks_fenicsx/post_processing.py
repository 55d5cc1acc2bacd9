"""``networks_fenicsx.post_processing`` -> :mod:`networks_fenicsx_amd.post_processing`."""

from networks_fenicsx_amd.post_processing import *  # noqa: F401,F403
from networks_fenicsx_amd.post_processing import __all__  # noqa: F401
