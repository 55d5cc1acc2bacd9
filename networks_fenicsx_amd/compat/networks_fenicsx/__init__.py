"""``networks_fenicsx`` alias of :mod:`networks_fenicsx_amd` (same public names as the
reference ``src/networks_fenicsx/__init__.py:12-25``)."""

import networks_fenicsx_amd as _amd
from networks_fenicsx_amd import (  # noqa: F401
    HydraulicNetworkAssembler,
    NetworkMesh,
    Solver,
    network_generation,
    post_processing,
)

__version__ = _amd.__version__
__program_name__ = "networks_fenicsx"
__license__ = _amd.__license__
__author__ = _amd.__author__
__email__ = _amd.__email__

__all__ = ["HydraulicNetworkAssembler", "NetworkMesh", "post_processing", "Solver",
           "network_generation"]
