"""MI355X-native assemble + solve path for 1-D hydraulic networks.

Drop-in for the hot path of ``networks_fenicsx`` (``NetworkMesh`` ->
``HydraulicNetworkAssembler`` -> ``Solver``): the same Python surface
(reference ``src/networks_fenicsx/__init__.py:12-25``), with the element assembly and
the linear solve running as hand-written HIP kernels on gfx950 behind the C ABI of
``include/nxhip.h``.
"""

__version__ = "0.1.0"
__program_name__ = "networks_fenicsx_amd"
__license__ = "MIT"
__author__ = ""
__email__ = ""

from . import network_generation, post_processing, timing  # noqa: E402
from .assembly import HydraulicNetworkAssembler  # noqa: E402
from .mesh import NetworkMesh  # noqa: E402
from .solver import Solver  # noqa: E402

__all__ = [
    "HydraulicNetworkAssembler",
    "NetworkMesh",
    "post_processing",
    "Solver",
    "network_generation",
    "timing",
]
