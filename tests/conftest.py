import sys
from pathlib import Path

import numpy as np
import pytest

REPO = Path(__file__).resolve().parent.parent
if str(REPO) not in sys.path:
    sys.path.insert(0, str(REPO))

GOLDEN = REPO / "tests" / "golden"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); run with -m gpu")
    config.addinivalue_line("markers", "slow: larger CPU cases")


@pytest.fixture(scope="session")
def graphs():
    with np.load(GOLDEN / "graphs.npz") as z:
        return {k: z[k] for k in z.files}


@pytest.fixture(scope="session")
def systems():
    with np.load(GOLDEN / "systems.npz") as z:
        return {k: z[k] for k in z.files}
