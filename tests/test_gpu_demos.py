"""The demo API surface on the device path: scripts under tests/demo_scripts run through
``python -m networks_fenicsx_amd.compat`` (the stand-in ufl / dolfinx / mpi4py /
networks_fenicsx packages) and check known answers (closed-form demo_tree fluxes to 1e-10,
junction flux conservation, ufl boundary data == callable boundary data bit for bit)."""

from __future__ import annotations

import subprocess
import sys
from pathlib import Path

import pytest

pytestmark = pytest.mark.gpu

REPO = Path(__file__).resolve().parent.parent


@pytest.mark.parametrize("script,marker", [("tree_flux.py", "tree flux OK"),
                                           ("arterial_nest.py", "arterial nest OK"),
                                           ("y_ufl_bc.py", "ufl bc OK")])
def test_demo_surface(script, marker, tmp_path):
    res = subprocess.run(
        [sys.executable, "-m", "networks_fenicsx_amd.compat",
         str(REPO / "tests" / "demo_scripts" / script), str(tmp_path)],
        cwd=REPO, capture_output=True, text=True, timeout=600)
    assert res.returncode == 0, res.stdout[-3000:] + res.stderr[-3000:]
    assert marker in res.stdout
