"""The demo stand-ins (networks_fenicsx_amd.compat): CPU checks of the ufl / dolfinx /
mpi4py / networks_fenicsx surface in a subprocess (they must not leak into this
process's imports)."""

from __future__ import annotations

import subprocess
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent


def test_shim_surface(tmp_path):
    res = subprocess.run(
        [sys.executable, "-m", "networks_fenicsx_amd.compat",
         str(REPO / "tests" / "demo_scripts" / "shim_surface.py"), str(tmp_path)],
        cwd=REPO, capture_output=True, text=True, timeout=300)
    assert res.returncode == 0, res.stdout + res.stderr
    assert "shim surface OK" in res.stdout


def test_shims_not_installed_by_default():
    import networks_fenicsx_amd  # noqa: F401

    assert "ufl" not in sys.modules or not hasattr(sys.modules["ufl"], "Form") or \
        "compat" not in str(getattr(sys.modules["ufl"], "__file__", ""))
    assert not any("compat" in p and "networks_fenicsx_amd" in p for p in sys.path)
