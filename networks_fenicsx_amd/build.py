"""Build the in-tree HIP library ``libnxhip.so`` for gfx950.

``hipcc`` cross-compiles for gfx950 without a GPU, so this runs in the CPU build
container too. The ``.so`` is written next to this file (in-tree, git-ignored) so
that it travels to the GPU box with the repository snapshot.
"""

from __future__ import annotations

import os
import shutil
import subprocess
from pathlib import Path

HERE = Path(__file__).resolve().parent
SRC = HERE / "csrc" / "nxhip.hip"
HEADER = HERE.parent / "include" / "nxhip.h"
LIB = HERE / "libnxhip.so"
ARCH = os.environ.get("NXHIP_ARCH", "gfx950")


def _hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), shutil.which("hipcc"), "/opt/rocm/bin/hipcc"):
        if cand and Path(cand).exists():
            return cand
    raise RuntimeError("hipcc not found: the HIP toolchain is required to build libnxhip.so")


def needs_build() -> bool:
    if not LIB.exists():
        return True
    t = LIB.stat().st_mtime
    return any(p.stat().st_mtime > t for p in (SRC, HEADER))


FAST_SRC = HERE / "csrc" / "nxfast.c"


def build_fast(force: bool = False) -> Path | None:
    """The CPython extension ``_nxfast`` (the per-step ``nx_assemble`` / ``nx_solve`` calls
    without ctypes; host plumbing, see csrc/nxfast.c), in-tree next to ``libnxhip.so``.
    Returns None when no C compiler or Python headers are available (ctypes is used)."""
    import sysconfig

    out = HERE / ("_nxfast" + (sysconfig.get_config_var("EXT_SUFFIX") or ".so"))
    if not force and out.exists() and out.stat().st_mtime >= FAST_SRC.stat().st_mtime:
        return out
    cc = shutil.which("gcc") or shutil.which("cc")
    inc = sysconfig.get_paths().get("include")
    if not cc or not inc or not (Path(inc) / "Python.h").exists():
        return None
    tmp = out.with_suffix(".tmp")
    res = subprocess.run([cc, "-O2", "-shared", "-fPIC", "-Wall", f"-I{inc}", "-o", str(tmp),
                          str(FAST_SRC)], capture_output=True, text=True)
    if res.returncode != 0:
        raise RuntimeError(f"building _nxfast failed:\n{res.stderr}")
    os.replace(tmp, out)
    return out


def build(force: bool = False, verbose: bool = False, phase_timing: bool = False) -> Path:
    """Compile ``csrc/nxhip.hip`` into ``libnxhip.so`` (skipped when up to date).
    ``phase_timing`` builds the instrumented debug variant ``libnxhip_phase.so`` instead
    (``-DNX_PHASE_TIMING``; scripts/phase_timing.py loads it via ``NXHIP_LIB``)."""
    out = HERE / "libnxhip_phase.so" if phase_timing else LIB
    if not phase_timing:
        build_fast(force)
    if not phase_timing and not force and not needs_build():
        return LIB
    tmp = out.with_suffix(".so.tmp")
    cmd = [
        _hipcc(),
        f"--offload-arch={ARCH}",
        "-O3",
        "-std=c++17",
        "-fPIC",
        "-shared",
        "-Wall",
        "-o",
        str(tmp),
        str(SRC),
        "-lrccl",
    ] + (["-DNX_PHASE_TIMING"] if phase_timing else [])
    if verbose:
        print(" ".join(cmd))
    res = subprocess.run(cmd, capture_output=True, text=True)
    if res.returncode != 0:
        raise RuntimeError(f"hipcc failed ({res.returncode}):\n{res.stderr}")
    os.replace(tmp, out)
    return out


if __name__ == "__main__":
    print(build(force=True, verbose=True))
