"""The C-ABI library: builds, loads, exports every symbol include/nxhip.h declares,
and fails loudly (no CPU fallback) when no HIP device is visible."""

import re
from pathlib import Path

import pytest

from networks_fenicsx_amd import _lib

HEADER = Path(__file__).resolve().parent.parent / "include" / "nxhip.h"


def declared_symbols():
    text = re.sub(r"/\*.*?\*/", "", HEADER.read_text(), flags=re.S)
    return sorted(set(re.findall(r"\b(?:int|const char\*)\s+(nx_\w+)\s*\(", text)))


def test_header_and_binding_agree():
    assert declared_symbols() == sorted(_lib.EXPORTED_SYMBOLS)


def test_library_exports_every_declared_symbol():
    L = _lib.lib()
    for name in declared_symbols():
        assert hasattr(L, name), name
    assert L.nx_version() >= 10000
    assert isinstance(L.nx_last_error(), bytes)


def test_no_silent_cpu_fallback():
    """Without a GPU the device entry points raise; they never compute on the CPU."""
    import numpy as np

    try:
        n = _lib.device_count()
    except _lib.NxError:
        n = 0
    if n > 0:
        pytest.skip("a HIP device is visible")
    with pytest.raises(_lib.NxError):
        _lib.Handle(0, 2, np.zeros((1, 6)), -np.ones((1, 2), np.int32),
                    np.zeros(1, np.int32), np.zeros(0, np.int32), np.zeros(0))


def test_create_argument_errors():
    """Argument validation happens before any device call."""
    import numpy as np

    with pytest.raises(_lib.NxError, match="N must be"):
        _lib.Handle(0, 0, np.zeros((1, 6)), -np.ones((1, 2), np.int32),
                    np.zeros(1, np.int32), np.zeros(0, np.int32), np.zeros(0))
    with pytest.raises(_lib.NxError, match="edge_lm"):
        _lib.Handle(0, 2, np.zeros((1, 6)), np.array([[0, -1]], np.int32),
                    np.zeros(1, np.int32), np.zeros(0, np.int32), np.zeros(0))


def test_create_fe_argument_errors():
    """nx_create_fe validates the layout and term tables before any device call."""
    import copy

    import numpy as np

    from networks_fenicsx_amd import NetworkMesh
    from networks_fenicsx_amd import network_generation as ng
    from networks_fenicsx_amd.layout_fe import build_fe_layout

    m = NetworkMesh(ng.make_tree(2, 1, 3), N=3)
    src, dst = m.edges
    lay = build_fe_layout(m.node_coordinates, src, dst, m.degrees, 3, 2, 1)
    bad = copy.copy(lay)
    bad.table_kind = lay.table_kind.copy()
    bad.table_kind[0] = 7
    with pytest.raises(_lib.NxError, match="table_kind"):
        _lib.Handle.create_fe(0, bad)
    bad = copy.copy(lay)
    bad.a_idx = lay.a_idx.copy()
    bad.a_idx[0] = 10 ** 6  # a mass term's cell out of range
    with pytest.raises(_lib.NxError, match="out of range"):
        _lib.Handle.create_fe(0, bad)
    bad = copy.copy(lay)
    bad.b_ptr = lay.b_ptr.copy()
    bad.b_ptr[1], bad.b_ptr[2] = bad.b_ptr[2] + 1, bad.b_ptr[1]
    with pytest.raises(_lib.NxError, match="monotone"):
        _lib.Handle.create_fe(0, bad)


def test_import_order_single_runtime_clean_exit():
    """Loading ``libnxhip.so`` BEFORE importing torch (the "wrong" order) must still give
    one HIP runtime in the process and a clean exit: ``_lib.lib()`` imports torch first
    when it is importable (a process that maps the library before torch's HIP libraries
    aborts at exit)."""
    import subprocess
    import sys

    code = (
        "import sys; sys.path.insert(0, %r)\n"
        "from networks_fenicsx_amd import _lib\n"
        "_lib.lib()\n"
        "import torch\n"
        "maps = open('/proc/self/maps').read().splitlines()\n"
        "libs = {l.split()[-1] for l in maps if 'libamdhip64' in l}\n"
        "assert len(libs) == 1, libs\n"
        "print('single runtime:', libs.pop())\n"
    ) % str(HEADER.parent.parent)
    res = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True,
                         timeout=600, cwd="/tmp")
    assert res.returncode == 0, (res.returncode, res.stdout, res.stderr[-2000:])
    assert "single runtime" in res.stdout
