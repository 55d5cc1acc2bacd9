#!/usr/bin/env python3
"""Phase timing of the MINRES + preconditioner kernels (debug build, GPU box).

Loads ``libnxhip_phase.so`` (``python -c 'from networks_fenicsx_amd import build;
build.build(phase_timing=True)'``), solves the bench workload and prints, for the last
complete iteration, workgroup 0's phase stamps and every kernel's latest workgroup start
and end (wall_clock64, 100 MHz), relative to k_mr_a's start.

    python scripts/phase_timing.py [levels] [N] [direct]

With ``direct`` the direct tree solve runs (its sweeps in mode 3; times relative to the up
sweep's start).
"""

from __future__ import annotations

import ctypes as C
import os
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
os.environ.setdefault("NXHIP_LIB", str(REPO / "networks_fenicsx_amd" / "libnxhip_phase.so"))
sys.path.insert(0, str(REPO))

from networks_fenicsx_amd import HydraulicNetworkAssembler, NetworkMesh, _lib  # noqa: E402
from networks_fenicsx_amd import network_generation as ng  # noqa: E402

KERNELS = {0: "k_mr_a", 16: "k_pc_up_lds", 32: "k_pc_top_lds", 48: "k_pc_down_lds"}
PHASES = {
    0: ["start", "rotation", "spmv+update"],
    16: ["start", "chains", "phase A", "levels+store", "levels", "wave set-up"],
    32: ["start", "A1/A2 gathers", "A3 fold", "up levels", "back-sub"],
    48: ["start", "phase A", "levels+slots", "chains"],
}


def main() -> int:
    levels = int(sys.argv[1]) if len(sys.argv) > 1 else 15
    N = int(sys.argv[2]) if len(sys.argv) > 2 else 15
    mesh = NetworkMesh(ng.make_tree(levels, levels, levels), N=N, color_strategy="smallest_last")
    asm = HydraulicNetworkAssembler(mesh)
    asm.compute_forms(p_bc_ex=lambda x: x[1])
    asm.assemble()
    h = asm.handle
    lib = _lib.lib()
    fn = lib.nx_debug_phases
    fn.argtypes = [C.POINTER(C.c_ulonglong), C.c_int32]
    direct = len(sys.argv) > 3 and sys.argv[3] == "direct"
    asm.set_direct(direct)
    _lib.set_lean(False)  # the general path: k_mr_a stamps of full iterations too
    for _ in range(3):
        it, rr, conv = h.solve(1e-12, 50000, 32)
    buf = (C.c_ulonglong * 128)()
    _lib.check(fn(buf, 128))
    g = list(buf)
    t0 = g[16] if direct else g[0]
    ref = "k_pc_up_lds" if direct else "k_mr_a"
    print(f"iterations {it}, converged {conv}; times in us relative to {ref} start (wg 0)")
    for base, name in KERNELS.items():
        stamps = [g[base + i] for i in range(len(PHASES[base]))]
        rel = [(x - t0) / 100.0 if x else float("nan") for x in stamps]
        steps = "  ".join(f"{p}={r:8.2f}" for p, r in zip(PHASES[base], rel))
        last_start = (g[base + 14] - t0) / 100.0
        last_end = (g[base + 15] - t0) / 100.0
        print(f"{name:14s} {steps}  | latest wg start {last_start:8.2f}  end {last_end:8.2f}")
    fw = lib.nx_debug_wg
    fw.argtypes = [C.POINTER(C.c_ulonglong), C.POINTER(C.c_ulonglong)]
    S = (C.c_ulonglong * (8 * 512))()
    E = (C.c_ulonglong * (8 * 512))()
    _lib.check(fw(S, E))
    import numpy as np

    S = np.array(S, dtype=np.float64).reshape(8, 512)
    E = np.array(E, dtype=np.float64).reshape(8, 512)
    njobs = asm._pc.n_jobs if asm._pc is not None else 0
    for k, name in ((1, "up"), (3, "down")):
        s0 = S[k, :njobs]
        e0 = E[k, :njobs]
        base = s0.min()
        st = (s0 - base) / 100.0
        en = (e0 - base) / 100.0
        dur = en - st
        late = np.argsort(st)[-5:]
        print(f"{name}: wg start spread {st.max():.2f} us; duration min/med/max "
              f"{dur.min():.2f}/{np.median(dur):.2f}/{dur.max():.2f} us; end spread "
              f"{en.min():.2f}..{en.max():.2f}; latest starters {late.tolist()} at "
              f"{np.round(st[late], 2).tolist()}; longest {np.argsort(dur)[-5:].tolist()}")
    asm.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
