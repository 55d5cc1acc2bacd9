#!/usr/bin/env python3
"""Store-site ledger of k_dir_step at C3.

Two modes:

* ``run``: the bench workload's direct step, ``--steps`` launches, on the debug build
  (``NXHIP_LIB=.../libnxhip_phase.so``); ``NXHIP_LEDGER`` (a bit mask, see NX_LEDGER in
  nxhip.hip) drops store classes. Run it under ``rocprofv3 --pmc WRITE_SIZE`` once per mask
  (scripts/gpu_run.sh ``ledger``).
* ``summarize <dir>``: reads ``<dir>/m<mask>/pmc_counter_collection.csv`` and prints, per
  mask, k_dir_step's average WRITE_SIZE per launch and the bytes the dropped class accounts
  for next to its algorithmic bytes.
"""

from __future__ import annotations

import csv
import json
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO))

CLASSES = {1: "CSR values", 2: "rhs", 4: "x", 16: "multiplier rows (values, rhs)"}


def algorithmic(E: int, N: int, B: int, nnz_lm: int) -> dict:
    dofs = E * (2 * N + 1) + B
    nnz = E * (7 * N + 1) + nnz_lm
    return {1: 8 * (nnz - nnz_lm), 2: 8 * (dofs - B), 4: 8 * dofs, 16: 8 * (nnz_lm + B)}


def run(steps: int) -> None:
    import torch  # noqa: F401  (before the HIP library)

    from networks_fenicsx_amd import HydraulicNetworkAssembler, NetworkMesh
    from networks_fenicsx_amd import network_generation as ng

    mesh = NetworkMesh(ng.make_tree(15, 15, 15), N=15, color_strategy="smallest_last")
    asm = HydraulicNetworkAssembler(mesh)
    asm.compute_forms(p_bc_ex=lambda x: x[1])
    asm.set_direct(True)
    h = asm.handle
    for _ in range(steps):
        asm.assemble()
        h.solve(1e-12, 100, 4)
    print("path", h.direct_path(), "E", mesh.num_edges, "B", len(mesh.bifurcation_values))
    asm.close()


def summarize(d: Path) -> None:
    rows = {}
    for sub in sorted(d.glob("m*")):
        mask = int(sub.name[1:])
        f = sub / "pmc_counter_collection.csv"
        if not f.exists():
            continue
        v = [float(r["Counter_Value"]) for r in csv.DictReader(open(f))
             if r["Counter_Name"] == "WRITE_SIZE" and "k_dir_step" in r["Kernel_Name"]]
        if v:
            rows[mask] = sum(v[1:]) / max(1, len(v) - 1) * 1024 if len(v) > 1 else v[0] * 1024
    E, N, B = 32767, 15, 16383
    alg = algorithmic(E, N, B, 6 * B)
    base = rows.get(0)
    out = {"write_bytes_per_launch": rows, "algorithmic": alg, "classes": {}}
    for bit, name in CLASSES.items():
        if base is not None and bit in rows:
            dropped = base - rows[bit]
            out["classes"][name] = {"written": dropped, "algorithmic": alg[bit],
                                    "ratio": dropped / alg[bit]}
    if base is not None:
        out["total_algorithmic_writes"] = sum(alg.values())
        out["unattributed"] = base - sum(c["written"] for c in out["classes"].values())
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run(int(sys.argv[2]) if len(sys.argv) > 2 else 6)
    else:
        summarize(Path(sys.argv[2]))
