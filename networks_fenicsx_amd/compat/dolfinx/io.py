"""``dolfinx.io.VTXWriter`` stand-in (``demos/demo_tree.py:57-62`` and the other demos).

ADIOS2 is not available, so the writer creates the ``.bp`` path as a directory and writes,
per ``write(t)``, one VTK XML file per function (``step_<k>_<name>.vtu``, what ParaView
would have shown from the ``.bp``; ``post_processing.write_vtu``) and one ``step_<k>.npz``
with every function's values, its graph edges and the vertex coordinates of its cells.
"""

from __future__ import annotations

from pathlib import Path

import numpy as np

__all__ = ["VTXWriter"]


class VTXWriter:
    def __init__(self, comm, filename, output, engine: str = "BP4", mesh_policy=None):
        del engine, mesh_policy
        self.comm = comm
        self.path = Path(filename)
        self.functions = list(output) if isinstance(output, (list, tuple)) else [output]
        self._step = 0

    def __enter__(self) -> "VTXWriter":
        return self

    def __exit__(self, *exc) -> None:
        self.close()

    def write(self, t: float) -> None:
        rank = getattr(self.comm, "rank", 0)
        self.path.mkdir(parents=True, exist_ok=True)
        arrays = {"t": np.float64(t)}
        for f in self.functions:
            V = f.function_space
            arrays[f"{f.name}/values"] = f.x.array
            if getattr(V, "edges", None) is not None:
                arrays[f"{f.name}/edges"] = np.asarray(V.edges)
                net = getattr(V.mesh, "network", V.mesh)
                if hasattr(net, "mesh") and hasattr(net, "N"):
                    N = net.N
                    cells = (np.asarray(V.edges)[:, None] * N + np.arange(N)[None, :]).ravel()
                    arrays[f"{f.name}/cell_x"] = net.mesh.geometry.x[net.mesh.cells[cells]]
        suffix = f"_r{rank}" if getattr(self.comm, "size", 1) > 1 else ""
        np.savez(self.path / f"step_{self._step:04d}{suffix}.npz", **arrays)
        from networks_fenicsx_amd.post_processing import _export_vtu

        for f in self.functions:
            if hasattr(getattr(f.function_space, "mesh", None), "N"):
                _export_vtu(f, self.path / f"step_{self._step:04d}{suffix}_{f.name}.vtu")
        self._step += 1

    def close(self) -> None:
        return None
