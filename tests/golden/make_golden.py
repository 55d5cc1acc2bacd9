"""Generate the committed golden fixtures under tests/golden/.

Run in the build container (it reads /root/reference, which does not exist on the GPU
box; the fixtures it writes are small data files that travel with the repo):

    python tests/golden/make_golden.py

* ``graphs.npz`` -- node coordinates / edges / radii produced by the REFERENCE's own
  ``network_generation.py`` (``/root/reference/src/networks_fenicsx``), imported with a
  no-op stand-in for its only DOLFINx use, the ``dolfinx.common.timed`` decorator
  (``network_generation.py:15, 41, 157``). These pin our generator restatement
  bit-for-bit.
* ``systems.npz`` -- for small configurations: the reference-form system assembled by
  the CPU oracle (``oracle/nx_oracle.py``), its direct solution and the analytic
  resistor-network solution. No reference output exists for these values (DOLFINx /
  PETSc are not installed); they pin the oracle and the device path against drift.
"""

from __future__ import annotations

import importlib.util
import sys
import types
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
REPO = HERE.parent.parent
REF = Path("/root/reference/src/networks_fenicsx/network_generation.py")

TREES = {  # name: make_tree args (n, H, W, dim)
    "Y": (2, 1, 3, 3),
    "demo_tree": (2, 1, 1, 3),
    "double_Y": (2, 3.1, 7.3, 3),
    "depth6": (7, 7, 7, 3),
    "tree5_2d": (5, 2, 1, 2),
    "depth11": (12, 12, 12, 3),
}
ARTERIAL = {  # name: make_arterial_tree kwargs
    "arterial5": dict(N=5, direction=[0.1, 1, 0]),
    "arterial7": dict(N=7),
}


def load_reference_generator():
    stub_dolfinx = types.ModuleType("dolfinx")
    stub_common = types.ModuleType("dolfinx.common")
    stub_common.timed = lambda name: (lambda f: f)
    stub_dolfinx.common = stub_common
    sys.modules.setdefault("dolfinx", stub_dolfinx)
    sys.modules.setdefault("dolfinx.common", stub_common)
    spec = importlib.util.spec_from_file_location("ref_network_generation", REF)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def graph_arrays(G):
    pos = np.asarray([G.nodes[v]["pos"] for v in G.nodes()], dtype=np.float64)
    edges = np.asarray(list(G.edges()), dtype=np.int64).reshape(-1, 2)
    radius = np.asarray([G.edges[e].get("radius", np.nan) for e in G.edges()], dtype=np.float64)
    return pos, edges, radius


def main() -> None:
    ref = load_reference_generator()
    out = {}
    for name, (n, H, W, dim) in TREES.items():
        pos, edges, _ = graph_arrays(ref.make_tree(n, H, W, dim=dim))
        out[f"{name}/pos"], out[f"{name}/edges"] = pos, edges
    for name, kw in ARTERIAL.items():
        kw = dict(kw)
        if "direction" in kw:
            kw["direction"] = np.asarray(kw["direction"], dtype=np.float64)
        pos, edges, radius = graph_arrays(ref.make_arterial_tree(**kw))
        out[f"{name}/pos"], out[f"{name}/edges"], out[f"{name}/radius"] = pos, edges, radius
    np.random.seed(1234)
    pos, edges, radius = graph_arrays(ref.make_arterial_tree(6, random=True))
    out["arterial6_random_seed1234/pos"] = pos
    out["arterial6_random_seed1234/edges"] = edges
    out["arterial6_random_seed1234/radius"] = radius
    np.savez_compressed(HERE / "graphs.npz", **out)

    # oracle systems for small configurations
    sys.path.insert(0, str(REPO))
    from oracle import nx_oracle as O

    systems = {}
    cases = {"Y_N4": ("Y", 4), "demo_tree_N2": ("demo_tree", 2), "demo_tree_N4": ("demo_tree", 4),
             "double_Y_N5": ("double_Y", 5), "depth6_N40": ("depth6", 40),
             "arterial5_N40": ("arterial5", 40)}  # C2, N = 40
    for case, (g, N) in cases.items():
        pos, edges = out[f"{g}/pos"], out[f"{g}/edges"]
        P = O.build_problem(pos, edges[:, 0], edges[:, 1], N)
        pbc = (lambda x: x[0]) if g == "double_Y" else (lambda x: x[1])
        A, b = O.assemble_reference(P, pbc)
        x = O.solve_reference(A, b)
        xa = O.resistor_network_solution(P, pbc)
        Ab, bb, perm, sign = O.to_build_layout(P, A, b)
        if A.shape[0] <= 200:
            systems[f"{case}/indptr"] = Ab.indptr
            systems[f"{case}/indices"] = Ab.indices
            systems[f"{case}/data"] = Ab.data
        systems[f"{case}/rhs_build"] = bb
        systems[f"{case}/x_build"] = x[perm]
        systems[f"{case}/x_analytic_build"] = xa[perm]
        if g.startswith("arterial"):
            # C2 as demo_arterial_tree.py runs it (largest_first colouring): the solution in
            # the reference's function order [flux colour blocks, pressure, multipliers]
            import networkx as nx

            G = ref.make_arterial_tree(**{**ARTERIAL[g],
                                          "direction": np.asarray(ARTERIAL[g]["direction"])})
            col = nx.coloring.greedy_color(nx.line_graph(G.to_undirected()),
                                           strategy=nx.coloring.strategy_largest_first)
            colors = np.asarray([col.get((u, v), col.get((v, u))) for u, v in G.edges()])
            Pc = O.build_problem(pos, edges[:, 0], edges[:, 1], N, colors)
            Ac, bc = O.assemble_reference(Pc, pbc)
            systems[f"{case}/colors"] = colors
            systems[f"{case}/x_ref_blocks"] = O.solve_reference(Ac, bc)
            systems[f"{case}/radius"] = out[f"{g}/radius"]
    np.savez_compressed(HERE / "systems.npz", **systems)
    print("wrote", HERE / "graphs.npz", "and", HERE / "systems.npz")


if __name__ == "__main__":
    main()
