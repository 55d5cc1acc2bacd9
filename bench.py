#!/usr/bin/env python3
"""Assemble + MINRES throughput on synthetic binary trees (BASELINE.json metric).

    python bench.py [--gpus N --steps K --warmup W]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N \
        --master-addr 127.0.0.1 --master-port P bench.py --gpus N --steps K --warmup W

Workload: ``make_tree(15 + log2(N), ...)`` with N=15 cells per edge, p_bc = y, f = 0,
R = 1. At one GPU this is the depth-14 tree (1,032,160 DoF, BASELINE
configs[3]); every doubling of the GPU count adds one tree generation, so the work
per GPU stays fixed (weak scaling) and 8 GPUs run the depth-17 tree (configs[4]).

One step = device assembly of the CSR matrix and rhs (``nx_assemble``) + MINRES to
rtol 1e-12 (``nx_solve``), inputs resident in HBM, solution left in HBM. Rank 0
prints one JSON line.
"""

from __future__ import annotations

import argparse
import json
import math
import os
import re
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parent
sys.path.insert(0, str(REPO))

# torch bundles its own HIP runtime / RCCL. Import it BEFORE libnxhip.so is loaded so
# the library binds to those same copies (by SONAME); loading libnxhip.so first would
# put two HIP runtimes in the process (they collide at exit).
import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from networks_fenicsx_amd import _lib  # noqa: E402

_lib.lib()

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md)


def spmv_bytes(n_rows: int, nnz: int) -> int:
    """Algorithmic bytes of one CSR SpMV: f64 values + i32 columns, i32 row pointers,
    x read once, y written once."""
    return 12 * nnz + 4 * (n_rows + 1) + 16 * n_rows


K_MAX_V = 8  # stored Lanczos vectors (csrc/nxhip.hip kMaxV)


def mr_spmv_bytes(n_rows: int, nnz: int, preconditioned: bool, iterations: int = 1) -> float:
    """Algorithmic bytes of one fused ``k_mr_a`` launch that ran a Lanczos step, averaged
    over the ``iterations`` launches of a solve: the CSR SpMV (matrix, row pointers, the
    gathered vector read once) plus the fused vector traffic.

    With the preconditioner the first ``K_MAX_V`` Lanczos vectors are stored and the solution
    is formed once at the end (csrc/nxhip.hip, MrVecs::vs): launch 1 writes y and v
    (2 passes of 8 B per row), launches 2..8 also read r_{k-1} (3 passes); launch 9 hands
    over to the w recurrence (reads v_1..v_8, writes x, w_7, w_8: 12 more passes); later
    launches run the recurrence (r1 r/w, v r/w, w1 r/w, w2 r, x r/w: 9 passes). Without the
    preconditioner every launch runs the recurrence on r (7 passes)."""
    spmv = 12 * nnz + 4 * (n_rows + 1) + 8 * n_rows
    if not preconditioned:
        return spmv + 8 * 7 * n_rows
    its = max(1, iterations)
    passes = 0
    for k in range(1, its + 1):
        passes += 2 if k == 1 else 3 if k <= K_MAX_V else 15 if k == K_MAX_V + 1 else 9
    return spmv + 8 * n_rows * passes / its


def pmc_traffic(kernel_prefix: str):
    """Per-launch HBM bytes of a kernel from the newest committed PMC summary
    (profiles/<tag>_summary.json, written by scripts/summarize_profile.py from
    separate rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of this same workload)."""
    # profile tags sort by round, then by letter suffix length, then letters
    # (r01b < r01z < r01aa < r02a); file mtimes are not meaningful in a fresh checkout
    def tag_key(p):
        m = re.match(r"r(\d+)([a-z]*)_", p.name)
        return (int(m.group(1)), len(m.group(2)), m.group(2)) if m else (-1, 0, p.name)

    cands = sorted((REPO / "profiles").glob("*_summary.json"), key=tag_key)
    for path in reversed(cands):
        doc = json.loads(path.read_text())
        for name, d in doc.get("kernels", {}).items():
            if name.startswith(kernel_prefix) and "hbm_bytes_per_launch" in d:
                return d["hbm_bytes_per_launch"], f"profiles/{path.name}", d.get("avg_ns")
    return None, None, None


def cpu_baseline(mesh, budget_s: float):
    """CPU restatement of the reference path on the host: oracle assembly + SuperLU
    direct solve (the MUMPS stand-in), repeated up to ``budget_s`` seconds."""
    from oracle import nx_oracle as O

    src, dst = mesh.edges
    P = O.build_problem(mesh.node_coordinates, src, dst, mesh.N, mesh.edge_colors)
    runs, t_total = 0, 0.0
    while runs < 1 or (t_total < budget_s and runs < 40):  # ~10-30 s of CPU work
        t0 = time.perf_counter()
        A, b = O.assemble_reference(P, lambda x: x[1])
        O.solve_reference(A, b)
        t_total += time.perf_counter() - t0
        runs += 1
    ms = 1e3 * t_total / runs
    return {"value": P.n_dofs / (ms / 1e3), "unit": "DoF/s", "cores": 1, "kind": "port",
            "ms_per_step": ms,
            "sample": f"{runs} full run(s) of the same workload ({P.n_dofs} DoF): numpy "
                      f"assembly of the reference forms + scipy SuperLU spsolve (1 thread)"}


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--levels", type=int, default=15, help="tree generations at 1 GPU")
    ap.add_argument("--N", type=int, default=15, help="cells per edge")
    ap.add_argument("--rtol", type=float, default=1e-12)
    ap.add_argument("--check-every", type=int, default=4)
    ap.add_argument("--cpu-budget", type=float, default=15.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-pc", action="store_true", help="plain (unpreconditioned) MINRES")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and world > 1:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE {world}", file=sys.stderr)

    if world > 1:
        dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(local_rank)

    from networks_fenicsx_amd import HydraulicNetworkAssembler, NetworkMesh
    from networks_fenicsx_amd import network_generation as ng
    from networks_fenicsx_amd.comm import SerialComm, TorchComm

    extra = int(round(math.log2(world))) if world > 1 else 0
    if world > 1 and 2**extra != world:
        raise SystemExit("world size must be a power of two")
    levels = args.levels + extra
    comm = TorchComm() if world > 1 else SerialComm()
    G = ng.make_tree(levels, levels, levels) if rank == 0 else None
    mesh = NetworkMesh(G, N=args.N, color_strategy="smallest_last", comm=comm)
    del G
    asm = HydraulicNetworkAssembler(mesh)
    asm.compute_forms(p_bc_ex=lambda x: x[1])
    if args.no_pc:
        asm.set_preconditioner(False)
    h = asm.handle
    E, B = mesh.num_edges, len(mesh.bifurcation_values)
    dof_total = E * (2 * args.N + 1) + B

    state = {}

    def step():
        h.assemble(True, True)
        it, rr, conv = h.solve(args.rtol, 50000, args.check_every)
        state["it"], state["relres"], state["conv"] = it, rr, conv

    def barrier():
        if world > 1:
            dist.barrier()

    for _ in range(args.warmup):
        step()
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    h.sync()
    torch.cuda.synchronize()
    barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    ms_per_step = 1e3 * elapsed / args.steps

    # --- per-kernel timing with HIP events on the library's stream (one profiled step)
    h.set_profiling(True)
    h.reset_profile()
    step()
    prof = h.profile()
    h.set_profiling(False)
    spmv_ms = prof["spmv_ms"] / max(prof["spmv_count"], 1)
    asm_ms = prof["asm_ms"] / max(prof["asm_count"], 1)
    warm_spmv_ms = h.bench_spmv(200)
    cold_spmv_ms, cold_copies = h.bench_spmv_cold(120)
    pc_on = asm.preconditioned
    nbytes = mr_spmv_bytes(h.n_rows, h.nnz, pc_on, max(int(prof["spmv_count"]), 1))
    achieved = nbytes / (spmv_ms * 1e-3) / 1e9
    sbytes = spmv_bytes(h.n_rows, h.nnz)
    kname = f"k_mr_a<{str(world > 1).lower()}, {str(pc_on).lower()}>"
    # the committed PMC summaries profile the default workload (C3) on one GPU only
    default_workload = world == 1 and (args.levels, args.N) == (15, 15) and not args.no_pc
    traffic, traffic_src, rocprof_ns = pmc_traffic(kname) if default_workload else (None, None, None)

    # --- parity outside the timed region
    true_rr = h.true_residual()
    parity = {"true_relres": true_rr, "minres_relres": state["relres"], "converged": state["conv"]}
    if world == 1:
        from oracle import nx_oracle as O

        src, dst = mesh.edges
        P = O.build_problem(mesh.node_coordinates, src, dst, mesh.N)
        xa = O.resistor_network_solution(P, lambda x: x[1])
        perm, _ = O.build_permutation(P)
        x = h.solution()
        parity["relerr_vs_analytic"] = float(np.linalg.norm(x - xa[perm]) / np.linalg.norm(xa))

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(mesh, args.cpu_budget)
        cpu["cores"] = 1

    if rank == 0:
        out = {
            "metric": "assemble+solve ms and SpMV HBM GB/s, depth-14 tree, 1/2/4/8 GPU",
            "value": dof_total / (ms_per_step / 1e3),
            "unit": "DoF/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_per_step,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (make_tree binary tree, p_bc = y, f = 0, R = 1)",
            "config": {
                "workload": f"make_tree({levels},{levels},{levels}) depth-{levels - 1} binary "
                            f"tree, N={args.N} cells/edge, assemble + MINRES rtol {args.rtol:g}",
                "dofs": dof_total,
                "nnz": E * (7 * args.N + 1) + 6 * B,
                "edges": E,
                "minres_iterations": state["it"],
                "parallelism": f"edge-partition x{world}" if world > 1 else "single GPU",
                "preconditioner": "tree Schur complement" if pc_on else "none",
            },
            "roofline": {
                "bound": "hbm",
                "kernel": f"{kname} (CSR SpMV fused with the Lanczos step, Givens rotation and "
                          "solution update)",
                "achieved": achieved,
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBS,
                "traffic": traffic,
                "traffic_unit": "bytes per launch (2 x FETCH_SIZE + WRITE_SIZE, gfx950-corrected)",
                "traffic_source": traffic_src,
                "rocprof_avg_launch_ms": rocprof_ns / 1e6 if rocprof_ns else None,
                "algorithmic_bytes_per_launch": nbytes,
                "avg_launch_ms": spmv_ms,
                "spmv_algorithmic_bytes": sbytes,
                "isolated_warm_spmv_ms": warm_spmv_ms,
                "isolated_warm_spmv_GBs": sbytes / (warm_spmv_ms * 1e-3) / 1e9,
                "isolated_cold_spmv_ms": cold_spmv_ms,
                "isolated_cold_spmv_GBs": sbytes / (cold_spmv_ms * 1e-3) / 1e9,
                "cold_rotation_copies": cold_copies,
                "assembly_kernel_ms": asm_ms,
            },
            "cpu_baseline": cpu,
            "parity": parity,
        }
        print(json.dumps(out))
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    asm.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
