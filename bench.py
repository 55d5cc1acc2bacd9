#!/usr/bin/env python3
"""Assemble + MINRES throughput on synthetic binary trees (BASELINE.json metric).

    python bench.py [--gpus N --steps K --warmup W]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N \
        --master-addr 127.0.0.1 --master-port P bench.py --gpus N --steps K --warmup W

``--gpus N > 1`` without a launcher starts the ``torch.distributed.run`` line above as a
child process (before torch or ``libnxhip.so`` is loaded) and exits with its code; a run
whose ``WORLD_SIZE`` differs from ``--gpus`` fails instead of measuring something else.

Workload (p_bc = y, f = 0, R = 1, ``color_strategy="smallest_last"``):

* 1 GPU: ``make_tree(15,15,15)``, N = 15 -- the depth-14 tree, 1,032,160 DoF (configs[3],
  the configuration the metric is quoted on);
* P = 2^k GPUs: ``make_tree(15+k, 15+k, 15+k)``, N = 15 -- one tree generation per GPU
  doubling, the same N as on one GPU, so every GPU carries the one-GPU load (weak scaling,
  ~1.03 M rows per GPU; 8 GPUs: 8,257,504 DoF). ``--N 19`` gives SURVEY's C4 at 8 GPUs
  (``make_tree(18,18,18)``, N = 19, 10,354,648 DoF, configs[4]). Rank 0 also times the SAME
  workload on its GPU alone (``strong_scaling``), so T1 / TP is measured in the same run.

One step = device assembly of the CSR matrix and rhs (``nx_assemble``) + the solve
(``nx_solve``), inputs resident in HBM, solution left in HBM. The solve is what the
reference's default options ask for (``ksp_type=preonly`` + ``pc_type=lu``: a direct
factorisation, solver.py:58-65): on one GPU the direct tree solve (block LU through the
tree sweeps, true residual checked, rtol 1e-12, one refinement step if it misses; across
P ranks one launch per rank, ``k_dir_xr``, exchanging the coarse partials and the residual
with the other ranks' kernels through peer-mapped mailboxes, the two-all-reduce graph path
as the fallback), with ``--solver minres`` preconditioned
MINRES to rtol 1e-12. The other solver is timed on the same workload and reported beside
(one GPU). Rank 0 prints one JSON line.
"""

from __future__ import annotations

import argparse
import json
import math
import os
import platform
import re
import socket
import subprocess
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parent
sys.path.insert(0, str(REPO))

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md)
PROF_STEPS = 20  # eager steps with HIP events bound to each dispatch (the roofline entries)
METRIC = "assemble+solve ms and SpMV HBM GB/s, depth-14 tree, 1/2/4/8 GPU"


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


def res_chunks(n: int) -> int:
    """256-row chunks per k_residual_ck block: csrc/nxhip.hip res_chunks()."""
    return 4 if n > (4 << 20) else 2


def direct_kernel_bytes(n: int, nnz: int, n_e: int, E: int, N: int, B: int, nblk: int,
                        fused: bool = False, n_jobs: int = 0, n_left: int = 0) -> dict:
    """Algorithmic bytes per launch of the direct solve's kernels:
    f64 vectors, int32 indices, the lumped mass dq (E (N+1)) read by every chain sweep.
    ``fused``: the down sweep forms the residual (reads the edge geometry and R to regenerate
    the cell masses, stores r), k_dir_publish_fr sums its partials and forms the ``n_left``
    multiplier rows of the top part from the CSR (3 entries each) instead of k_residual_ck."""
    dq = 8 * E * (N + 1)
    if fused:
        return {
            "k_dir_publish_fr": 16 * n_jobs + n_left * (8 + 3 * 20 + 16),
            "k_pc_up_lds": 8 * n_e + dq + 24 * E + 8 * E + 64 * B,
            # + edge_x / R (56 B per edge) read, r stored at the edge DoFs and local multipliers
            # (+ the top part's inputs, ~40 B per top slot and hanging chain: < 0.1 MB)
            "k_pc_down_lds": 8 * n_e + dq + 8 * n + 16 * E + 24 * B + 56 * E + 8 * n_e + 8 * B,
            "k_pc_top_lds": 64 * 1024,
            "k_assemble_seg": 8 * nnz + 8 * n + dq + 80 * E,
        }
    return {
        # CSR SpMV of x, b read, r stored (for a refinement step); two partials per block
        "k_residual_ck": 12 * nnz + 4 * (n + 1) + 8 * n + 8 * n + 8 * n + 16 * nblk,
        # b at the edge DoFs + dq, chain T / It / Ib written, junction slots (b, D, J, A, B
        # and their static indices: ~64 B each), chain statics (edge, flip: 8 B)
        "k_pc_up_lds": 8 * n_e + dq + 24 * E + 8 * E + 64 * B,
        # b at the edge DoFs + dq read, x written (edge DoFs + multipliers), chain and slot
        # statics (up, lo, edge, flip: 16 B; A, B, parent, lambda: 24 B)
        "k_pc_down_lds": 8 * n_e + dq + 8 * n + 16 * E + 24 * B,
        "k_pc_top_lds": 64 * 1024,  # <= 1024 junctions above the cut
        # values + rhs written, dq written, edge inputs read (edge_x 48, R, bc 16, lm 8, seg 4)
        "k_assemble_seg": 8 * nnz + 8 * n + dq + 80 * E,
    }


def dstep_bytes(n: int, nnz: int, E: int, N: int, B: int, nnz_lm: int) -> int:
    """Algorithmic bytes of one k_dir_step launch (the whole one-rank direct step, DESIGN.md
    section 3c): the edge inputs (80 B per edge, as the assembly kernel), the chain statics
    (edge, flip, up, lo in phase 1; up, lo and two post slots in phase 2: 32 B per chain), the
    junction slots' statics (~88 B each), the multiplier rows' values read; written: the CSR
    values, rhs and x (the residual is formed in registers, not stored; since round 5 the
    lumped mass is not written either -- only a later MINRES or refinement pass reads it, and
    ensure_dq forms it then)."""
    return 8 * nnz + 16 * n + 80 * E + 32 * E + 88 * B + 8 * nnz_lm


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


def cpu_model() -> str:
    try:
        for line in Path("/proc/cpuinfo").read_text().splitlines():
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or "unknown"


def cgroup_cpus() -> int | None:
    """The CPUs this process's cgroup may use: ``cpu.max`` (v2) or ``cpu.cfs_quota_us`` /
    ``cpu.cfs_period_us`` (v1), rounded down (at least 1); None when unlimited or unknown."""
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            return max(1, int(int(q) // int(p)))
        return None
    except (OSError, ValueError):
        pass
    try:
        q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
        p = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
        return max(1, q // p) if q > 0 and p > 0 else None
    except (OSError, ValueError):
        return None


def cpu_baseline(mesh, asm, dof: int, budget_s: float):
    """The hot path on the host cores (rank 0, one GPU only), in legs:

    * ``port-direct`` / ``port``: ``oracle/nx_cpu.c`` -- OpenMP assembly in the device layout
      + the direct tree solve (the GPU default's algorithm) / MINRES with the same exact tree
      preconditioner, on all threads OpenMP is given (OMP_NUM_THREADS);
    * ``superlu``: the oracle's numpy assembly of the reference forms + SuperLU ``spsolve``
      (1 thread; the stand-in for the reference's MUMPS direct solve).

    The direct port runs at the OpenMP default (``OMP_NUM_THREADS``) and, when it differs, at
    the CPU share the process's cgroup grants (``cpu.max`` quota / period: SURVEY 8d's "all
    host cores" this process may actually use -- the affinity mask names the whole shared
    host, 256 CPUs, and oversubscribing a 16-CPU share measured 1.3 s per step, noise); the
    headline ``value`` is the faster. The legs share ``budget_s`` equally."""
    from networks_fenicsx_amd.assembly import edge_boundary_rhs, evaluate_nodal
    from oracle import nx_cpu
    from oracle import nx_oracle as O

    legs = []
    lp = asm.local_problem
    bc = edge_boundary_rhs(mesh, lp.edges, evaluate_nodal(lambda x: x[1], mesh.node_coordinates))
    port = nx_cpu.CpuStep(lp, asm.tree_preconditioner, bc)
    port.assemble()
    port.solve()  # first touch of every buffer outside the timing
    omp = nx_cpu.threads()
    try:
        affinity = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        affinity = None
    quota = cgroup_cpus()
    share = min(x for x in (quota, affinity) if x) if (quota or affinity) else None
    runs_of = [(True, "port-direct", omp, "the direct tree solve (as the GPU's default)"),
               (False, "port", omp, "MINRES with the exact tree preconditioner")]
    if share and share != omp:  # every CPU this process may use
        runs_of.insert(1, (True, "port-direct-share", share,
                           "the direct tree solve, one thread per CPU of the process's "
                           "cgroup CPU share"))
    for direct, leg, threads, what in runs_of:
        nx_cpu.set_threads(threads)
        ms, runs, its = port.time_steps(budget_s / (len(runs_of) + 1), direct=direct)
        legs.append({"leg": leg, "ms_per_step": ms, "value": dof / (ms / 1e3), "cores": threads,
                     "iterations": its,
                     "sample": f"{runs} full steps of the same workload ({dof} DoF): OpenMP "
                               f"assembly + {what} (oracle/nx_cpu.c), {threads} threads"})
    nx_cpu.set_threads(omp)
    del port
    src, dst = mesh.edges
    P = O.build_problem(mesh.node_coordinates, src, dst, mesh.N, mesh.edge_colors)
    runs, t_total = 0, 0.0
    while runs < 1 or (t_total < budget_s / (len(runs_of) + 1) and runs < 40):
        t0 = time.perf_counter()
        A, b = O.assemble_reference(P, lambda x: x[1])
        O.solve_reference(A, b)
        t_total += time.perf_counter() - t0
        runs += 1
    ms1 = 1e3 * t_total / runs
    legs.append({"leg": "superlu", "ms_per_step": ms1, "value": dof / (ms1 / 1e3), "cores": 1,
                 "sample": f"{runs} full run(s) of the same workload: numpy assembly of the "
                           "reference forms + scipy SuperLU spsolve (1 thread, the MUMPS "
                           "stand-in)"})
    # the headline: the faster of the direct legs (the GPU default's algorithm) on the host
    head = max((g for g in legs if g["leg"].startswith("port-direct")), key=lambda g: g["value"])
    return {"value": head["value"], "unit": "DoF/s", "cores": head["cores"], "kind": "port",
            "ms_per_step": head["ms_per_step"], "sample": head["sample"],
            "cpu_model": cpu_model(), "os_cpu_count": os.cpu_count(),
            "affinity_cpus": affinity, "cgroup_cpus": quota,
            "omp_num_threads_env": os.environ.get("OMP_NUM_THREADS"),
            "cores_note": (f"direct legs at the OpenMP default ({omp} threads, from "
                           "OMP_NUM_THREADS) and, if different, at the cgroup CPU share "
                           f"({quota}; cpu.max quota / period); the headline is the faster; "
                           "os.cpu_count() and the affinity mask are the whole shared host"),
            "legs": legs}


C4_LEVELS, C4_N = 18, 19  # configs[4]: the depth-17 tree, N = 19, 10,354,648 DoF


def c4_leg(args, world: int, rank: int, comm, timed_steps, state, allsum):
    """configs[4] (``make_tree(18,18,18)``, N = 19) on the same GPUs as the headline, timed
    the same way (assemble + the direct solve, ``args.steps`` steps after ``args.warmup``;
    at P > 1 the exchange step, one launch per rank), with its error against the analytic
    answer. A fixed-size workload: over the driver's 1, 2, 4, 8-GPU runs it is the strong
    scaling of SURVEY's C4 (``north_star``: >= 6x from 1 to 8 GPUs)."""
    import numpy as np

    from networks_fenicsx_amd import HydraulicNetworkAssembler, NetworkMesh
    from networks_fenicsx_amd import network_generation as ng
    from oracle import nx_oracle as O

    t0 = time.perf_counter()
    G = ng.make_tree(C4_LEVELS, C4_LEVELS, C4_LEVELS) if rank == 0 else None
    mesh = NetworkMesh(G, N=C4_N, color_strategy="smallest_last", comm=comm)
    del G
    asm = HydraulicNetworkAssembler(mesh)
    asm.compute_forms(p_bc_ex=lambda x: x[1])
    asm.set_direct(True)
    setup = time.perf_counter() - t0
    h = asm.handle
    try:
        el = timed_steps(h, args.steps, args.warmup, world > 1)
        ms = 1e3 * el / args.steps
        E, B = mesh.num_edges, len(mesh.bifurcation_values)
        dof = E * (2 * C4_N + 1) + B
        out = {"workload": f"make_tree({C4_LEVELS},{C4_LEVELS},{C4_LEVELS}) depth-{C4_LEVELS - 1} "
                           f"binary tree, N={C4_N} (configs[4]), assemble + solve",
               "dofs": dof, "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
               "ms_per_step": ms, "value": dof / (ms / 1e3), "unit": "DoF/s",
               "solver": "direct" if h.solver()[1] == 1 else "minres",
               "direct_path": h.direct_path(), "relres": state["relres"],
               "iterations": state["it"], "setup_s": setup}
        src, dst = mesh.edges
        P = O.build_problem(mesh.node_coordinates, src, dst, mesh.N)
        xa = O.resistor_network_solution(P, lambda x: x[1])[O.build_permutation(P)[0]]
        lp = asm.local_problem
        per = 2 * C4_N + 1
        rows = np.concatenate([(lp.edges[:, None] * per + np.arange(per)[None, :]).ravel(),
                               E * per + mesh.bifurcation_index[lp.lm_nodes]])
        x = h.solution()
        d2, r2 = allsum([float(np.sum((x - xa[rows]) ** 2)), float(np.sum(xa[rows] ** 2))])
        out["relerr_vs_analytic"] = math.sqrt(d2 / r2)
        return out
    finally:
        asm.close()


# the committed rocprofv3 passes (kernel trace + FETCH_SIZE / WRITE_SIZE) of the (2, 1)
# direct step on this leg's workload (scripts/fe_timing.py 15 15 "2,1" direct)
FE21_PROFILE = "r06zm"


def summary_kernel(tag: str, prefix: str):
    """(calls, avg ns, HBM bytes per launch) of a kernel in profiles/<tag>_summary.json."""
    path = REPO / "profiles" / f"{tag}_summary.json"
    if not path.exists():
        return None
    for name, d in json.loads(path.read_text()).get("kernels", {}).items():
        if name == prefix or name.startswith(prefix + "<"):
            return d.get("calls"), d.get("avg_ns"), d.get("hbm_bytes_per_launch")
    return None


def fe21_kernels(h, N: int, E: int, nn: int) -> dict:
    """Continuous pressure (2, 1): every kernel of the direct step with its algorithmic bytes
    per step (what it must read and write once: CSR values and rhs, b, x, cell lengths, the
    per-vertex factors, the node records, blocks and pivots), the rocprof average and the
    PMC traffic from the committed passes on this workload (FE21_PROFILE), and the HBM
    fraction. Launches per step: one each, the node forest four (two per direction)."""
    per = 2 * N + 1 + N - 1
    n, nnz = h.n_rows, h.nnz
    alg = {
        "k_fe_tasm": 8 * nnz + 8 * n + 8 * E * N + 32 * E,
        "k_cp_edge": 8 * E * per + 8 * E * N + 24 * E + 8 * 14 * E * (N + 1) + 8 * 20 * E,
        "k_cp_nodes_rec": nn * 256 + 144 * E + nn * 160,
        "k_cp_back": 8 * 14 * E * (N + 1) + 8 * E * per + 8 * E * N + 48 * E + 8 * E * per
                     + 16 * nn,
        "k_fe_tres": 3 * 8 * n + 8 * E * N + 32 * E,
    }
    launches = {"k_cp_nodes_rec": 4}
    out = {}
    for k, b in alg.items():
        got = summary_kernel(FE21_PROFILE, k)
        if not got:
            out[k] = {"algorithmic_bytes_per_step": b}
            continue
        calls, avg_ns, traffic = got
        nl = launches.get(k, 1)
        t = (avg_ns or 0.0) * nl * 1e-9
        ach = b / t / 1e9 if t > 0 else None
        out[k] = {"algorithmic_bytes_per_step": b, "launches_per_step": nl,
                  "rocprof_us_per_step": t * 1e6, "achieved_GBs": ach,
                  "frac": ach / HBM_PEAK_GBS if ach else None,
                  "traffic_bytes_per_step": traffic * nl if traffic else None,
                  "traffic_ratio": traffic * nl / b if traffic else None,
                  "source": f"profiles/{FE21_PROFILE}_summary.json"}
    return out


# the committed bench profile whose MINRES legs ran this workload (the preconditioner's
# MINRES-mode sweeps, k_mr_a): profiles/r06u_*
MINRES_PROFILE = "r06u"


def minres_sweep_kernels(n: int, E: int, N: int, B: int) -> dict:
    """The preconditioner's sweeps in MINRES mode (P^{-1} r' per iteration, mode 0) with
    their algorithmic bytes per launch -- up: y and r2 at the edge DoFs read, y' = y - c r2
    written back, the lumped mass read, the chains' T / It / Ib written, the slots' y, r2 and
    statics; down: y at the edge DoFs and the lumped mass read, z written, the chain and slot
    statics -- beside the rocprof average and the PMC traffic of MINRES_PROFILE's passes."""
    n_e = E * (2 * N + 1)
    dq = 8 * E * (N + 1)
    alg = {"k_pc_up_lds<false, 8, 2>": 24 * n_e + dq + 32 * E + 80 * B,
           "k_pc_down_lds<false, 8, 2, false>": 8 * n_e + dq + 8 * n + 16 * E + 32 * B}
    out = {}
    for k, b in alg.items():
        got = summary_kernel(MINRES_PROFILE, k)
        if not got:
            out[k] = {"algorithmic_bytes_per_launch": b}
            continue
        calls, avg_ns, traffic = got
        t = (avg_ns or 0.0) * 1e-9
        ach = b / t / 1e9 if t > 0 else None
        out[k] = {"algorithmic_bytes_per_launch": b, "rocprof_avg_launch_ms": t * 1e3,
                  "achieved_GBs": ach, "frac": ach / HBM_PEAK_GBS if ach else None,
                  "traffic": traffic, "traffic_ratio": traffic / b if traffic else None,
                  "source": f"profiles/{MINRES_PROFILE}_summary.json (its calls average the "
                            "iterations' launches with the start's)"}
    return out


def fe_leg(mesh, steps: int = 20, warmup: int = 5) -> dict:
    """General element degrees on the headline tree (one GPU, reported beside the headline):
    (2, 0) through the condensed direct solve and (2, 1) through the node-condensed one,
    assemble + solve timed like the headline (``nx_assemble`` + ``nx_solve`` per step)."""
    from networks_fenicsx_amd import HydraulicNetworkAssembler

    out = {}
    for k, m in ((2, 0), (2, 1)):
        key = f"k{k}_m{m}"
        try:
            t0 = time.perf_counter()
            asm = HydraulicNetworkAssembler(mesh, flux_degree=k, pressure_degree=m)
            asm.compute_forms(p_bc_ex=lambda x: x[1])
            asm.set_direct(True)
            setup = time.perf_counter() - t0
            h = asm.handle
            try:
                res = None
                for _ in range(warmup):
                    asm.assemble()
                    res = h.solve(1e-12, 50000, 32)
                h.sync()
                ts = time.perf_counter()
                for _ in range(steps):
                    asm.assemble()
                    res = h.solve(1e-12, 50000, 32)
                h.sync()
                ms = 1e3 * (time.perf_counter() - ts) / steps
                out[key] = {"rows": h.n_rows, "ms_per_step": ms, "steps": steps,
                            "solver": "direct" if h.solver()[1] == 1 else "minres",
                            "direct_path": h.direct_path(), "passes": res[0],
                            "relres": res[1], "converged": res[2], "setup_s": setup}
                if (k, m) == (2, 1):
                    out[key]["kernels"] = fe21_kernels(h, mesh.N, mesh.num_edges,
                                                       len(mesh.node_coordinates))
            finally:
                asm.close()
        except Exception as e:  # (reported, never fatal to the headline)
            out[key] = {"error": f"{type(e).__name__}: {e}"}
    return out


def fe_leg_ranks(mesh, world: int, barrier, allmax, steps: int = 10, warmup: int = 3) -> dict:
    """``--fe-ranks``: the general-degree direct solves on the bench's ranks (RCCL at P > 1:
    (2, 0)'s condensed solve -- its auxiliary handle's team tree solve --, (2, 1)'s
    node-condensed one with its all-reduce of the border blocks), timed like the headline,
    with every rank's path, convergence and reported residual; the ranks must report the same
    residual bits (one all-reduce of its sums). Opt-in: a rank that failed inside one of its
    collectives would leave the others waiting in RCCL (no timeout), and the headline's JSON
    line must come out; the host-transport tests cover the same code on one GPU
    (tests/test_gpu_fe_ranks.py)."""
    from networks_fenicsx_amd import HydraulicNetworkAssembler

    out = {}
    for k, m in ((2, 0), (2, 1)):
        key = f"k{k}_m{m}"
        asm = HydraulicNetworkAssembler(mesh, flux_degree=k, pressure_degree=m)
        try:
            asm.compute_forms(p_bc_ex=lambda x: x[1])
            asm.set_direct(True)
            h = asm.handle
            res = None
            for _ in range(warmup):
                asm.assemble()
                res = h.solve(1e-12, 50000, 32)
            h.sync()
            barrier()
            ts = time.perf_counter()
            for _ in range(steps):
                asm.assemble()
                res = h.solve(1e-12, 50000, 32)
            h.sync()
            barrier()
            ms = allmax(1e3 * (time.perf_counter() - ts) / steps)
            rr = float(res[1])
            out[key] = {"ranks": world, "rows_max_per_rank": allmax(h.n_rows), "ms_per_step": ms,
                        "steps": steps, "direct_path": h.direct_path(),
                        "solver": "direct" if h.solver()[1] == 1 else "minres",
                        "passes": res[0], "relres": rr, "converged": bool(res[2]),
                        "all_ranks_direct": allmax(0.0 if h.solver()[1] == 1 else 1.0) == 0.0,
                        "relres_equal_on_ranks": allmax(rr) == -allmax(-rr)}
        finally:
            asm.close()
    return out


def _free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return int(s.getsockname()[1])


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # defaults: ~7 ms timed at C3 after ~4 ms of warm-up (the GPU idles through the host
    # set-up; a few warm-up steps leave the first timed ones slow)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=50)
    ap.add_argument("--levels", type=int, default=None,
                    help="tree generations (default: 15 at 1 GPU, 15 + log2(P) at P GPUs)")
    ap.add_argument("--N", type=int, default=None,
                    help="cells per edge (default 15 at every GPU count; 19: C4 at 8 GPUs)")
    ap.add_argument("--rtol", type=float, default=1e-12)
    ap.add_argument("--check-every", type=int, default=4)
    ap.add_argument("--cpu-budget", type=float, default=20.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-strong", action="store_true",
                    help="P > 1: skip rank 0's one-GPU time of the same workload")
    ap.add_argument("--api-steps", type=int, default=200,
                    help="steps through the public Solver.assemble/solve surface (0: skip)")
    ap.add_argument("--no-pc", action="store_true", help="plain (unpreconditioned) MINRES")
    ap.add_argument("--fe-ranks", action="store_true",
                    help="at P > 1 also the general-degree direct solves over the ranks "
                         "(RCCL; opt-in, see fe_leg_ranks)")
    ap.add_argument("--no-fe", dest="fe", action="store_false",
                    help="skip the general-degree leg ((2, 0) and (2, 1) on the headline tree)")
    ap.add_argument("--no-c4", dest="c4", action="store_false",
                    help="skip the configs[4] leg (C4, make_tree(18), N = 19, on these GPUs)")
    ap.add_argument("--solver", choices=("direct", "minres"), default="direct",
                    help="the direct tree solve (reference default preonly + lu) or MINRES")
    ap.add_argument("--allow-fallback", action="store_true",
                    help="report a run whose direct solve fell back to MINRES instead of "
                         "failing (exit status 3)")
    return ap.parse_args(argv)


def main() -> int:
    args = parse_args()
    world_env = os.environ.get("WORLD_SIZE")
    if world_env is None and args.gpus > 1:
        # one process per GPU: start the launcher as a child (nothing has touched the GPU)
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
               f"--nproc-per-node={args.gpus}", "--master-addr", "127.0.0.1",
               "--master-port", str(_free_port()), str(Path(__file__).resolve()), *sys.argv[1:]]
        return subprocess.call(cmd)
    world = int(world_env or "1")
    if world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}; refusing to measure a "
              "different configuration", file=sys.stderr)
        return 2
    return run(args, world)


def run(args, world: int) -> int:
    # torch first: libnxhip.so binds to torch's HIP runtime / RCCL (networks_fenicsx_amd._lib)
    import numpy as np
    import torch
    import torch.distributed as dist

    from networks_fenicsx_amd import _lib

    _lib.lib()
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        dist.init_process_group("gloo", rank=rank, world_size=world)
    # (ranks beyond the visible GPUs share them: a one-GPU rehearsal of the multi-rank path
    # with NXHIP_TRANSPORT=host; the driver's runs give every rank its own GPU)
    torch.cuda.set_device(local_rank % max(1, torch.cuda.device_count()))

    from networks_fenicsx_amd import HydraulicNetworkAssembler, NetworkMesh, Solver
    from networks_fenicsx_amd import network_generation as ng
    from networks_fenicsx_amd.comm import SerialComm, TorchComm

    extra = int(round(math.log2(world))) if world > 1 else 0
    if world > 1 and 2**extra != world:
        raise SystemExit("world size must be a power of two")
    levels = args.levels if args.levels is not None else 15 + extra
    N = args.N if args.N is not None else 15  # (the one-GPU load on every GPU: weak scaling)
    comm = TorchComm() if world > 1 else SerialComm()

    def barrier():
        if world > 1:
            dist.barrier()

    def allmax(v: float) -> float:
        if world == 1:
            return v
        t = torch.tensor([v], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    def allsum(vals):
        if world == 1:
            return list(vals)
        t = torch.tensor(list(vals), dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        return t.tolist()

    # ---- setup (host: graph, topology, layout, preconditioner decomposition; device:
    # pattern, coefficient upload) -- reported, not part of the step
    barrier()
    t0 = time.perf_counter()
    G = ng.make_tree(levels, levels, levels) if rank == 0 else None
    t_graph = time.perf_counter() - t0
    mesh = NetworkMesh(G, N=N, color_strategy="smallest_last", comm=comm)
    del G
    t_mesh = time.perf_counter() - t0 - t_graph
    asm = HydraulicNetworkAssembler(mesh)
    t_asm = time.perf_counter() - t0 - t_graph - t_mesh
    asm.compute_forms(p_bc_ex=lambda x: x[1])
    if args.no_pc:
        asm.set_preconditioner(False)
    torch.cuda.synchronize()
    setup = {"total": time.perf_counter() - t0, "graph": t_graph, "mesh": t_mesh,
             "assembler": t_asm}
    setup["forms"] = setup["total"] - t_graph - t_mesh - t_asm
    setup = {k: allmax(v) for k, v in setup.items()}
    h = asm.handle
    E, B = mesh.num_edges, len(mesh.bifurcation_values)
    dof_total = E * (2 * N + 1) + B
    state = {}

    def step(hd):
        hd.assemble(True, True)
        it, rr, conv = hd.solve(args.rtol, 50000, args.check_every)
        state["it"], state["relres"], state["conv"] = it, rr, conv

    def timed_steps(hd, steps, warmup, collective):
        for _ in range(warmup):
            step(hd)
        if collective:
            barrier()
        torch.cuda.synchronize()
        ts = time.perf_counter()
        for _ in range(steps):
            step(hd)
        hd.sync()
        torch.cuda.synchronize()
        if collective:
            barrier()
        el = time.perf_counter() - ts
        return allmax(el) if collective else el

    pc_on = asm.preconditioned
    direct = args.solver == "direct" and pc_on
    asm.set_direct(direct)
    elapsed = timed_steps(h, args.steps, args.warmup, True)
    ms_per_step = 1e3 * elapsed / args.steps
    iters = state["it"]
    solver_used = "direct" if h.solver()[1] == 1 else "minres"
    # every rank's path and exchange status after the timed steps (one all-reduce of a row
    # per rank): the driver's scaling run shows which ranks ran the exchange step
    rank_status = None
    if world > 1:
        codes = {"fused": 1, "condensed": 2, "exchange": 3, "node-condensed": 4, "launches": 5}
        xs = h.xr_status()
        row = [0.0] * (5 * world)
        row[5 * rank:5 * rank + 5] = [codes.get(h.direct_path(), 0) if solver_used == "direct"
                                      else 0, float(xs["off"]), xs["why"], xs["agreed"],
                                      xs["tag"]]
        got = allsum(row)
        names = {v: k for k, v in codes.items()}
        rank_status = [{"rank": r, "path": names.get(int(got[5 * r]), "minres"),
                        "xr_off": bool(got[5 * r + 1]), "xr_why": int(got[5 * r + 2]),
                        "xr_agreed": int(got[5 * r + 3]), "xr_tag": int(got[5 * r + 4])}
                       for r in range(world)]
    if direct and solver_used != "direct" and not args.allow_fallback:
        # the ranks decide together (schedule signature), so every rank stops here
        print(f"bench.py: rank {rank}: the direct solve was requested but the ranks ran "
              "MINRES (a rank's decomposition cannot run it exactly); --allow-fallback "
              "measures the fallback", file=sys.stderr, flush=True)
        return 3
    # the committed PMC summaries profile the default workload (C3) on one GPU only
    default_workload = world == 1 and (levels, N) == (15, 15) and not args.no_pc

    def minres_roofline():
        """k_mr_a: HIP events bound to its dispatches over PROF_STEPS profiled MINRES steps
        (after a warm one)."""
        h.set_profiling(True)
        step(h)
        h.reset_profile()
        for _ in range(PROF_STEPS):
            step(h)
        prof = h.profile()
        h.set_profiling(False)
        spmv_ms = prof["spmv_ms"] / max(prof["spmv_count"], 1)
        nbytes = mr_spmv_bytes(h.n_rows, h.nnz, pc_on,
                               max(int(prof["spmv_count"]) // PROF_STEPS, 1))
        # beta^2 travels point-to-point with the halo, so the multi-rank k_mr_a is MULTI = false
        kname = f"k_mr_a<false, {str(pc_on).lower()}>"
        traffic, tsrc, rocprof_ns = (pmc_traffic(kname) if default_workload
                                     else (None, None, None))
        achieved = nbytes / (spmv_ms * 1e-3) / 1e9
        return {"bound": "hbm",
                "kernel": f"{kname} (CSR SpMV fused with the Lanczos step, Givens rotation "
                          "and solution update)",
                "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                "traffic_unit": "bytes per launch (2 x FETCH_SIZE + WRITE_SIZE, gfx950-corrected)",
                "traffic_source": tsrc,
                "rocprof_avg_launch_ms": rocprof_ns / 1e6 if rocprof_ns else None,
                "algorithmic_bytes_per_launch": nbytes, "avg_launch_ms": spmv_ms,
                "assembly_kernel_ms": prof["asm_ms"] / max(prof["asm_count"], 1),
                "sweeps": (minres_sweep_kernels(h.n_rows, E, N, B) if default_workload and pc_on
                           else None)}

    def direct_roofline():
        """The direct solve's kernels (events bound to each dispatch, PROF_STEPS profiled
        steps after a warm one): the dominant one by time is the roofline kernel; all are
        listed."""
        h.set_profiling(True)
        step(h)  # the first profiled step runs cold (~1.5x); not averaged
        h.reset_profile()
        for _ in range(PROF_STEPS):
            step(h)
        pd = h.profile_direct()
        prof = h.profile()
        path = h.direct_path()
        h.set_profiling(False)
        cnt = max(pd["count"], 1)
        n, nnz = h.n_rows, h.nnz
        if path in ("fused", "exchange") and pd["up_ms"] > 0:
            # one launch per step (per rank): k_dir_step, or k_dir_xr with the ranks'
            # exchanges inside (its time is pd's first slot)
            t = pd["up_ms"] / cnt
            kb = dstep_bytes(n, nnz, E, N, B, (nnz - E * (7 * N + 1)) // 2)
            ach = kb / (t * 1e-3) / 1e9
            kname = "k_dir_step" if path == "fused" else "k_dir_xr"
            # (round 6: phase 2 by superposition is its own instantiation, <8, 2, true>)
            rocname = f"{kname}<8, 2{', true' if h.direct_sup() else ''}>"
            traffic, tsrc, rocprof_ns = (pmc_traffic(rocname) if default_workload
                                         else (None, None, None))
            k = {"avg_launch_ms": t, "algorithmic_bytes_per_launch": kb, "achieved_GBs": ach,
                 "frac": ach / HBM_PEAK_GBS, "traffic": traffic,
                 "traffic_ratio": traffic / kb if traffic else None}
            what = ("the whole direct step in one launch: assembly, up sweep, top part, down "
                    "sweep, fused residual check, published state; latency-bound"
                    if path == "fused" else
                    "one rank's whole direct step in one launch, the coarse partials and the "
                    "residual exchanged with the other ranks' kernels through peer-mapped "
                    "mailboxes; latency-bound")
            return {"bound": "hbm",
                    "kernel": f"{rocname} ({what})",
                    "achieved": ach, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": ach / HBM_PEAK_GBS, "traffic": traffic,
                    "traffic_unit": "bytes per launch (2 x FETCH_SIZE + WRITE_SIZE, gfx950-corrected)",
                    "traffic_source": tsrc,
                    "rocprof_avg_launch_ms": rocprof_ns / 1e6 if rocprof_ns else None,
                    "algorithmic_bytes_per_launch": kb, "avg_launch_ms": t,
                    "kernels": {kname: k}, "assembly_kernel_ms": None,
                    "direct_path": path}
        n_e = E * (2 * N + 1)
        nblk = -(-n // (256 * res_chunks(n)))  # k_residual_ck blocks (partials)
        info = h.direct_info()
        fused = info["fused_residual"]
        rname = "k_dir_publish_fr" if fused else "k_residual_ck"
        kb = direct_kernel_bytes(n, nnz, n_e, E, N, B, nblk, fused=fused,
                                 n_jobs=asm.tree_preconditioner.n_jobs, n_left=info["n_left"])
        ms = {rname: pd["residual_ms"] / cnt, "k_pc_up_lds": pd["up_ms"] / cnt,
              "k_pc_top_lds": pd["top_ms"] / cnt, "k_pc_down_lds": pd["down_ms"] / cnt,
              "k_assemble_seg": prof["asm_ms"] / max(prof["asm_count"], 1)}
        kernels = {}
        for k, t in ms.items():
            if t > 0:
                ach = kb[k] / (t * 1e-3) / 1e9
                kernels[k] = {"avg_launch_ms": t, "algorithmic_bytes_per_launch": kb[k],
                              "achieved_GBs": ach, "frac": ach / HBM_PEAK_GBS}
        if not kernels:  # nothing timed (several ranks replay one captured graph)
            return {"bound": "hbm", "kernel": None, "achieved": None, "peak": HBM_PEAK_GBS,
                    "unit": "GB/s", "frac": None, "traffic": None, "kernels": {},
                    "note": "no per-dispatch events in the captured multi-rank graph"}
        dom = max(kernels, key=lambda k: kernels[k]["avg_launch_ms"])
        d = kernels[dom]
        rocnames = {"k_residual_ck": "k_residual_ck", "k_dir_publish_fr": "k_dir_publish_fr",
                    "k_pc_up_lds": "k_pc_up_lds<false, 8, 2>",
                    "k_pc_down_lds": "k_pc_down_lds<false, 8, 2, true>",
                    "k_pc_top_lds": "k_pc_top_lds<false>",
                    "k_assemble_seg": "k_assemble_seg<16>"}
        for k, v in kernels.items():  # every kernel's counter bytes and their ratio
            tr = pmc_traffic(rocnames.get(k, k))[0] if default_workload else None
            v["traffic"] = tr
            v["traffic_ratio"] = tr / v["algorithmic_bytes_per_launch"] if tr else None
        names = {"k_residual_ck": "k_residual_ck (CSR SpMV r = b - A x: the direct solve's "
                                  "true-residual check)",
                 "k_dir_publish_fr": "k_dir_publish_fr (the fused residual check's sums, the top "
                                     "part's multiplier rows, the published state)",
                 "k_pc_up_lds": "k_pc_up_lds<false, 8, 2> (direct mode: M^-1 b_q per chain, "
                                "chain condensation, junction elimination)",
                 "k_pc_down_lds": "k_pc_down_lds<false, 8, 2, true> (direct mode: the top "
                                  "part's solve in every workgroup, back-substitution, cells, "
                                  "conservative x_q, the fused residual)",
                 "k_pc_top_lds": "k_pc_top_lds<false> (junctions above the cut)",
                 "k_assemble_seg": "k_assemble_seg<16> (CSR values + rhs)"}
        # kernel names as scripts/summarize_profile.py writes them (short form)
        rocname = {"k_residual_ck": "k_residual_ck", "k_dir_publish_fr": "k_dir_publish_fr",
                   "k_pc_up_lds": "k_pc_up_lds<false, 8, 2>",
                   "k_pc_down_lds": "k_pc_down_lds<false, 8, 2, true>",
                   "k_pc_top_lds": "k_pc_top_lds<false>",
                   "k_assemble_seg": "k_assemble_seg<16>"}.get(dom, dom)
        traffic, tsrc, rocprof_ns = (pmc_traffic(rocname) if default_workload
                                     else (None, None, None))
        return {"bound": "hbm", "kernel": names.get(dom, dom),
                "achieved": d["achieved_GBs"], "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": d["frac"], "traffic": traffic,
                "traffic_unit": "bytes per launch (2 x FETCH_SIZE + WRITE_SIZE, gfx950-corrected)",
                "traffic_source": tsrc,
                "rocprof_avg_launch_ms": rocprof_ns / 1e6 if rocprof_ns else None,
                "algorithmic_bytes_per_launch": d["algorithmic_bytes_per_launch"],
                "avg_launch_ms": d["avg_launch_ms"], "kernels": kernels,
                "assembly_kernel_ms": ms["k_assemble_seg"], "direct_path": path}

    roof = direct_roofline() if solver_used == "direct" else minres_roofline()
    warm_spmv_ms = h.bench_spmv(200)
    cold_spmv_ms, cold_copies = h.bench_spmv_cold(120)
    sbytes = spmv_bytes(h.n_rows, h.nnz)
    roof.update({"spmv_algorithmic_bytes": sbytes,
                 "isolated_warm_spmv_ms": warm_spmv_ms,
                 "isolated_warm_spmv_GBs": sbytes / (warm_spmv_ms * 1e-3) / 1e9,
                 "isolated_cold_spmv_ms": cold_spmv_ms,
                 "isolated_cold_spmv_GBs": sbytes / (cold_spmv_ms * 1e-3) / 1e9,
                 "cold_rotation_copies": cold_copies})

    # --- the other single-GPU solver on the same workload (same steps, same clock)
    other = None
    if world == 1 and pc_on:
        asm.set_direct(solver_used != "direct")
        el2 = timed_steps(h, args.steps, args.warmup, False)
        used2 = "direct" if h.solver()[1] == 1 else "minres"
        other = {"solver": used2, "ms_per_step": 1e3 * el2 / args.steps,
                 "value": dof_total / (el2 / args.steps), "iterations": state["it"],
                 "relres": state["relres"]}
        if used2 == "minres":
            other["roofline"] = minres_roofline()
        asm.set_direct(direct)
        step(h)  # leave the headline solver's solution in place for the parity check
        state["it"] = iters

    # --- the public surface: Solver.assemble() + Solver.solve() returning the Functions
    # (the reference's nxfx:Solver:solve includes the assign into Functions, solver.py:107-135)
    api_ms = api_host_ms = None
    if args.api_steps > 0:
        solver = Solver(asm)

        def api_loop(read: bool) -> float:
            solver.assemble()
            fns = solver.solve()
            if read:
                fns[0].x.array  # noqa: B018 - one DMA fills every function of the solve
            barrier()
            ts = time.perf_counter()
            for _ in range(args.api_steps):
                solver.assemble()
                fns = solver.solve()
                if read:
                    fns[0].x.array  # noqa: B018
            h.sync()
            barrier()
            el = allmax(time.perf_counter() - ts)
            del fns
            return 1e3 * el / args.api_steps

        # the functions hold a device snapshot until read (the default) / read every step
        api_ms = api_loop(False)
        api_host_ms = api_loop(True)
        del solver

    # --- parity outside the timed region: true residual and error vs the analytic answer
    from oracle import nx_oracle as O

    true_rr = h.true_residual()
    parity = {"true_relres": true_rr, "solver_relres": state["relres"], "converged": state["conv"]}
    src, dst = mesh.edges
    P = O.build_problem(mesh.node_coordinates, src, dst, mesh.N)
    xa = O.resistor_network_solution(P, lambda x: x[1])
    perm, _ = O.build_permutation(P)
    xa_b = xa[perm]  # build layout in global edge order
    lp = asm.local_problem
    per = 2 * N + 1
    rows = np.concatenate([(lp.edges[:, None] * per + np.arange(per)[None, :]).ravel(),
                           E * per + mesh.bifurcation_index[lp.lm_nodes]])
    x = h.solution()
    d2, r2 = allsum([float(np.sum((x - xa_b[rows]) ** 2)), float(np.sum(xa_b[rows] ** 2))])
    parity["relerr_vs_analytic"] = math.sqrt(d2 / r2)
    del xa, xa_b, P

    # --- rank 0 alone on the same workload (strong scaling T1), the others wait
    strong = None
    if world > 1 and not args.no_strong:
        barrier()
        if rank == 0:
            ts = time.perf_counter()
            asm1 = HydraulicNetworkAssembler(mesh.with_comm(None))
            asm1.compute_forms(p_bc_ex=lambda x: x[1])
            torch.cuda.synchronize()
            setup1 = time.perf_counter() - ts
            asm1.set_direct(False)
            el1 = timed_steps(asm1.handle, args.steps, args.warmup, False)
            t1 = 1e3 * el1 / args.steps
            it1 = state["it"]
            # the same tree by the direct tree solve on one GPU
            asm1.set_direct(True)
            el1d = timed_steps(asm1.handle, args.steps, args.warmup, False)
            t1d = 1e3 * el1d / args.steps
            asm1.close()
            # speedup of the same solver (the headline's) from one GPU to P
            t1_same = t1d if solver_used == "direct" else t1
            strong = {"workload": "same tree, one GPU (rank 0)", "n_gpus": world,
                      "solver_tP": solver_used, "tP_ms_per_step": ms_per_step,
                      "t1_ms_per_step": t1_same, "speedup_t1_over_tP": t1_same / ms_per_step,
                      "t1_minres_ms_per_step": t1, "t1_minres_iterations": it1,
                      "t1_direct_ms_per_step": t1d, "t1_setup_s": setup1}
        barrier()

    # --- SURVEY's C4 (configs[4]: make_tree(18), N = 19, 10,354,648 DoF) on the same GPUs:
    # the fixed-size workload, so the driver's N = 1, 2, 4, 8 runs give its strong scaling
    c4 = None
    if args.c4 and (levels, N) != (C4_LEVELS, C4_N):
        c4 = c4_leg(args, world, rank, comm, timed_steps, state, allsum)

    fe = None
    if args.fe and world == 1 and (levels, N) == (15, 15):
        fe = fe_leg(mesh)
    elif args.fe_ranks and world > 1:
        fe = fe_leg_ranks(mesh, world, barrier, allmax)

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(mesh, asm, dof_total, args.cpu_budget)

    if rank == 0:
        out = {
            "metric": METRIC,
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
                            f"tree, N={N} cells/edge, assemble + solve ({solver_used}, "
                            f"rtol {args.rtol:g})",
                "dofs": dof_total,
                "nnz": E * (7 * N + 1) + 6 * B,
                "edges": E,
                "N": N,
                "solver": solver_used,
                "iterations": iters,
                "parallelism": f"edge-partition x{world}" if world > 1 else "single GPU",
                "rccl_ranks": h.comm_count() if world > 1 else None,
                "preconditioner": "tree Schur complement" if pc_on else "none",
            },
            "setup_s": setup,
            "rank_status": rank_status,
            "api_ms_per_step": api_ms,
            "api_host_ms_per_step": api_host_ms,
            "strong_scaling": strong,
            "c4": c4,
            "general_degrees": fe,
            "solver": solver_used,
            "roofline": roof,
            "other_solver": other,
            "cpu_baseline": cpu,
            "parity": parity,
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    asm.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
