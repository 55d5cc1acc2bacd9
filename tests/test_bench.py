"""bench.py helpers that need no GPU: algorithmic byte models and the choice of the
committed PMC summary (profiles/<tag>_summary.json) the roofline's traffic comes from."""

import json

import bench


def test_spmv_bytes_c3():
    # 12 nnz + 4 (n + 1) + 16 n at C3 = 63.50 MB
    assert bench.spmv_bytes(1_032_160, 3_571_600) == 63_502_404


def test_profile_tags_order_by_suffix_length(tmp_path, monkeypatch):
    prof = tmp_path / "profiles"
    prof.mkdir()
    kname = "k_mr_a<false, true>"
    for i, tag in enumerate(["r01b", "r01y", "r01af", "r01z", "r01ab"]):
        doc = {"kernels": {kname: {"hbm_bytes_per_launch": float(i), "avg_ns": 1.0}}}
        (prof / f"{tag}_summary.json").write_text(json.dumps(doc))
    monkeypatch.setattr(bench, "REPO", tmp_path)
    traffic, src, _ = bench.pmc_traffic(kname)
    assert src == "profiles/r01af_summary.json" and traffic == 2.0
    (prof / "r02a_summary.json").write_text(
        json.dumps({"kernels": {kname: {"hbm_bytes_per_launch": 9.0}}}))
    assert bench.pmc_traffic(kname)[1] == "profiles/r02a_summary.json"


def test_committed_summary_has_the_bench_kernel():
    traffic, src, ns = bench.pmc_traffic("k_mr_a<false, true>")
    assert src is not None and traffic > 0 and ns > 0


def test_world_size_mismatch_refuses_to_measure():
    """WORLD_SIZE set by a launcher but different from --gpus: non-zero exit before any
    GPU work (bench.py would otherwise measure another configuration)."""
    import os
    import subprocess
    import sys
    from pathlib import Path

    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    res = subprocess.run([sys.executable, str(Path(bench.__file__)), "--gpus", "4"],
                         capture_output=True, text=True, env=env, timeout=120)
    assert res.returncode == 2
    assert "refusing" in res.stderr


def test_default_workloads():
    args = bench.parse_args([])
    assert args.gpus == 1 and args.levels is None and args.N is None


def test_direct_kernel_bytes_c3():
    """The residual SpMV of the direct solve reads the CSR, x and b once (SURVEY 8(d) + b)."""
    n, nnz, E, N, B = 1_032_160, 3_571_600, 32_767, 15, 16_383
    nblk = (n + 255) // 256
    kb = bench.direct_kernel_bytes(n, nnz, E * (2 * N + 1), E, N, B, nblk)
    assert kb["k_residual_ck"] == bench.spmv_bytes(n, nnz) + 8 * n + 16 * nblk  # + r stored
    assert set(kb) == {"k_residual_ck", "k_pc_up_lds", "k_pc_down_lds", "k_pc_top_lds",
                       "k_assemble_seg"}
    assert 13e6 < kb["k_pc_up_lds"] < 16e6 and 20e6 < kb["k_pc_down_lds"] < 23e6


def test_direct_kernel_bytes_fused_c3():
    """Fused residual check: no residual SpMV; the down sweep also reads the edge geometry and
    stores r (8 B per edge DoF and local multiplier), the publish step is small."""
    n, nnz, E, N, B = 1_032_160, 3_571_600, 32_767, 15, 16_383
    n_e = E * (2 * N + 1)
    plain = bench.direct_kernel_bytes(n, nnz, n_e, E, N, B, 1)
    kb = bench.direct_kernel_bytes(n, nnz, n_e, E, N, B, 1, fused=True, n_jobs=256, n_left=255)
    assert set(kb) == {"k_dir_publish_fr", "k_pc_up_lds", "k_pc_down_lds", "k_pc_top_lds",
                       "k_assemble_seg"}
    assert kb["k_pc_down_lds"] - plain["k_pc_down_lds"] == 56 * E + 8 * n_e + 8 * B
    assert kb["k_dir_publish_fr"] < 64 * 1024


def test_solver_option_defaults_to_direct():
    assert bench.parse_args([]).solver == "direct"
    assert bench.parse_args(["--solver", "minres"]).solver == "minres"
