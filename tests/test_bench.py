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
