#!/usr/bin/env python3
"""Summarise a scripts/profile.sh run into profiles/<tag>_*.

* ``<tag>_kernel_stats.csv``  -- rocprofv3 --kernel-trace --stats summary (copied)
* ``<tag>_summary.json``      -- per kernel: calls, average ns, and per-launch HBM
  traffic from the PMC passes, corrected as MI355X_MICROARCH.md §HBM prescribes:
  FETCH_SIZE and WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE reports half of the
  bytes of wide coalesced streaming reads, so read bytes = 2 * FETCH_SIZE * 1024
  (stated as an upper estimate for the gathered accesses, which are uncalibrated);
  write bytes = WRITE_SIZE * 1024.

Usage: python scripts/summarize_profile.py <tag> [gpurun_out/prof_<tag>]
"""

from __future__ import annotations

import collections
import csv
import json
import shutil
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent


def short(name: str) -> str:
    name = name.replace("(anonymous namespace)::", "")
    return name.split("(")[0].replace("void ", "").strip()


def main() -> None:
    tag = sys.argv[1]
    src = Path(sys.argv[2]) if len(sys.argv) > 2 else REPO / "gpurun_out" / f"prof_{tag}"
    out = REPO / "profiles"
    out.mkdir(exist_ok=True)
    stats = src / "trace" / "trace_kernel_stats.csv"
    shutil.copy(stats, out / f"{tag}_kernel_stats.csv")
    summary: dict[str, dict] = {}
    for r in csv.DictReader(open(stats)):
        summary[short(r["Name"])] = {"calls": int(r["Calls"]), "avg_ns": float(r["AverageNs"]),
                                     "total_pct": float(r["Percentage"])}
    for counter, sub in (("FETCH_SIZE", "pmc_fetch"), ("WRITE_SIZE", "pmc_write")):
        f = src / sub / "pmc_counter_collection.csv"
        if not f.exists():
            continue
        agg = collections.defaultdict(list)
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == counter:
                agg[short(r["Kernel_Name"])].append(float(r["Counter_Value"]))
        for k, v in agg.items():
            d = summary.setdefault(k, {})
            d[f"{counter}_KiB_avg"] = sum(v) / len(v)
            d[f"{counter}_launches"] = len(v)
    for k, d in summary.items():
        if "FETCH_SIZE_KiB_avg" in d and "WRITE_SIZE_KiB_avg" in d:
            d["hbm_read_bytes_per_launch"] = 2 * d["FETCH_SIZE_KiB_avg"] * 1024
            d["hbm_write_bytes_per_launch"] = d["WRITE_SIZE_KiB_avg"] * 1024
            d["hbm_bytes_per_launch"] = d["hbm_read_bytes_per_launch"] + d["hbm_write_bytes_per_launch"]
    doc = {"tag": tag, "source": str(src.relative_to(REPO)) if src.is_relative_to(REPO) else str(src),
           "correction": "read = 2 x FETCH_SIZE KiB (gfx950 half-count), write = WRITE_SIZE KiB",
           "kernels": summary}
    (out / f"{tag}_summary.json").write_text(json.dumps(doc, indent=1))
    for k, d in sorted(summary.items(), key=lambda kv: -kv[1].get("total_pct", 0))[:8]:
        print(f"{k:28s} calls={d.get('calls', 0):6d} avg={d.get('avg_ns', 0) / 1e3:8.2f} us "
              f"hbm={d.get('hbm_bytes_per_launch', 0) / 1e6:8.2f} MB")


if __name__ == "__main__":
    main()
