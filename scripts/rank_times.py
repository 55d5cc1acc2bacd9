#!/usr/bin/env python3
"""Per-rank launch times of the multi-rank kernels from a rocprofv3 kernel trace of the
8-rank group rehearsal (scripts/rehearsal_profile.sh): the group launches each kernel
once per rank, back to back, so runs of P identical names are one launch per rank.

    python scripts/rank_times.py gpurun_out/prof_reh_b/trace_kernel_trace.csv [P]
"""
import csv
import re
import sys
from collections import defaultdict

import numpy as np

path = sys.argv[1]
P = int(sys.argv[2]) if len(sys.argv) > 2 else 8
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
ks = []
for r in rows:
    name = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "")
    ks.append((re.sub(r"\(.*", "", name),
               (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3))
runs = defaultdict(list)
i = 0
while i < len(ks):
    j = i
    while j < len(ks) and ks[j][0] == ks[i][0]:
        j += 1
    if j - i == P:
        runs[ks[i][0]].append([t for _, t in ks[i:j]])
    i = j
for name, rr in runs.items():
    a = np.array(rr[-9:])
    print(f"{name:34s} launches {len(rr):3d}  per-rank mean us: {np.round(a.mean(0), 1)}")
