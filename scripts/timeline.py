#!/usr/bin/env python3
"""Per-step GPU timeline from a rocprofv3 kernel trace (scripts/profile.sh output):
kernel start offsets, durations and the idle gaps between consecutive dispatches.

Usage: python scripts/timeline.py gpurun_out/prof_<tag>/trace/trace_kernel_trace.csv [anchor]
(anchor = the kernel that starts a step, default k_assemble; optional third argument:
the index of the anchor that starts the step to print)
"""

import csv
import sys


def short(name: str) -> str:
    return name.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0].strip()


def main() -> None:
    rows = list(csv.DictReader(open(sys.argv[1])))
    anchor = sys.argv[2] if len(sys.argv) > 2 else "k_assemble"
    ks = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]))
                 for r in rows), key=lambda t: t[0])
    starts = [i for i, k in enumerate(ks) if k[2] == anchor]
    # a full timed step: between the third- and second-to-last anchors (the last one is
    # the bench's profiled step)
    if len(sys.argv) > 3:  # explicit step index (the n-th anchor)
        k = int(sys.argv[3])
        i0, i1 = starts[k], starts[k + 1]
    else:
        i0, i1 = starts[-3], starts[-2]
    t0 = ks[i0][0]
    prev_end = t0
    busy = 0
    for s, e, n in ks[i0:i1]:
        print(f"{(s - t0) / 1e3:9.2f} us  +gap {(s - prev_end) / 1e3:6.2f}  "
              f"dur {(e - s) / 1e3:7.2f}  {n}")
        busy += e - s
        prev_end = e
    print(f"step span {(ks[i1][0] - t0) / 1e3:.2f} us, kernel busy {busy / 1e3:.2f} us")


if __name__ == "__main__":
    main()
