"""``dolfinx.common`` subset: the timer registry of :mod:`networks_fenicsx_amd.timing`,
which carries the reference's ``nxfx:*`` timer names (``demos/demo_perf.py:85-150``)."""

from __future__ import annotations

import enum

from networks_fenicsx_amd.timing import Timer, list_timings as _list, reset_timings, timed, timing

__all__ = ["Timer", "TimingType", "list_timings", "reset_timings", "timed", "timing"]


class TimingType(enum.Enum):
    wall = 0
    user = 1
    system = 2


def list_timings(comm=None, types=None) -> None:
    """Print the timer table (``dolfinx.common.list_timings`` prints a summary table)."""
    del comm, types
    rows = sorted(_list().items())
    print(f"{'timer':60s} {'count':>7s} {'total [s]':>12s}")
    for name, (count, total) in rows:
        print(f"{name:60s} {count:7d} {total:12.6f}")
