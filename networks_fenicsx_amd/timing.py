"""Wall-clock timer registry with the reference's timer names.

The reference decorates its setup and hot-path functions with
``dolfinx.common.timed("nxfx:...")`` and reads them back with
``dolfinx.common.timing(name) -> (count, timedelta)``
(reference ``demos/demo_perf.py:85-150``; timer names at ``mesh.py:29,117,138,425``,
``assembly.py:28,120,164,328``, ``solver.py:107``, ``network_generation.py:41,157``).
This module keeps the same names and the same read-back shape so that
demo_perf-style scripts keep working without DOLFINx.

Device work is asynchronous: the decorated GPU entry points synchronise their
stream before returning, so the wall time recorded here covers the device work.
"""

from __future__ import annotations

import datetime
import functools
import threading
import time
from typing import Callable, TypeVar

__all__ = ["timed", "timing", "list_timings", "reset_timings", "Timer"]

_F = TypeVar("_F", bound=Callable)
_lock = threading.Lock()
_table: dict[str, list] = {}  # name -> [count, total_seconds]


def _record(name: str, seconds: float) -> None:
    with _lock:
        entry = _table.setdefault(name, [0, 0.0])
        entry[0] += 1
        entry[1] += seconds


class Timer:
    """Context manager that accumulates into the registry under ``name``."""

    def __init__(self, name: str):
        self.name = name
        self._t0 = 0.0
        self.elapsed = 0.0

    def __enter__(self) -> "Timer":
        self._t0 = time.perf_counter()
        return self

    def __exit__(self, *exc) -> None:
        self.elapsed = time.perf_counter() - self._t0
        _record(self.name, self.elapsed)


def timed(name: str) -> Callable[[_F], _F]:
    """Decorator: accumulate the wall time of every call under ``name``."""

    def deco(fn: _F) -> _F:
        @functools.wraps(fn)
        def wrapper(*args, **kwargs):
            t0 = time.perf_counter()
            try:
                return fn(*args, **kwargs)
            finally:
                _record(name, time.perf_counter() - t0)

        return wrapper  # type: ignore[return-value]

    return deco


def timing(name: str) -> tuple[int, datetime.timedelta]:
    """Return ``(count, total wall time)`` for ``name``; ``(0, 0)`` if never called."""
    with _lock:
        count, total = _table.get(name, [0, 0.0])
    return count, datetime.timedelta(seconds=total)


def list_timings() -> dict[str, tuple[int, float]]:
    with _lock:
        return {k: (v[0], v[1]) for k, v in _table.items()}


def reset_timings() -> None:
    with _lock:
        _table.clear()
