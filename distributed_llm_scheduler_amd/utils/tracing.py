"""Tracing: roctx ranges per DAG node and Chrome-trace export of measured timelines.

The reference's only instrumentation is ``time.time()`` around ``schedule()``
(simulation.py:327-333) and its Gantt is synthetic (visu.py:206-248). Here:

* :class:`Roctx` — ``roctxRangePushA``/``roctxRangePop``/``roctxMarkA`` from ROCm's
  ``librocprofiler-sdk-roctx`` (ctypes, no-op when the library is absent). With
  ``DAGExecutor(trace=True)`` every load / send / recv / kernel group of a step is a
  named range, so ``rocprofv3 --marker-trace --kernel-trace`` attributes each HIP kernel
  to the DAG node that launched it.
* :func:`chrome_trace` — measured per-rank events (hipEvent-timed on GPU, host-timed on
  the CPU backend) written as Chrome ``about:tracing`` / Perfetto JSON: one process per
  rank, one thread row per stream class (compute, param H2D, p2p comm).
"""
from __future__ import annotations

import ctypes
import json
import os
from contextlib import contextmanager
from typing import Dict, Iterable, List, Optional, Sequence, Tuple

_LIBS = ("librocprofiler-sdk-roctx.so.1", "librocprofiler-sdk-roctx.so", "libroctx64.so.4", "libroctx64.so")


class Roctx:
    """Thin ctypes binding of the roctx range API (lazily loaded, process-wide)."""

    _lib = None
    _tried = False

    @classmethod
    def lib(cls):
        if not cls._tried:
            cls._tried = True
            if os.environ.get("DLS_NO_ROCTX"):
                return None
            roots = [os.environ.get("ROCM_PATH", "/opt/rocm")]
            for name in _LIBS:
                for cand in [name] + [os.path.join(r, "lib", name) for r in roots]:
                    try:
                        lib = ctypes.CDLL(cand)
                    except OSError:
                        continue
                    lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
                    lib.roctxRangePushA.restype = ctypes.c_int
                    lib.roctxRangePop.restype = ctypes.c_int
                    lib.roctxMarkA.argtypes = [ctypes.c_char_p]
                    cls._lib = lib
                    return lib
        return cls._lib

    @classmethod
    def available(cls) -> bool:
        return cls.lib() is not None

    @classmethod
    def push(cls, name: str) -> None:
        lib = cls.lib()
        if lib is not None:
            lib.roctxRangePushA(name.encode())

    @classmethod
    def pop(cls) -> None:
        lib = cls.lib()
        if lib is not None:
            lib.roctxRangePop()

    @classmethod
    def mark(cls, name: str) -> None:
        lib = cls.lib()
        if lib is not None:
            lib.roctxMarkA(name.encode())


@contextmanager
def roctx_range(name: str, enabled: bool = True):
    if enabled:
        Roctx.push(name)
    try:
        yield
    finally:
        if enabled:
            Roctx.pop()


# (name, category, start_ms, end_ms); category in {"kernel", "load", "send", "recv"}
Event = Tuple[str, str, float, float]
_TID = {"kernel": 0, "load": 1, "recv": 2, "send": 3}
_TNAME = {0: "compute stream (HIP kernels)", 1: "param fill (H2D)", 2: "p2p recv (RCCL)", 3: "p2p send (RCCL)"}


def chrome_trace(events_by_rank: Dict[int, Sequence[Event]], path: Optional[str] = None,
                 meta: Optional[dict] = None) -> dict:
    """Chrome-trace JSON (``traceEvents`` complete events, µs) of measured per-rank events."""
    out: List[dict] = []
    for rank, evs in sorted(events_by_rank.items()):
        out.append({"name": "process_name", "ph": "M", "pid": rank, "args": {"name": f"GPU {rank}"}})
        for tid, tname in _TNAME.items():
            out.append({"name": "thread_name", "ph": "M", "pid": rank, "tid": tid, "args": {"name": tname}})
        for name, cat, a, b in evs:
            out.append({"name": name, "cat": cat, "ph": "X", "pid": rank, "tid": _TID.get(cat, 0),
                        "ts": round(a * 1e3, 3), "dur": round(max(b - a, 0.0) * 1e3, 3)})
    doc = {"traceEvents": out, "displayTimeUnit": "ms", "otherData": dict(meta or {})}
    if path:
        d = os.path.dirname(path)
        if d:
            os.makedirs(d, exist_ok=True)
        with open(path, "w") as f:
            json.dump(doc, f)
    return doc


def kernel_timeline(events: Iterable[Event]) -> List[Tuple[str, float, float]]:
    """The (task, start, end) kernel rows of an event list (what ``measured_gantt`` draws)."""
    return [(n, a, b) for n, c, a, b in events if c == "kernel"]


def summarize(events: Iterable[Event]) -> Dict[str, float]:
    """Busy time per category and the step span (ms)."""
    tot: Dict[str, float] = {}
    lo, hi = float("inf"), 0.0
    for _, c, a, b in events:
        tot[c] = tot.get(c, 0.0) + (b - a)
        lo, hi = min(lo, a), max(hi, b)
    tot["span"] = (hi - lo) if hi >= lo else 0.0
    return tot
