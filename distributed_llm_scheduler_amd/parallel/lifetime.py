"""Deferred destruction of native GPU resources (hipGraphs, native step runners, hipMalloc'd
buffers).

Why: the single-GPU multi-rank harness (parallel/loopback.py) captures hipGraphs on several rank
threads of ONE process at once. Destroying a hipGraph / hipGraphExec, a runner's hipEvents or a
hipMalloc'd buffer while another thread of the process is inside a stream capture aborted the
process (round 4: an empty segment graph torn down mid-capture; round 5's driver GPU suite died
at the first 4-rank harness case with no summary line). Such a destruction can happen on ANY
thread at ANY time: the cyclic garbage collector runs on whichever thread allocates, and it
finalises executors left over from earlier tests.

The rule here: an owner (an executor, a device-transport world) registers its native objects
with :func:`keep`. They stay alive for as long as the owner does, even when the owner drops its
own reference (a re-capture replacing a graph, a runner rebuilt). When the owner dies — on
whatever thread — the objects move to a graveyard instead of being destroyed, and the
graveyard is emptied only by :func:`release`, which callers invoke at quiesce points on the
main thread (the harness before it starts its rank threads and after it has joined them, the
test suite between tests). :func:`quiesced` wraps a concurrent-capture section: it collects
garbage and empties the graveyard first, then pauses the cyclic collector until the section
ends.
"""
from __future__ import annotations

import contextlib
import gc
import threading
import weakref
from typing import List

_LOCK = threading.Lock()
_GRAVE: List[object] = []
_BUSY = 0  # > 0 while a concurrent-capture section runs (release() then does nothing)


def _bury(objs: list) -> None:
    """weakref.finalize callback of an owner: take over its native objects (no destruction)."""
    with _LOCK:
        _GRAVE.extend(objs)
    objs.clear()


def keep(owner, obj) -> object:
    """Keep ``obj`` alive until ``owner`` dies; then it goes to the graveyard. Returns ``obj``."""
    lst = owner.__dict__.get("_native_keep")
    if lst is None:
        lst = owner.__dict__["_native_keep"] = []
        weakref.finalize(owner, _bury, lst)
    lst.append(obj)
    return obj


def retire(owner) -> int:
    """The owner replaces its native objects (a re-capture, a rebuilt runner): move the ones kept
    so far to the graveyard — destroyed at the next :func:`release`, never here. The caller must
    not use them any more and must have synchronised with their last launches. Returns the
    count moved."""
    lst = owner.__dict__.get("_native_keep")
    if not lst:
        return 0
    with _LOCK:
        _GRAVE.extend(lst)
    n = len(lst)
    lst.clear()
    return n


def release_on_main_thread() -> int:
    """:func:`release` when called on the main thread (rank threads of the single-GPU harness
    capture inside :func:`quiesced`, where release is a no-op anyway): keeps a long-lived
    executor that re-captures many times (in-DAG tuning) from accumulating dead graphs."""
    if threading.current_thread() is not threading.main_thread():
        return 0
    return release()


def graveyard_size() -> int:
    with _LOCK:
        return len(_GRAVE)


def release() -> int:
    """Destroy the graveyard's objects (call only where no other thread of this process can be
    capturing a graph). Returns how many were released; 0 while a quiesced section runs."""
    if _BUSY:
        return 0
    with _LOCK:
        objs = list(_GRAVE)
        _GRAVE.clear()
    n = len(objs)
    del objs  # the last references: destructors run here, on the calling thread
    return n


@contextlib.contextmanager
def quiesced():
    """A section in which several threads may capture hipGraphs: garbage from before is
    collected and released HERE (on the calling thread), and the cyclic collector is paused
    until the section ends, so no finaliser of an unrelated object runs on a capturing thread."""
    global _BUSY
    gc.collect()
    release()
    was = gc.isenabled()
    gc.disable()
    with _LOCK:
        _BUSY += 1
    try:
        yield
    finally:
        with _LOCK:
            _BUSY -= 1
        if was:
            gc.enable()
