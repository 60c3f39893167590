"""Loader for the native scheduling core (``_dlsched_core``).

The shared object is git-ignored (the history stays source-only), so a fresh checkout
builds it on first import (g++, ~15 s). A failed build or import RAISES: the native core is
the scheduling and memory-planning engine, and a silent fallback would hide a broken build
(the pure-Python engine then decides every placement). Set ``DLS_NO_NATIVE=1`` to run the
pure-Python engine on purpose.
"""
from __future__ import annotations

import importlib
import os
import threading

_lock = threading.Lock()
_mod = None
_err = None


class NativeCoreError(RuntimeError):
    pass


def load(build_if_missing: bool = True):
    """Return the ``_dlsched_core`` module, building it if needed; None only under
    ``DLS_NO_NATIVE=1``. Raises :class:`NativeCoreError` if it cannot be built or imported."""
    global _mod, _err
    if os.environ.get("DLS_NO_NATIVE") == "1":
        return None
    if _mod is not None:
        return _mod
    with _lock:
        if _mod is not None:
            return _mod
        try:
            from .. import _build
            if build_if_missing:
                _build.build_core()
            _mod = importlib.import_module("distributed_llm_scheduler_amd._dlsched_core")
        except Exception as e:  # pragma: no cover - a broken toolchain / library
            _err = e
            _mod = None
            raise NativeCoreError(f"native scheduling core unavailable ({e!r}); fix the build or set "
                                  "DLS_NO_NATIVE=1 to use the pure-Python engine") from e
    return _mod


def available() -> bool:
    return load() is not None


def error():
    return _err
