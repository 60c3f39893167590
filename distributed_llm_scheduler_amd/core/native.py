"""Loader for the native scheduling core (``_dlsched_core``).

The shared object is git-ignored (the history stays source-only), so a fresh checkout
builds it on first import (g++, ~15 s). Set ``DLS_NO_NATIVE=1`` to force the pure-Python
engine.
"""
from __future__ import annotations

import importlib
import os
import threading

_lock = threading.Lock()
_mod = None
_err = None


def load(build_if_missing: bool = True):
    """Return the ``_dlsched_core`` module, building it if needed; None if unavailable."""
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
        except Exception as e:  # pragma: no cover - reported through available()
            _err = e
            _mod = None
    return _mod


def available() -> bool:
    return load() is not None


def error():
    return _err
