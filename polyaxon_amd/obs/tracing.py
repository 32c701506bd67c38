"""roctx ranges: scheduler phases and trial phases show up as named ranges in
``rocprofv3 --marker-trace`` timelines next to the HIP kernels they enclose.

The ROCm tracer library (libroctx64) is loaded lazily with ctypes; without it (CPU hosts) every range is
a no-op.  ``trace_range`` is cheap enough for per-trial use (not per kernel).
"""
from __future__ import annotations

import contextlib
import ctypes
import ctypes.util
import os
import threading
import time
from typing import Dict, List, Optional

_lib = None
_tried = False
_lock = threading.Lock()
SPANS: List[Dict] = []  # in-process record (name, start, end) for tests / the API
_RECORD = os.environ.get("PLX_TRACE_RECORD", "0") == "1"


def _roctx():
    global _lib, _tried
    with _lock:
        if not _tried:
            _tried = True
            for name in ("/opt/rocm/lib/libroctx64.so", ctypes.util.find_library("roctx64") or ""):
                if name and os.path.exists(name):
                    try:
                        lib = ctypes.CDLL(name)
                        lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
                        lib.roctxRangePushA.restype = ctypes.c_int
                        lib.roctxRangePop.restype = ctypes.c_int
                        lib.roctxMarkA.argtypes = [ctypes.c_char_p]
                        _lib = lib
                        break
                    except OSError:
                        continue
    return _lib


@contextlib.contextmanager
def trace_range(name: str):
    lib = _roctx()
    t0 = time.perf_counter()
    if lib is not None:
        lib.roctxRangePushA(name.encode())
    try:
        yield
    finally:
        if lib is not None:
            lib.roctxRangePop()
        if _RECORD:
            SPANS.append({"name": name, "start": t0, "end": time.perf_counter()})


def mark(name: str) -> None:
    lib = _roctx()
    if lib is not None:
        lib.roctxMarkA(name.encode())


def available() -> bool:
    return _roctx() is not None
