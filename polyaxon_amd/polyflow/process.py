"""Python face of the native process supervisor (csrc/procmon.cpp)."""
from __future__ import annotations

import ctypes
import os
import signal
from typing import Dict, List, Optional, Sequence, Tuple

from polyaxon_amd.ops import _native


def _cstr_array(items: Sequence[str]):
    arr = (ctypes.c_char_p * (len(items) + 1))()
    arr[:-1] = [s.encode() for s in items]
    arr[-1] = None
    return arr


class ProcessMonitor:
    """Spawn replica processes (own process group, output appended to a log file) and wait for any exit."""

    def __init__(self):
        self._lib = _native.lib("plx_procmon")
        self._h = self._lib.plx_pm_create()
        if not self._h:
            raise OSError("plx_pm_create failed")

    def spawn(self, argv: List[str], env: Dict[str, str], cwd: Optional[str] = None,
              log_path: Optional[str] = None) -> int:
        if log_path:
            os.makedirs(os.path.dirname(os.path.abspath(log_path)), exist_ok=True)
        a = _cstr_array(argv)
        e = _cstr_array([f"{k}={v}" for k, v in env.items()])
        pid = ctypes.c_int(0)
        rc = self._lib.plx_pm_spawn(self._h, a, e, (cwd or "").encode(), (log_path or "").encode(),
                                    ctypes.byref(pid))
        if rc != 0:
            raise OSError(rc, f"spawn failed: {os.strerror(rc) if rc > 0 else rc}: {argv[0]}")
        return int(pid.value)

    def wait(self, timeout_s: Optional[float] = None) -> Optional[Tuple[int, int]]:
        """(pid, exit status) for one exited child; None on timeout or wake(). status < 0 = killed by -signal."""
        ms = -1 if timeout_s is None else max(0, int(timeout_s * 1000))
        pid, st = ctypes.c_int(0), ctypes.c_int(0)
        r = self._lib.plx_pm_wait(self._h, ms, ctypes.byref(pid), ctypes.byref(st))
        if r == 1:
            return int(pid.value), int(st.value)
        if r < 0:
            raise OSError(-r, os.strerror(-r))
        return None

    def wake(self) -> None:
        self._lib.plx_pm_wake(self._h)

    def signal(self, pid: int, sig: int = signal.SIGTERM, group: bool = True) -> bool:
        return self._lib.plx_pm_signal(self._h, pid, int(sig), int(group)) == 0

    def count(self) -> int:
        return int(self._lib.plx_pm_count(self._h))

    def close(self) -> None:
        if self._h:
            self._lib.plx_pm_destroy(self._h)
            self._h = None

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass
