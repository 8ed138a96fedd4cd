"""roctx ranges around the trainer's phases (tracing).

Off unless DXRL_ROCTX=1: then PGTrainer.iteration() pushes one roctx range per phase
(rollout, critic_values, advantages, actor_train, ...), which `rocprofv3 --marker-trace`
shows on the host timeline next to the kernels each phase launched.  The ranges are
host-side markers (no GPU work, no synchronisation)."""
from __future__ import annotations

import contextlib
import ctypes
import os

_lib = None
_tried = False


def _roctx():
    global _lib, _tried
    if not _tried:
        _tried = True
        for name in ("librocprofiler-sdk-roctx.so.1", "libroctx64.so.4", "libroctx64.so"):
            try:
                lib = ctypes.CDLL(name)
                lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
                lib.roctxRangePushA.restype = ctypes.c_int
                lib.roctxRangePop.restype = ctypes.c_int
                _lib = lib
                break
            except OSError:
                continue
    return _lib


def enabled() -> bool:
    return os.environ.get("DXRL_ROCTX", "0") == "1" and _roctx() is not None


@contextlib.contextmanager
def range_(name: str):
    lib = _roctx() if enabled() else None
    if lib is None:
        yield
        return
    lib.roctxRangePushA(name.encode())
    try:
        yield
    finally:
        lib.roctxRangePop()
