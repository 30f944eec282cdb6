"""roctx ranges around engine steps: `OMX_ROCTX=1` loads /opt/rocm/lib/libroctx64.so
and brackets prefill / decode / TP collectives so `rocprofv3 --marker-trace` (or --sys-trace) shows
them on the timeline next to the kernels. Off (zero-cost context manager) by default and on CPU.
The reference has no tracing at all."""
from __future__ import annotations

import contextlib
import ctypes
import os

_lib = None
_enabled = os.environ.get("OMX_ROCTX", "0") == "1"


def _load():
    global _lib, _enabled
    if _lib is not None or not _enabled:
        return _lib
    for name in ("libroctx64.so", os.path.join(os.environ.get("ROCM_PATH", "/opt/rocm"), "lib", "libroctx64.so")):
        try:
            _lib = ctypes.CDLL(name)
            _lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
            _lib.roctxRangePushA.restype = ctypes.c_int
            _lib.roctxRangePop.restype = ctypes.c_int
            _lib.roctxMarkA.argtypes = [ctypes.c_char_p]
            return _lib
        except OSError:
            continue
    _enabled = False
    return None


def enabled() -> bool:
    return _enabled and _load() is not None


@contextlib.contextmanager
def trace_range(name: str):
    lib = _load() if _enabled else None
    if lib is None:
        yield
        return
    lib.roctxRangePushA(name.encode())
    try:
        yield
    finally:
        lib.roctxRangePop()


def mark(name: str) -> None:
    lib = _load() if _enabled else None
    if lib is not None:
        lib.roctxMarkA(name.encode())
