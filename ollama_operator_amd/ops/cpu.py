"""The CPU serving backend module (`ollama_operator_amd/_cpu`, csrc/cpu, built by build_native.py).

It has no HIP dependency, so a CPU-only node (BASELINE config 1, `image: phi` on kind) loads it
without the GPU extension. `OMX_CPU_THREADS` sets its OpenMP thread count (default: all cores)."""
from __future__ import annotations

import os

_MOD = None
_ERR: Exception | None = None


def cpu_module():
    """The `_cpu` module, or None when it is not built."""
    global _MOD, _ERR
    if _MOD is None and _ERR is None:
        try:
            from .. import _cpu  # type: ignore[attr-defined]
            n = int(os.environ.get("OMX_CPU_THREADS", "0") or 0)
            if n > 0:
                _cpu.set_threads(n)
            _MOD = _cpu
        except ImportError as e:  # pragma: no cover - depends on build state
            _ERR = e
    return _MOD
