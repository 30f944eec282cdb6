"""Access to the native core (`ollama_operator_amd/_C`, built by `build_native.py`).

torch is imported first on purpose: torch ships `libamdhip64.so.7`, and the native module links the
same SONAME, so both share ONE HIP runtime instance (streams/graphs/pointers interoperate).
On a GPU box a missing extension is an error, never a silent fallback (`require_native`).
"""
from __future__ import annotations

import torch  # noqa: F401  (must precede _C)

try:
    from .. import _C  # type: ignore[attr-defined]
    _IMPORT_ERROR: Exception | None = None
except ImportError as e:  # pragma: no cover - depends on build state
    _C = None
    _IMPORT_ERROR = e


def has_native() -> bool:
    return _C is not None


def native():
    if _C is None:
        raise RuntimeError(f"native extension ollama_operator_amd._C is not built ({_IMPORT_ERROR}); "
                           "run `python build_native.py`")
    return _C


def require_native_on_gpu() -> None:
    """Fail loudly when a GPU is present but the HIP extension is not."""
    if torch.cuda.is_available():
        native()


def stream_handle() -> int:
    return torch.cuda.current_stream().cuda_stream


NORM_NONE, NORM_RMS, NORM_LAYER = 0, 1, 2
EPI_STORE, EPI_ADD, EPI_GLU, EPI_GELU, EPI_QKV = 0, 1, 2, 3, 4
