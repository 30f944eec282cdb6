"""Pure-Python GGUF reader (memory-mapped, zero-copy tensor views).

This is the Python twin of the native reader in `csrc/gguf/gguf.cpp`, which is what the engine
uses to upload weights. The Python one serves tests, `/api/show` metadata and tooling.
Untrusted-input hardening: every length is bounds-checked against the file size, since blobs come
from a registry (reference `pkg/model/pod.go:72-75`, `ollama pull <image>`).
"""
from __future__ import annotations

import mmap
import struct
from dataclasses import dataclass, field
from typing import Any

import numpy as np

from .constants import (BLOCK_GEOMETRY, GGUF_DEFAULT_ALIGNMENT, GGUF_MAGIC, GGMLType, ValueType,
                        tensor_nbytes)

_SCALAR_FMT = {
    ValueType.UINT8: "<B", ValueType.INT8: "<b", ValueType.UINT16: "<H", ValueType.INT16: "<h",
    ValueType.UINT32: "<I", ValueType.INT32: "<i", ValueType.FLOAT32: "<f", ValueType.BOOL: "<?",
    ValueType.UINT64: "<Q", ValueType.INT64: "<q", ValueType.FLOAT64: "<d",
}
_NP_DTYPE = {
    ValueType.UINT8: np.uint8, ValueType.INT8: np.int8, ValueType.UINT16: np.uint16,
    ValueType.INT16: np.int16, ValueType.UINT32: np.uint32, ValueType.INT32: np.int32,
    ValueType.FLOAT32: np.float32, ValueType.BOOL: np.bool_, ValueType.UINT64: np.uint64,
    ValueType.INT64: np.int64, ValueType.FLOAT64: np.float64,
}

MAX_STRING = 1 << 24
MAX_ARRAY = 1 << 28
MAX_DIMS = 4


class GGUFError(ValueError):
    pass


@dataclass
class TensorInfo:
    name: str
    shape: tuple[int, ...]  # ggml order: shape[0] = ne0 (innermost, contiguous)
    ggml_type: GGMLType
    offset: int  # absolute file offset of the data
    nbytes: int

    @property
    def n_elements(self) -> int:
        n = 1
        for d in self.shape:
            n *= d
        return n

    @property
    def torch_shape(self) -> tuple[int, ...]:
        """Row-major (outermost first) shape, i.e. [out_features, in_features] for a matrix."""
        return tuple(reversed(self.shape))


@dataclass
class GGUFFile:
    path: str
    version: int
    metadata: dict[str, Any]
    tensors: dict[str, TensorInfo]
    alignment: int
    data_offset: int
    _mm: mmap.mmap | None = field(default=None, repr=False)

    def raw(self, name: str) -> np.ndarray:
        """Zero-copy uint8 view of a tensor's bytes."""
        t = self.tensors[name]
        return np.frombuffer(self._mm, dtype=np.uint8, count=t.nbytes, offset=t.offset)

    def array(self, name: str) -> np.ndarray:
        """F32/F16/BF16 tensors as float32 numpy arrays in row-major torch shape."""
        t = self.tensors[name]
        raw = self.raw(name)
        if t.ggml_type == GGMLType.F32:
            a = raw.view(np.float32)
        elif t.ggml_type == GGMLType.F16:
            a = raw.view(np.float16).astype(np.float32)
        elif t.ggml_type == GGMLType.BF16:
            a = (raw.view(np.uint16).astype(np.uint32) << 16).view(np.float32)
        else:
            from ..quant import dequantize
            a = dequantize(raw, t.ggml_type, t.n_elements)
        return a.reshape(t.torch_shape)

    def close(self) -> None:
        if self._mm is not None:
            self._mm.close()
            self._mm = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    @property
    def architecture(self) -> str:
        return str(self.metadata.get("general.architecture", "llama"))


class _Cursor:
    def __init__(self, buf, size: int):
        self.buf = buf
        self.size = size
        self.pos = 0

    def take(self, n: int) -> memoryview:
        if n < 0 or self.pos + n > self.size:
            raise GGUFError(f"truncated GGUF: need {n} bytes at {self.pos}, file has {self.size}")
        mv = memoryview(self.buf)[self.pos:self.pos + n]
        self.pos += n
        return mv

    def scalar(self, vt: ValueType):
        fmt = _SCALAR_FMT[vt]
        return struct.unpack(fmt, self.take(struct.calcsize(fmt)))[0]

    def string(self) -> str:
        n = self.scalar(ValueType.UINT64)
        if n > MAX_STRING:
            raise GGUFError(f"string length {n} exceeds limit")
        return bytes(self.take(n)).decode("utf-8", errors="replace")

    def value(self, vt: ValueType, depth: int = 0):
        if vt == ValueType.STRING:
            return self.string()
        if vt == ValueType.ARRAY:
            if depth > 2:
                raise GGUFError("nested arrays too deep")
            et = ValueType(self.scalar(ValueType.UINT32))
            n = self.scalar(ValueType.UINT64)
            if n > MAX_ARRAY:
                raise GGUFError(f"array length {n} exceeds limit")
            if et in _NP_DTYPE:
                dt = np.dtype(_NP_DTYPE[et]).newbyteorder("<")
                arr = np.frombuffer(self.take(n * dt.itemsize), dtype=dt).copy()
                return arr.tolist()
            return [self.value(et, depth + 1) for _ in range(n)]
        try:
            return self.scalar(vt)
        except KeyError as e:
            raise GGUFError(f"unknown value type {vt}") from e


def read_gguf(path: str) -> GGUFFile:
    f = open(path, "rb")
    try:
        mm = mmap.mmap(f.fileno(), 0, access=mmap.ACCESS_READ)
    finally:
        f.close()
    size = len(mm)
    c = _Cursor(mm, size)
    try:
        magic = c.scalar(ValueType.UINT32)
        if magic != GGUF_MAGIC:
            raise GGUFError(f"not a GGUF file (magic {magic:#x})")
        version = c.scalar(ValueType.UINT32)
        if version not in (2, 3):
            raise GGUFError(f"unsupported GGUF version {version}")
        n_tensors = c.scalar(ValueType.UINT64)
        n_kv = c.scalar(ValueType.UINT64)
        if n_tensors > 1 << 20 or n_kv > 1 << 20:
            raise GGUFError("implausible tensor/kv count")
        md: dict[str, Any] = {}
        for _ in range(n_kv):
            key = c.string()
            vt = ValueType(c.scalar(ValueType.UINT32))
            md[key] = c.value(vt)
        infos = []
        for _ in range(n_tensors):
            name = c.string()
            nd = c.scalar(ValueType.UINT32)
            if nd == 0 or nd > MAX_DIMS:
                raise GGUFError(f"tensor {name}: bad n_dims {nd}")
            shape = tuple(int(c.scalar(ValueType.UINT64)) for _ in range(nd))
            tt = c.scalar(ValueType.UINT32)
            try:
                gt = GGMLType(tt)
            except ValueError as e:
                raise GGUFError(f"tensor {name}: unknown ggml type {tt}") from e
            if gt not in BLOCK_GEOMETRY:
                raise GGUFError(f"tensor {name}: unsupported ggml type {gt.name}")
            off = c.scalar(ValueType.UINT64)
            infos.append((name, shape, gt, off))
        align = int(md.get("general.alignment", GGUF_DEFAULT_ALIGNMENT))
        if align <= 0 or align & (align - 1):
            raise GGUFError(f"bad alignment {align}")
        data_off = (c.pos + align - 1) // align * align
        tensors: dict[str, TensorInfo] = {}
        for name, shape, gt, off in infos:
            n = 1
            for d in shape:
                n *= d
            nb = tensor_nbytes(gt, n)
            start = data_off + off
            if off % align or start + nb > size:
                raise GGUFError(f"tensor {name}: data [{start}, {start + nb}) outside file ({size})")
            tensors[name] = TensorInfo(name, shape, gt, start, nb)
    except (struct.error, UnicodeDecodeError) as e:
        mm.close()
        raise GGUFError(str(e)) from e
    except Exception:
        mm.close()
        raise
    return GGUFFile(path, version, md, tensors, align, data_off, mm)
