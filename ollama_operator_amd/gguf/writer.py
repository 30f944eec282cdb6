"""Streaming GGUF v3 writer. Used to build random-init model fixtures of real architectures
(the north star mandates random-init GGUF weights; no network for real checkpoints)."""
from __future__ import annotations

import struct
from typing import Any, Callable

import numpy as np

from .constants import GGUF_DEFAULT_ALIGNMENT, GGUF_MAGIC, GGUF_VERSION, GGMLType, ValueType, tensor_nbytes


def _enc_str(s: str) -> bytes:
    b = s.encode("utf-8")
    return struct.pack("<Q", len(b)) + b


def _infer_vt(v: Any) -> ValueType:
    if isinstance(v, bool):
        return ValueType.BOOL
    if isinstance(v, int):
        return ValueType.UINT32 if 0 <= v < 2**32 else ValueType.INT64
    if isinstance(v, float):
        return ValueType.FLOAT32
    if isinstance(v, str):
        return ValueType.STRING
    if isinstance(v, (list, tuple, np.ndarray)):
        return ValueType.ARRAY
    raise TypeError(f"cannot encode {type(v)}")


_FMT = {ValueType.UINT8: "B", ValueType.INT8: "b", ValueType.UINT16: "H", ValueType.INT16: "h",
        ValueType.UINT32: "I", ValueType.INT32: "i", ValueType.FLOAT32: "f", ValueType.BOOL: "?",
        ValueType.UINT64: "Q", ValueType.INT64: "q", ValueType.FLOAT64: "d"}


def _enc_value(v: Any, vt: ValueType, elem_vt: ValueType | None = None) -> bytes:
    if vt == ValueType.STRING:
        return _enc_str(v)
    if vt == ValueType.ARRAY:
        items = list(v) if not isinstance(v, np.ndarray) else v
        if elem_vt is None:
            if isinstance(v, np.ndarray):
                elem_vt = {np.dtype(np.float32): ValueType.FLOAT32, np.dtype(np.int32): ValueType.INT32,
                           np.dtype(np.uint8): ValueType.UINT8}.get(v.dtype, ValueType.INT32)
            else:
                elem_vt = _infer_vt(items[0]) if len(items) else ValueType.INT32
                if elem_vt == ValueType.UINT32 and any(isinstance(x, int) and x < 0 for x in items):
                    elem_vt = ValueType.INT32
        out = struct.pack("<IQ", int(elem_vt), len(items))
        if elem_vt == ValueType.STRING:
            return out + b"".join(_enc_str(s) for s in items)
        dt = {ValueType.FLOAT32: "<f4", ValueType.INT32: "<i4", ValueType.UINT32: "<u4",
              ValueType.UINT8: "u1", ValueType.INT8: "i1", ValueType.BOOL: "?", ValueType.INT64: "<i8",
              ValueType.UINT64: "<u8", ValueType.FLOAT64: "<f8", ValueType.INT16: "<i2",
              ValueType.UINT16: "<u2"}[elem_vt]
        return out + np.asarray(items, dtype=dt).tobytes()
    return struct.pack("<" + _FMT[vt], v)


class GGUFWriter:
    """kv = metadata; tensors are added with a byte producer so multi-GB files stream to disk."""

    def __init__(self, path: str, alignment: int = GGUF_DEFAULT_ALIGNMENT):
        self.path = path
        self.alignment = alignment
        self.kv: list[tuple[str, ValueType, Any, ValueType | None]] = []
        self.tensors: list[tuple[str, tuple[int, ...], GGMLType, int, Callable[[], bytes | np.ndarray]]] = []
        if alignment != GGUF_DEFAULT_ALIGNMENT:
            self.add("general.alignment", alignment, ValueType.UINT32)

    def add(self, key: str, value: Any, vt: ValueType | None = None, elem_vt: ValueType | None = None):
        self.kv.append((key, vt if vt is not None else _infer_vt(value), value, elem_vt))

    def add_tensor(self, name: str, shape_ggml: tuple[int, ...], ggml_type: GGMLType,
                   producer: Callable[[], bytes | np.ndarray] | bytes | np.ndarray):
        n = 1
        for d in shape_ggml:
            n *= d
        nb = tensor_nbytes(ggml_type, n)
        if not callable(producer):
            data = producer
            producer = lambda d=data: d  # noqa: E731
        self.tensors.append((name, tuple(int(d) for d in shape_ggml), GGMLType(ggml_type), nb, producer))

    def write(self) -> None:
        a = self.alignment
        header = bytearray(struct.pack("<IIQQ", GGUF_MAGIC, GGUF_VERSION, len(self.tensors), len(self.kv)))
        for key, vt, val, evt in self.kv:
            header += _enc_str(key) + struct.pack("<I", int(vt)) + _enc_value(val, vt, evt)
        off = 0
        offsets = []
        for name, shape, gt, nb, _ in self.tensors:
            offsets.append(off)
            header += _enc_str(name) + struct.pack("<I", len(shape))
            header += struct.pack(f"<{len(shape)}Q", *shape)
            header += struct.pack("<IQ", int(gt), off)
            off = (off + nb + a - 1) // a * a
        pad = (-len(header)) % a
        header += b"\0" * pad
        with open(self.path, "wb") as f:
            f.write(header)
            for (name, shape, gt, nb, producer), o in zip(self.tensors, offsets):
                data = producer()
                if isinstance(data, np.ndarray):
                    data = np.ascontiguousarray(data).view(np.uint8).reshape(-1)
                    if data.nbytes != nb:
                        raise ValueError(f"{name}: produced {data.nbytes} bytes, expected {nb}")
                    f.write(memoryview(data))
                else:
                    if len(data) != nb:
                        raise ValueError(f"{name}: produced {len(data)} bytes, expected {nb}")
                    f.write(data)
                f.write(b"\0" * ((-nb) % a))
