"""GGUF container constants (public GGUF v3 spec) and ggml quant-type geometry.

The reference operator never parses GGUF itself: its pods run `ollama pull` / `ollama serve`
(reference `pkg/model/pod.go:14-83`) and the model layer of the pulled image is a GGUF file
(reference `README.md:41`, "As long as it's a GGUF formatted model"). Our server replaces that
image, so the container format is defined here.
"""
from __future__ import annotations

import enum

GGUF_MAGIC = 0x46554747  # b"GGUF" little-endian
GGUF_VERSION = 3
GGUF_DEFAULT_ALIGNMENT = 32


class ValueType(enum.IntEnum):
    UINT8 = 0
    INT8 = 1
    UINT16 = 2
    INT16 = 3
    UINT32 = 4
    INT32 = 5
    FLOAT32 = 6
    BOOL = 7
    STRING = 8
    ARRAY = 9
    UINT64 = 10
    INT64 = 11
    FLOAT64 = 12


class GGMLType(enum.IntEnum):
    F32 = 0
    F16 = 1
    Q4_0 = 2
    Q4_1 = 3
    Q5_0 = 6
    Q5_1 = 7
    Q8_0 = 8
    Q8_1 = 9
    Q2_K = 10
    Q3_K = 11
    Q4_K = 12
    Q5_K = 13
    Q6_K = 14
    Q8_K = 15
    BF16 = 30


# (elements per block, bytes per block)
BLOCK_GEOMETRY = {
    GGMLType.F32: (1, 4),
    GGMLType.F16: (1, 2),
    GGMLType.BF16: (1, 2),
    GGMLType.Q4_0: (32, 18),
    GGMLType.Q4_1: (32, 20),
    GGMLType.Q5_0: (32, 22),
    GGMLType.Q5_1: (32, 24),
    GGMLType.Q8_0: (32, 34),
    GGMLType.Q8_1: (32, 36),
    GGMLType.Q2_K: (256, 84),
    GGMLType.Q3_K: (256, 110),
    GGMLType.Q4_K: (256, 144),
    GGMLType.Q5_K: (256, 176),
    GGMLType.Q6_K: (256, 210),
    GGMLType.Q8_K: (256, 292),
}

QK_K = 256


class FileType(enum.IntEnum):
    """`general.file_type` values (llama.cpp LLAMA_FTYPE_*)."""
    ALL_F32 = 0
    MOSTLY_F16 = 1
    MOSTLY_Q4_0 = 2
    MOSTLY_Q4_1 = 3
    MOSTLY_Q8_0 = 7
    MOSTLY_Q5_0 = 8
    MOSTLY_Q5_1 = 9
    MOSTLY_Q2_K = 10
    MOSTLY_Q3_K_S = 11
    MOSTLY_Q3_K_M = 12
    MOSTLY_Q3_K_L = 13
    MOSTLY_Q4_K_S = 14
    MOSTLY_Q4_K_M = 15
    MOSTLY_Q5_K_S = 16
    MOSTLY_Q5_K_M = 17
    MOSTLY_Q6_K = 18
    MOSTLY_BF16 = 32


FILE_TYPE_NAMES = {
    FileType.ALL_F32: "F32",
    FileType.MOSTLY_F16: "F16",
    FileType.MOSTLY_Q4_0: "Q4_0",
    FileType.MOSTLY_Q4_1: "Q4_1",
    FileType.MOSTLY_Q8_0: "Q8_0",
    FileType.MOSTLY_Q5_0: "Q5_0",
    FileType.MOSTLY_Q5_1: "Q5_1",
    FileType.MOSTLY_Q2_K: "Q2_K",
    FileType.MOSTLY_Q3_K_S: "Q3_K_S",
    FileType.MOSTLY_Q3_K_M: "Q3_K_M",
    FileType.MOSTLY_Q3_K_L: "Q3_K_L",
    FileType.MOSTLY_Q4_K_S: "Q4_K_S",
    FileType.MOSTLY_Q4_K_M: "Q4_K_M",
    FileType.MOSTLY_Q5_K_S: "Q5_K_S",
    FileType.MOSTLY_Q5_K_M: "Q5_K_M",
    FileType.MOSTLY_Q6_K: "Q6_K",
    FileType.MOSTLY_BF16: "BF16",
}


def tensor_nbytes(ggml_type: int, n_elements: int) -> int:
    blk, nb = BLOCK_GEOMETRY[GGMLType(ggml_type)]
    if n_elements % blk:
        raise ValueError(f"{GGMLType(ggml_type).name}: {n_elements} elements not a multiple of {blk}")
    return n_elements // blk * nb
