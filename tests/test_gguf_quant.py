import struct

import numpy as np
import pytest

from ollama_operator_amd.gguf import GGMLType, GGUFError, GGUFWriter, read_gguf
from ollama_operator_amd.quant import (dequantize, pack_q4k_scales, quantize, random_blocks, repack,
                                       unpack_q4k_scales, unrepack)

QTYPES = [GGMLType.Q4_0, GGMLType.Q8_0, GGMLType.Q4_K, GGMLType.Q6_K]


def test_gguf_roundtrip(tmp_path):
    p = str(tmp_path / "t.gguf")
    w = GGUFWriter(p)
    w.add("general.architecture", "llama")
    w.add("llama.block_count", 3)
    w.add("some.float", 1.5)
    w.add("some.list", ["a", "bb", "ccc"])
    w.add("some.ints", [1, -2, 3])
    w.add("some.bool", True)
    a = np.arange(512, dtype=np.float32).reshape(2, 256)
    w.add_tensor("a", (256, 2), GGMLType.F32, a)
    q = quantize(np.linspace(-1, 1, 512, dtype=np.float32), GGMLType.Q4_K)
    w.add_tensor("q", (256, 2), GGMLType.Q4_K, q)
    w.write()
    g = read_gguf(p)
    assert g.metadata["general.architecture"] == "llama"
    assert g.metadata["llama.block_count"] == 3
    assert g.metadata["some.float"] == pytest.approx(1.5)
    assert g.metadata["some.list"] == ["a", "bb", "ccc"]
    assert g.metadata["some.ints"] == [1, -2, 3]
    assert g.metadata["some.bool"] is True
    assert g.tensors["a"].torch_shape == (2, 256)
    np.testing.assert_array_equal(g.array("a"), a)
    assert g.tensors["q"].offset % 32 == 0
    np.testing.assert_array_equal(g.raw("q"), q)
    g.close()


def test_gguf_rejects_garbage(tmp_path):
    p = tmp_path / "bad.gguf"
    p.write_bytes(b"NOPE" + b"\0" * 100)
    with pytest.raises(GGUFError):
        read_gguf(str(p))
    # truncated tensor data
    hdr = struct.pack("<IIQQ", 0x46554747, 3, 1, 0)
    hdr += struct.pack("<Q", 1) + b"t" + struct.pack("<I", 1) + struct.pack("<Q", 1 << 20)
    hdr += struct.pack("<IQ", 0, 0)
    p.write_bytes(hdr)
    with pytest.raises(GGUFError):
        read_gguf(str(p))


def test_q4k_scale_pack_roundtrip():
    rng = np.random.default_rng(0)
    sc = rng.integers(0, 64, (100, 8))
    m = rng.integers(0, 64, (100, 8))
    s2, m2 = unpack_q4k_scales(pack_q4k_scales(sc, m))
    np.testing.assert_array_equal(s2, sc)
    np.testing.assert_array_equal(m2, m)


@pytest.mark.parametrize("t", QTYPES)
def test_quant_error_bounded(t):
    rng = np.random.default_rng(1)
    x = rng.standard_normal(256 * 64).astype(np.float32)
    y = dequantize(quantize(x, t), t, x.size)
    rel = np.linalg.norm(y - x) / np.linalg.norm(x)
    bound = {GGMLType.Q4_0: 0.12, GGMLType.Q8_0: 0.01, GGMLType.Q4_K: 0.12, GGMLType.Q6_K: 0.03}[t]
    assert rel < bound, rel


@pytest.mark.parametrize("t", QTYPES)
def test_repack_roundtrip(t):
    rng = np.random.default_rng(2)
    n, k = 8, 512
    raw = random_blocks(t, n, k, rng)
    s = repack(raw, t, n, k)
    assert sum(v.nbytes for v in s.values()) == raw.nbytes  # no extra bandwidth
    np.testing.assert_array_equal(unrepack(s, t, n, k), raw)


@pytest.mark.parametrize("t", QTYPES)
def test_random_blocks_std(t):
    rng = np.random.default_rng(3)
    y = dequantize(random_blocks(t, 64, 1024, rng, std=0.02), t, 64 * 1024)
    assert 0.01 < y.std() < 0.04
    assert abs(y.mean()) < 0.01
