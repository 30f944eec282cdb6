import struct

import numpy as np
import pytest

from ollama_operator_amd.gguf import GGMLType, GGUFError, GGUFWriter, read_gguf
from ollama_operator_amd.gguf.constants import BLOCK_GEOMETRY
from ollama_operator_amd.quant import (dequantize, pack_q4k_scales, quantize, random_blocks, repack,
                                       unpack_q4k_scales, unrepack)

QTYPES = [GGMLType.Q4_0, GGMLType.Q8_0, GGMLType.Q4_K, GGMLType.Q5_K, GGMLType.Q6_K]


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
    bound = {GGMLType.Q4_0: 0.12, GGMLType.Q8_0: 0.01, GGMLType.Q4_K: 0.12, GGMLType.Q5_K: 0.06,
             GGMLType.Q6_K: 0.03}[t]
    assert rel < bound, rel


@pytest.mark.parametrize("t", QTYPES)
@pytest.mark.parametrize("k", [512, 288])
def test_repack_roundtrip(t, k):
    if k % 256 and t in (GGMLType.Q4_K, GGMLType.Q5_K, GGMLType.Q6_K):
        pytest.skip("k-quants are whole super-blocks")
    rng = np.random.default_rng(2)
    n = 8
    raw = random_blocks(t, n, k, rng)
    s = repack(raw, t, n, k)
    padded = n * ((k + 255) // 256 * 256 // BLOCK_GEOMETRY[t][0]) * BLOCK_GEOMETRY[t][1]
    assert sum(v.nbytes for v in s.values()) == padded  # no extra bandwidth beyond K padding
    np.testing.assert_array_equal(unrepack(s, t, n, k), raw)


def _kernel_model_dequant(s, t, n, k):
    """numpy model of how csrc/kernels/gemv.hip decodes layout-v2 streams (piece-major codes,
    signed high nibble, Q6_K H0/H1 fields) -- pins the layout contract the HIP kernel relies on."""
    sb = (k + 255) // 256
    w = np.zeros((n, sb * 256), np.float32)
    f16 = lambda b: b.view(np.float16).astype(np.float32)  # noqa: E731
    for r in range(n):
        for b in range(sb):
            for t_ in range(8):
                if t == GGMLType.Q8_0:
                    q = s["qs"][r].reshape(8, sb, 32)[t_, b].view(np.int8).astype(np.float32)
                    d = f16(s["d"][r].reshape(sb, 8, 2)[b, t_].copy())[0]
                    w[r, 256 * b + 32 * t_: 256 * b + 32 * t_ + 32] = d * q
                    continue
                a = s["qs" if t != GGMLType.Q6_K else "ql"][r].reshape(8, sb, 16)[t_, b]
                if t == GGMLType.Q5_K:  # unsigned nibbles + 5th bit from the piece dword H
                    m = s["meta"][r].reshape(sb, 16)[b]
                    d, dmin = f16(m[0:2].copy())[0], f16(m[2:4].copy())[0]
                    sc, mn = unpack_q4k_scales(m[4:16])
                    H = int(s["qh"][r].reshape(8, sb, 4)[t_, b].view(np.uint32)[0])
                    lo5 = np.array([(int(a[i]) & 15) | (((H >> (8 * (i & 3) + (i >> 2))) & 1) << 4) for i in range(16)])
                    hi5 = np.array([(int(a[i]) >> 4) | (((H >> (8 * (i & 3) + 4 + (i >> 2))) & 1) << 4)
                                    for i in range(16)])
                    c, h = t_ >> 1, t_ & 1
                    o = 256 * b + 64 * c + 16 * h
                    w[r, o:o + 16] = d * sc[2 * c] * lo5 - dmin * mn[2 * c]
                    w[r, o + 32:o + 48] = d * sc[2 * c + 1] * hi5 - dmin * mn[2 * c + 1]
                    continue
                lo = (a & 0x0F).astype(np.float32)
                hi16 = (a & 0xF0).view(np.int8).astype(np.float32)  # = 16 * (n - 8) for 4-bit types
                if t == GGMLType.Q4_0:
                    d = f16(s["d"][r].reshape(sb, 8, 2)[b, t_].copy())[0]
                    w[r, 256 * b + 32 * t_: 256 * b + 32 * t_ + 16] = d * (lo - 8)
                    w[r, 256 * b + 32 * t_ + 16: 256 * b + 32 * t_ + 32] = d * hi16 / 16
                elif t == GGMLType.Q4_K:
                    m = s["meta"][r].reshape(sb, 16)[b]
                    d, dmin = f16(m[0:2].copy())[0], f16(m[2:4].copy())[0]
                    sc, mn = unpack_q4k_scales(m[4:16])
                    c, h = t_ >> 1, t_ & 1
                    o = 256 * b + 64 * c + 16 * h
                    w[r, o:o + 16] = d * sc[2 * c] * lo - dmin * mn[2 * c]
                    w[r, o + 32:o + 48] = d * sc[2 * c + 1] * (hi16 / 16 + 8) - dmin * mn[2 * c + 1]
                else:
                    hq = s["qh"][r].reshape(8, sb, 8)[t_, b].view(np.uint32)
                    hi = ((a >> 4) & 0x0F).astype(np.int32)
                    ql = (a & 0x0F).astype(np.int32)
                    for kk in range(4):  # lo dword kk: bytes j <- field kk of H0 byte j
                        for j in range(4):
                            i = 4 * kk + j
                            ql[i] |= ((int(hq[0]) >> (8 * j + 2 * kk)) & 3) << 4
                            hi[i] |= ((int(hq[1]) >> (8 * j + 2 * kk)) & 3) << 4
                    sc = s["sc"][r].reshape(sb, 16)[b].view(np.int8).astype(np.float32)
                    d = f16(s["d"][r].reshape(sb, 2)[b].copy())[0]
                    nn, sub = t_ >> 2, t_ & 3
                    o = 256 * b + 128 * nn + 16 * sub
                    w[r, o:o + 16] = d * sc[8 * nn + sub] * (ql - 32)
                    w[r, o + 64:o + 80] = d * sc[8 * nn + sub + 4] * (hi - 32)
    return w[:, :k]


@pytest.mark.parametrize("t", QTYPES)
def test_repack_kernel_contract(t):
    rng = np.random.default_rng(3)
    n, k = 3, 512 if t in (GGMLType.Q4_K, GGMLType.Q5_K, GGMLType.Q6_K) else 288
    raw = random_blocks(t, n, k, rng)
    got = _kernel_model_dequant(repack(raw, t, n, k), t, n, k)
    np.testing.assert_allclose(got, dequantize(raw, t, n * k).reshape(n, k), rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("t", QTYPES)
def test_random_blocks_std(t):
    rng = np.random.default_rng(3)
    y = dequantize(random_blocks(t, 64, 1024, rng, std=0.02), t, 64 * 1024)
    assert 0.01 < y.std() < 0.04
    assert abs(y.mean()) < 0.01


@pytest.mark.parametrize("t", QTYPES)
def test_native_repack_matches_numpy(t):
    """csrc/gguf/gguf.cpp repack_rows (the load path) == quant.repack (the layout spec), incl. a row
    permutation (TP shards) and a K block range."""
    from ollama_operator_amd.ops import native
    from ollama_operator_amd.quant import REPACK_STREAMS, repack_row_bytes
    try:
        nat = native()
    except Exception as e:  # extension not built in this environment
        pytest.skip(str(e))
    rng = np.random.default_rng(4)
    n, k = 6, 1024
    raw = random_blocks(t, n, k, rng)
    blk = BLOCK_GEOMETRY[t][0]
    kb0, kb1 = 256 // blk, 1024 // blk  # columns 256..1023
    rows = np.array([5, 0, 3], np.int64)
    dst_rows = np.arange(3, dtype=np.int64)
    kk = (kb1 - kb0) * blk
    dst = [np.zeros((3, b), np.uint8) for b in repack_row_bytes(t, kk)]
    nat.repack_ptr(raw.ctypes.data, int(t), k, rows, dst_rows, kb0, kb1, [d.ctypes.data for d in dst], 2)
    sub = raw.reshape(n, -1)[rows][:, kb0 * BLOCK_GEOMETRY[t][1]:kb1 * BLOCK_GEOMETRY[t][1]]
    want = repack(np.ascontiguousarray(sub).reshape(-1), t, 3, kk)
    for name, d in zip(REPACK_STREAMS[t], dst):
        np.testing.assert_array_equal(d, want[name].reshape(3, -1), err_msg=name)


@pytest.mark.parametrize("t", QTYPES)
def test_repack_padded_k_native_matches_numpy(t):
    """K_out > K (the GPU loader's ffn_down padding, weights.ffn_pad): every stream keeps the real
    super-blocks at their piece-major places with the padded stride, zeros past K; the native repacker
    and its numpy twin agree, and unrepacking the padded rows gives the source columns then zeros."""
    from ollama_operator_amd.engine.weights import _np_repack_rows
    from ollama_operator_amd.ops import native
    from ollama_operator_amd.quant import repack_row_bytes, unrepack
    rng = np.random.default_rng(5)
    n, k, k_out = 4, 768, 1536  # 3 super-blocks stored as 6
    raw = random_blocks(t, n, k, rng)
    blk = BLOCK_GEOMETRY[t][0]
    rows, dst_rows = np.arange(n, dtype=np.int64), np.arange(n, dtype=np.int64)
    want = [np.zeros((n, b), np.uint8) for b in repack_row_bytes(t, k_out)]
    _np_repack_rows(raw, int(t), k, rows, dst_rows, 0, k // blk, want, k_out)
    try:
        nat = native()
    except Exception:
        nat = None
    if nat is not None:
        got = [np.zeros((n, b), np.uint8) for b in repack_row_bytes(t, k_out)]
        nat.repack_ptr(raw.ctypes.data, int(t), k, rows, dst_rows, 0, k // blk, [d.ctypes.data for d in got], 2, k_out)
        for a, b in zip(got, want):
            np.testing.assert_array_equal(a, b)
    from ollama_operator_amd.quant import REPACK_STREAMS
    back = unrepack({nm: w for nm, w in zip(REPACK_STREAMS[t], want)}, t, n, k_out)
    y = dequantize(back.reshape(-1), t, n * k_out).reshape(n, k_out)
    x = dequantize(raw.reshape(-1), t, n * k).reshape(n, k)
    np.testing.assert_array_equal(y[:, :k], x)
    assert not y[:, k:].any()
