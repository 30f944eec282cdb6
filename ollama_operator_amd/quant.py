"""Reference (numpy) quantize / dequantize for the ggml block formats the engine serves, plus the
device repack that splits each block into 16-byte-aligned streams for the gfx950 GEMV kernels.

Block layouts follow the public ggml definitions:
  Q4_0 : fp16 d | 16 B nibbles                          (32 weights, 18 B)   x = (q - 8) * d
  Q8_0 : fp16 d | int8[32]                              (32 weights, 34 B)   x = q * d
  Q4_K : fp16 d | fp16 dmin | 12 B 6-bit (sc, m) x 8 | 128 B nibbles  (256 w, 144 B)
         x = d*sc_j*q - dmin*m_j   (sub-block j of 32)
  Q5_K : fp16 d | fp16 dmin | 12 B 6-bit (sc, m) x 8 | 32 B qh | 128 B nibbles  (256 w, 176 B)
         x = d*sc_j*(n + 16*h) - dmin*m_j   (h = bit j of qh[l])
  Q6_K : 128 B ql | 64 B qh | int8 sc[16] | fp16 d    (256 w, 210 B)    x = d*sc_g*(q - 32)

Device layout ("repacked"): every type is stored as separate row-major streams so that one lane's
16-byte load is always a whole, aligned group of weights (see csrc/kernels/gemv.hip):
  Q4_K -> qs [N, K/2]  + meta [N, K/256, 16]  (d, dmin, scales12: byte-identical to the block head)
  Q5_K -> qs [N, K/2]  + meta [N, K/16]  + qh [N, K/8]  (high bits regrouped per piece)
  Q6_K -> ql [N, K/2]  + qh [N, K/4] + sc [N, K/16] int8 + d [N, K/256] fp16
  Q4_0 -> qs [N, K/2]  + d [N, K/32] fp16
  Q8_0 -> qs [N, K]    + d [N, K/32] fp16
Total bytes are identical to the GGUF blocks: the repack costs no bandwidth.
"""
from __future__ import annotations

import numpy as np

from .gguf.constants import BLOCK_GEOMETRY, GGMLType

QK_K = 256


# ----------------------------------------------------------------------------------------------
# dequantize
# ----------------------------------------------------------------------------------------------

def _f16(b: np.ndarray) -> np.ndarray:
    return np.ascontiguousarray(b).view(np.float16).astype(np.float32)


def unpack_q4k_scales(sc12: np.ndarray) -> tuple[np.ndarray, np.ndarray]:
    """sc12: [..., 12] uint8 -> (sc [..., 8], m [..., 8]) as float32."""
    q = sc12.astype(np.uint8)
    sc = np.empty(q.shape[:-1] + (8,), np.uint8)
    m = np.empty_like(sc)
    sc[..., :4] = q[..., 0:4] & 63
    m[..., :4] = q[..., 4:8] & 63
    sc[..., 4:] = (q[..., 8:12] & 0xF) | ((q[..., 0:4] >> 6) << 4)
    m[..., 4:] = (q[..., 8:12] >> 4) | ((q[..., 4:8] >> 6) << 4)
    return sc.astype(np.float32), m.astype(np.float32)


def pack_q4k_scales(sc: np.ndarray, m: np.ndarray) -> np.ndarray:
    sc = sc.astype(np.uint8)
    m = m.astype(np.uint8)
    out = np.empty(sc.shape[:-1] + (12,), np.uint8)
    out[..., 0:4] = (sc[..., 0:4] & 63) | ((sc[..., 4:8] >> 4) << 6)
    out[..., 4:8] = (m[..., 0:4] & 63) | ((m[..., 4:8] >> 4) << 6)
    out[..., 8:12] = (sc[..., 4:8] & 0xF) | ((m[..., 4:8] & 0xF) << 4)
    return out


def dequantize(raw: np.ndarray, ggml_type: int, n_elements: int) -> np.ndarray:
    t = GGMLType(ggml_type)
    raw = np.ascontiguousarray(raw).view(np.uint8).reshape(-1)
    if t == GGMLType.F32:
        return raw.view(np.float32)[:n_elements].copy()
    if t == GGMLType.F16:
        return raw.view(np.float16)[:n_elements].astype(np.float32)
    if t == GGMLType.BF16:
        return (raw.view(np.uint16)[:n_elements].astype(np.uint32) << 16).view(np.float32)
    blk, nb = BLOCK_GEOMETRY[t]
    nblk = n_elements // blk
    b = raw[: nblk * nb].reshape(nblk, nb)
    if t == GGMLType.Q4_0:
        d = _f16(b[:, 0:2]).reshape(nblk, 1)
        qs = b[:, 2:18]
        q = np.concatenate([qs & 0xF, qs >> 4], axis=1).astype(np.float32) - 8.0
        return (q * d).reshape(-1)
    if t == GGMLType.Q4_1:
        d = _f16(b[:, 0:2]).reshape(nblk, 1)
        mn = _f16(b[:, 2:4]).reshape(nblk, 1)
        qs = b[:, 4:20]
        q = np.concatenate([qs & 0xF, qs >> 4], axis=1).astype(np.float32)
        return (q * d + mn).reshape(-1)
    if t == GGMLType.Q5_0:
        d = _f16(b[:, 0:2]).reshape(nblk, 1)
        qh = b[:, 2:6].copy().view(np.uint32).reshape(nblk, 1)
        qs = b[:, 6:22]
        j = np.arange(16, dtype=np.uint32)
        hlo = ((qh >> j) & 1) << 4
        hhi = ((qh >> (j + 16)) & 1) << 4
        q = np.concatenate([(qs & 0xF) | hlo, (qs >> 4) | hhi], axis=1).astype(np.float32) - 16.0
        return (q * d).reshape(-1)
    if t == GGMLType.Q5_1:
        d = _f16(b[:, 0:2]).reshape(nblk, 1)
        mn = _f16(b[:, 2:4]).reshape(nblk, 1)
        qh = b[:, 4:8].copy().view(np.uint32).reshape(nblk, 1)
        qs = b[:, 8:24]
        j = np.arange(16, dtype=np.uint32)
        hlo = ((qh >> j) & 1) << 4
        hhi = ((qh >> (j + 16)) & 1) << 4
        q = np.concatenate([(qs & 0xF) | hlo, (qs >> 4) | hhi], axis=1).astype(np.float32)
        return (q * d + mn).reshape(-1)
    if t == GGMLType.Q8_0:
        d = _f16(b[:, 0:2]).reshape(nblk, 1)
        q = b[:, 2:34].view(np.int8).astype(np.float32)
        return (q * d).reshape(-1)
    if t == GGMLType.Q4_K:
        d = _f16(b[:, 0:2]).reshape(nblk, 1, 1)
        dmin = _f16(b[:, 2:4]).reshape(nblk, 1, 1)
        sc, m = unpack_q4k_scales(b[:, 4:16])  # [nblk, 8]
        qs = b[:, 16:144].reshape(nblk, 4, 32)
        q = np.stack([qs & 0xF, qs >> 4], axis=2).reshape(nblk, 8, 32).astype(np.float32)
        y = d * sc[:, :, None] * q - dmin * m[:, :, None]
        return y.reshape(-1)
    if t == GGMLType.Q5_K:
        d = _f16(b[:, 0:2]).reshape(nblk, 1, 1)
        dmin = _f16(b[:, 2:4]).reshape(nblk, 1, 1)
        sc, m = unpack_q4k_scales(b[:, 4:16])
        qh = b[:, 16:48]  # [nblk, 32]
        qs = b[:, 48:176].reshape(nblk, 4, 32)
        lo = np.stack([qs & 0xF, qs >> 4], axis=2).reshape(nblk, 8, 32)
        hb = np.stack([(qh >> i) & 1 for i in range(8)], axis=1)  # [nblk, 8, 32]
        q = (lo | (hb << 4)).astype(np.float32)
        y = d * sc[:, :, None] * q - dmin * m[:, :, None]
        return y.reshape(-1)
    if t == GGMLType.Q6_K:
        ql = b[:, 0:128].reshape(nblk, 2, 64)
        qh = b[:, 128:192].reshape(nblk, 2, 32)
        sc = b[:, 192:208].view(np.int8).astype(np.float32).reshape(nblk, 16)
        d = _f16(b[:, 208:210]).reshape(nblk, 1)
        q1 = (ql[:, :, 0:32] & 0xF) | (((qh >> 0) & 3) << 4)
        q2 = (ql[:, :, 32:64] & 0xF) | (((qh >> 2) & 3) << 4)
        q3 = (ql[:, :, 0:32] >> 4) | (((qh >> 4) & 3) << 4)
        q4 = (ql[:, :, 32:64] >> 4) | (((qh >> 6) & 3) << 4)
        q = np.stack([q1, q2, q3, q4], axis=2).reshape(nblk, 256).astype(np.float32) - 32.0
        s = np.repeat(sc, 16, axis=1)
        return (q * s * d).reshape(-1)
    raise NotImplementedError(f"dequantize {t.name}")


# ----------------------------------------------------------------------------------------------
# quantize (reference quality, used for test fixtures and `create` from float weights)
# ----------------------------------------------------------------------------------------------

def _to_f16_bytes(a: np.ndarray) -> np.ndarray:
    return a.astype(np.float16).view(np.uint8).reshape(a.shape[0], 2)


def quantize(x: np.ndarray, ggml_type: int) -> np.ndarray:
    """x: float array whose size is a multiple of the block size -> uint8 bytes of ggml blocks."""
    t = GGMLType(ggml_type)
    x = np.ascontiguousarray(x, dtype=np.float32).reshape(-1)
    if t == GGMLType.F32:
        return x.view(np.uint8).copy()
    if t == GGMLType.F16:
        return x.astype(np.float16).view(np.uint8).copy()
    if t == GGMLType.BF16:
        u = x.view(np.uint32)
        r = ((u + 0x7FFF + ((u >> 16) & 1)) >> 16).astype(np.uint16)
        return r.view(np.uint8).copy()
    blk, nb = BLOCK_GEOMETRY[t]
    nblk = x.size // blk
    xb = x.reshape(nblk, blk)
    out = np.zeros((nblk, nb), np.uint8)
    if t == GGMLType.Q8_0:
        amax = np.abs(xb).max(axis=1)
        d = (amax / 127.0).astype(np.float16).astype(np.float32)
        inv = np.where(d > 0, 1.0 / np.where(d > 0, d, 1), 0)
        q = np.clip(np.rint(xb * inv[:, None]), -127, 127).astype(np.int8)
        out[:, 0:2] = _to_f16_bytes(d)
        out[:, 2:34] = q.view(np.uint8)
        return out.reshape(-1)
    if t == GGMLType.Q4_0:
        # ggml: d = max_signed / -8 so the extreme value maps exactly to q = 0
        idx = np.abs(xb).argmax(axis=1)
        mx = xb[np.arange(nblk), idx]
        d = (mx / -8.0).astype(np.float16).astype(np.float32)
        inv = np.where(d != 0, 1.0 / np.where(d != 0, d, 1), 0)
        q = np.clip(np.rint(xb * inv[:, None] + 8.0), 0, 15).astype(np.uint8)
        out[:, 0:2] = _to_f16_bytes(d)
        out[:, 2:18] = q[:, :16] | (q[:, 16:] << 4)
        return out.reshape(-1)
    if t == GGMLType.Q4_K:
        sub = xb.reshape(nblk, 8, 32)
        mn = np.minimum(sub.min(axis=2), 0.0)
        mx = sub.max(axis=2)
        scale = (mx - mn) / 15.0
        mins = -mn
        d = (scale.max(axis=1) / 63.0).astype(np.float16).astype(np.float32)
        dmin = (mins.max(axis=1) / 63.0).astype(np.float16).astype(np.float32)
        sc = np.clip(np.rint(scale / np.where(d > 0, d, 1)[:, None]), 0, 63)
        m = np.clip(np.rint(mins / np.where(dmin > 0, dmin, 1)[:, None]), 0, 63)
        eff_d = d[:, None] * sc
        eff_m = dmin[:, None] * m
        q = np.rint((sub + eff_m[:, :, None]) / np.where(eff_d > 0, eff_d, 1)[:, :, None])
        q = np.clip(q, 0, 15).astype(np.uint8)  # [nblk, 8, 32]
        q = q.reshape(nblk, 4, 2, 32)
        qs = q[:, :, 0, :] | (q[:, :, 1, :] << 4)
        out[:, 0:2] = _to_f16_bytes(d)
        out[:, 2:4] = _to_f16_bytes(dmin)
        out[:, 4:16] = pack_q4k_scales(sc, m)
        out[:, 16:144] = qs.reshape(nblk, 128)
        return out.reshape(-1)
    if t == GGMLType.Q5_K:
        sub = xb.reshape(nblk, 8, 32)
        mn = np.minimum(sub.min(axis=2), 0.0)
        mx = sub.max(axis=2)
        scale = (mx - mn) / 31.0
        mins = -mn
        d = (scale.max(axis=1) / 63.0).astype(np.float16).astype(np.float32)
        dmin = (mins.max(axis=1) / 63.0).astype(np.float16).astype(np.float32)
        sc = np.clip(np.rint(scale / np.where(d > 0, d, 1)[:, None]), 0, 63)
        m = np.clip(np.rint(mins / np.where(dmin > 0, dmin, 1)[:, None]), 0, 63)
        eff_d = d[:, None] * sc
        eff_m = dmin[:, None] * m
        q = np.rint((sub + eff_m[:, :, None]) / np.where(eff_d > 0, eff_d, 1)[:, :, None])
        q = np.clip(q, 0, 31).astype(np.uint8)  # [nblk, 8, 32]
        lo = (q & 0xF).reshape(nblk, 4, 2, 32)
        qs = lo[:, :, 0, :] | (lo[:, :, 1, :] << 4)
        qh = np.zeros((nblk, 32), np.uint8)
        for j in range(8):
            qh |= ((q[:, j, :] >> 4) & 1) << j
        out[:, 0:2] = _to_f16_bytes(d)
        out[:, 2:4] = _to_f16_bytes(dmin)
        out[:, 4:16] = pack_q4k_scales(sc, m)
        out[:, 16:48] = qh
        out[:, 48:176] = qs.reshape(nblk, 128)
        return out.reshape(-1)
    if t == GGMLType.Q6_K:
        g = xb.reshape(nblk, 16, 16)
        idx = np.abs(g).argmax(axis=2)
        mxv = np.take_along_axis(g, idx[:, :, None], axis=2)[:, :, 0]
        scale = mxv / -32.0
        amax_s = np.abs(scale).max(axis=1)
        d = (amax_s / 127.0).astype(np.float16).astype(np.float32)
        sc = np.clip(np.rint(scale / np.where(d > 0, d, 1)[:, None]), -128, 127)
        eff = d[:, None] * sc
        q = np.rint(g / np.where(eff != 0, eff, 1)[:, :, None])
        q = (np.clip(q, -32, 31) + 32).astype(np.uint8).reshape(nblk, 2, 4, 32)
        q1, q2, q3, q4 = q[:, :, 0], q[:, :, 1], q[:, :, 2], q[:, :, 3]
        ql = np.concatenate([(q1 & 0xF) | ((q3 & 0xF) << 4), (q2 & 0xF) | ((q4 & 0xF) << 4)], axis=2)
        qh = (q1 >> 4) | ((q2 >> 4) << 2) | ((q3 >> 4) << 4) | ((q4 >> 4) << 6)
        out[:, 0:128] = ql.reshape(nblk, 128)
        out[:, 128:192] = qh.reshape(nblk, 64)
        out[:, 192:208] = sc.astype(np.int8).view(np.uint8)
        out[:, 208:210] = _to_f16_bytes(d)
        return out.reshape(-1)
    raise NotImplementedError(f"quantize {t.name}")


def random_blocks(ggml_type: int, n_rows: int, k: int, rng: np.random.Generator,
                  std: float = 0.02) -> np.ndarray:
    """Random-init quantized weights directly in block form (no float pass: a 7B model takes
    seconds). Scales are chosen so the dequantized weights have roughly the requested std."""
    t = GGMLType(ggml_type)
    n = n_rows * k
    if t in (GGMLType.F32, GGMLType.F16, GGMLType.BF16):
        return quantize(rng.standard_normal(n, dtype=np.float32) * std, t)
    blk, nb = BLOCK_GEOMETRY[t]
    nblk = n // blk
    out = np.frombuffer(rng.bytes(nblk * nb), dtype=np.uint8).reshape(nblk, nb).copy()
    if t in (GGMLType.Q4_0,):
        d = np.full(nblk, std / 4.6, np.float32) * rng.uniform(0.75, 1.25, nblk).astype(np.float32)
        out[:, 0:2] = _to_f16_bytes(d)
    elif t == GGMLType.Q8_0:
        d = np.full(nblk, std / 73.0, np.float32) * rng.uniform(0.75, 1.25, nblk).astype(np.float32)
        out[:, 0:2] = _to_f16_bytes(d)
    elif t == GGMLType.Q4_K:
        # q uniform in 0..15 (std 4.6); sc in 32..63, m chosen to centre at zero
        d = (std / 4.6 / 47.0) * rng.uniform(0.8, 1.2, nblk).astype(np.float32)
        sc = rng.integers(32, 64, size=(nblk, 8)).astype(np.float32)
        dmin = d * 7.5 * 64.0 / 63.0
        m = np.clip(np.rint(sc * d[:, None] * 7.5 / dmin[:, None]), 0, 63)
        out[:, 0:2] = _to_f16_bytes(d)
        out[:, 2:4] = _to_f16_bytes(dmin)
        out[:, 4:16] = pack_q4k_scales(sc, m)
    elif t == GGMLType.Q5_K:
        # q uniform in 0..31 (std 9.2); sc in 32..63, m chosen to centre at zero
        d = (std / 9.2 / 47.0) * rng.uniform(0.8, 1.2, nblk).astype(np.float32)
        sc = rng.integers(32, 64, size=(nblk, 8)).astype(np.float32)
        dmin = d * 15.5 * 64.0 / 63.0
        m = np.clip(np.rint(sc * d[:, None] * 15.5 / dmin[:, None]), 0, 63)
        out[:, 0:2] = _to_f16_bytes(d)
        out[:, 2:4] = _to_f16_bytes(dmin)
        out[:, 4:16] = pack_q4k_scales(sc, m)
    elif t == GGMLType.Q6_K:
        d = (std / 18.5 / 96.0) * rng.uniform(0.8, 1.2, nblk).astype(np.float32)
        sc = rng.integers(64, 128, size=(nblk, 16)).astype(np.int8)
        out[:, 192:208] = sc.view(np.uint8)
        out[:, 208:210] = _to_f16_bytes(d)
    else:
        raise NotImplementedError(t.name)
    return out.reshape(-1)


# ----------------------------------------------------------------------------------------------
# device repack (block form -> GEMV streams, layout v2). Inverse provided for tests.
#
# K is padded to SB = ceil(K/256) super-blocks of 256 weights (zero blocks; only Q4_0/Q8_0 rows can
# need it). A "piece" is the 32 weights one lane consumes with one 16-B load; super-block `sb` holds
# pieces t = 0..7. Quant codes are stored piece-major *across* super-blocks,
#     qs[row][t][sb][16 B]     (Q8_0: 32 B, Q6_K high bits: 8 B)
# so the 16 lanes of a row group (lane s owns super-blocks s, s+16, ...) read one contiguous 256 B
# run per load instruction, while each lane's piece index t is a compile-time constant -- the
# per-super-block scales are decoded once per 256 weights instead of once per piece
# (csrc/kernels/gemv.hip). Scales / mins stay per super-block: meta[row][sb][16 B].
# 4-bit codes store the HIGH nibble of every byte as a signed two's-complement (n - 8) (byte ^ 0x80),
# so `q & 0xF0F0F0F0` is directly 16*(n-8) as int8 for v_dot4_i32_i8 (one VALU op, no shift).
# Q5_K codes are stored unsigned (no ^0x80: the kernels shift the high nibble down and OR in bit 4).
# Q5_K high bits are regrouped per piece into one dword H: byte j holds the bits of the piece's lo
# weights j, 4+j, 8+j, 12+j at bits 0-3 and of its hi weights at bits 4-7, so `(H << (4 - k)) & 0x10101010`
# is bit 4 of the k-th dword of lo codes (hi: `(H >> k) & 0x10101010`).
# Q6_K high bits are regrouped per piece: byte j of dword H0 (lo half) / H1 (hi half) holds the
# 2-bit fields of weights j, 4+j, 8+j, 12+j at bits 0-1, 2-3, 4-5, 6-7.
# ----------------------------------------------------------------------------------------------

REPACK_TYPES = (GGMLType.Q4_0, GGMLType.Q8_0, GGMLType.Q4_K, GGMLType.Q5_K, GGMLType.Q6_K)
REPACK_STREAMS = {GGMLType.Q4_K: ["qs", "meta"], GGMLType.Q5_K: ["qs", "meta", "qh"],
                  GGMLType.Q6_K: ["ql", "qh", "sc", "d"],
                  GGMLType.Q4_0: ["qs", "d"], GGMLType.Q8_0: ["qs", "d"]}


def n_superblocks(k: int) -> int:
    return (k + 255) // 256


def repack_row_bytes(ggml_type: int, k: int) -> list[int]:
    """Bytes per row of each repacked stream (order of REPACK_STREAMS)."""
    sb = n_superblocks(k)
    t = GGMLType(ggml_type)
    if t == GGMLType.Q4_K:
        return [128 * sb, 16 * sb]
    if t == GGMLType.Q5_K:
        return [128 * sb, 16 * sb, 32 * sb]
    if t == GGMLType.Q6_K:
        return [128 * sb, 64 * sb, 16 * sb, 2 * sb]
    if t == GGMLType.Q4_0:
        return [128 * sb, 16 * sb]
    if t == GGMLType.Q8_0:
        return [256 * sb, 16 * sb]
    raise ValueError(f"no device layout for {t.name}")


def _q5k_qh_split(qh: np.ndarray) -> np.ndarray:
    """qh [..., 32] (ggml order: bit j of qh[l] = high bit of weight l of sub-block j)
    -> [..., 8 pieces, 4 B] (piece t = 2c + h: lo = sub-block 2c, hi = 2c + 1, weights l = 16h + i)."""
    q = qh.astype(np.uint32)
    out = np.zeros(qh.shape[:-1] + (8, 4), np.uint32)
    for t in range(8):
        c, h = t >> 1, t & 1
        for i in range(16):
            j, k = i & 3, i >> 2
            out[..., t, j] |= ((q[..., 16 * h + i] >> (2 * c)) & 1) << k
            out[..., t, j] |= ((q[..., 16 * h + i] >> (2 * c + 1)) & 1) << (4 + k)
    return out.astype(np.uint8)


def _q5k_qh_join(hp: np.ndarray) -> np.ndarray:
    """inverse of _q5k_qh_split: [..., 8, 4] -> [..., 32]."""
    h = hp.astype(np.uint32)
    q = np.zeros(hp.shape[:-2] + (32,), np.uint32)
    for t in range(8):
        c, hh = t >> 1, t & 1
        for i in range(16):
            j, k = i & 3, i >> 2
            q[..., 16 * hh + i] |= ((h[..., t, j] >> k) & 1) << (2 * c)
            q[..., 16 * hh + i] |= ((h[..., t, j] >> (4 + k)) & 1) << (2 * c + 1)
    return q.astype(np.uint8)


def _q6k_qh_split(qh: np.ndarray) -> np.ndarray:
    """qh [..., 64] (ggml order) -> [..., 8 pieces, 8 B] (H0 | H1 per piece)."""
    q = qh.reshape(qh.shape[:-1] + (2, 32)).astype(np.uint32)   # [.., n, l]
    out = np.zeros(qh.shape[:-1] + (2, 4, 2, 4), np.uint32)     # [.., n, sub, half, byte j]
    for sub in range(4):
        lsel = q[..., (sub & 1) * 16:(sub & 1) * 16 + 16]      # [.., n, 16] weight i
        for half in range(2):
            f = (sub >> 1) + 2 * half                           # field of qh holding this weight
            bits = (lsel >> (2 * f)) & 3                        # [.., n, i]
            for k in range(4):
                out[..., sub, half, :] |= bits[..., 4 * k:4 * k + 4] << (2 * k)
    return out.astype(np.uint8).reshape(qh.shape[:-1] + (8, 8))


def _q6k_qh_join(h: np.ndarray) -> np.ndarray:
    """inverse of _q6k_qh_split: [..., 8, 8] -> [..., 64]."""
    h = h.reshape(h.shape[:-2] + (2, 4, 2, 4)).astype(np.uint32)
    q = np.zeros(h.shape[:-4] + (2, 32), np.uint32)
    for sub in range(4):
        for half in range(2):
            f = (sub >> 1) + 2 * half
            for k in range(4):
                bits = (h[..., sub, half, :] >> (2 * k)) & 3      # [.., n, j]
                q[..., (sub & 1) * 16 + 4 * k:(sub & 1) * 16 + 4 * k + 4] |= bits << (2 * f)
    return q.astype(np.uint8).reshape(h.shape[:-4] + (64,))


def repack(raw: np.ndarray, ggml_type: int, n_rows: int, k: int) -> dict[str, np.ndarray]:
    t = GGMLType(ggml_type)
    blk, nb = BLOCK_GEOMETRY[t]
    if k % blk:
        raise ValueError(f"K={k} not a multiple of {blk} for {t.name}")
    sb = n_superblocks(k)
    b = np.ascontiguousarray(raw).view(np.uint8).reshape(n_rows, k // blk, nb)
    if blk == 32 and k % 256:  # pad Q4_0 / Q8_0 rows to whole super-blocks with zero blocks
        b = np.concatenate([b, np.zeros((n_rows, sb * 8 - k // 32, nb), np.uint8)], axis=1)

    def pm(x, w):  # [rows, sb, 8, w] -> piece-major [rows, 8 * sb * w]
        return np.ascontiguousarray(x.reshape(n_rows, sb, 8, w).transpose(0, 2, 1, 3)).reshape(n_rows, -1)

    if t == GGMLType.Q4_K:
        return {"qs": pm(b[:, :, 16:144] ^ 0x80, 16),
                "meta": np.ascontiguousarray(b[:, :, 0:16]).reshape(n_rows, 16 * sb)}
    if t == GGMLType.Q5_K:
        return {"qs": pm(b[:, :, 48:176], 16),
                "meta": np.ascontiguousarray(b[:, :, 0:16]).reshape(n_rows, 16 * sb),
                "qh": pm(_q5k_qh_split(b[:, :, 16:48]), 4)}
    if t == GGMLType.Q6_K:
        return {"ql": pm(b[:, :, 0:128], 16),
                "qh": pm(_q6k_qh_split(b[:, :, 128:192]), 8),
                "sc": np.ascontiguousarray(b[:, :, 192:208]).reshape(n_rows, 16 * sb),
                "d": np.ascontiguousarray(b[:, :, 208:210]).reshape(n_rows, 2 * sb)}
    if t == GGMLType.Q4_0:
        return {"qs": pm(b[:, :, 2:18] ^ 0x80, 16),
                "d": np.ascontiguousarray(b[:, :, 0:2]).reshape(n_rows, 16 * sb)}
    if t == GGMLType.Q8_0:
        return {"qs": pm(b[:, :, 2:34], 32),
                "d": np.ascontiguousarray(b[:, :, 0:2]).reshape(n_rows, 16 * sb)}
    raise NotImplementedError(f"repack {t.name}")


def unrepack(streams: dict[str, np.ndarray], ggml_type: int, n_rows: int, k: int) -> np.ndarray:
    t = GGMLType(ggml_type)
    blk, nb = BLOCK_GEOMETRY[t]
    sb = n_superblocks(k)
    s = {n: np.asarray(v).reshape(n_rows, -1) for n, v in streams.items()}

    def bm(x, w):  # piece-major -> [rows, sb, 8 * w]
        return x.reshape(n_rows, 8, sb, w).transpose(0, 2, 1, 3).reshape(n_rows, sb, 8 * w)

    if t in (GGMLType.Q4_K, GGMLType.Q5_K, GGMLType.Q6_K):
        out = np.empty((n_rows, sb, nb), np.uint8)
        if t == GGMLType.Q4_K:
            out[:, :, 0:16] = s["meta"].reshape(n_rows, sb, 16)
            out[:, :, 16:144] = bm(s["qs"], 16) ^ 0x80
        elif t == GGMLType.Q5_K:
            out[:, :, 0:16] = s["meta"].reshape(n_rows, sb, 16)
            out[:, :, 16:48] = _q5k_qh_join(bm(s["qh"], 4).reshape(n_rows, sb, 8, 4))
            out[:, :, 48:176] = bm(s["qs"], 16)
        else:
            out[:, :, 0:128] = bm(s["ql"], 16)
            out[:, :, 128:192] = _q6k_qh_join(bm(s["qh"], 8).reshape(n_rows, sb, 8, 8))
            out[:, :, 192:208] = s["sc"].reshape(n_rows, sb, 16)
            out[:, :, 208:210] = s["d"].reshape(n_rows, sb, 2)
        return out.reshape(-1)
    out = np.empty((n_rows, sb * 8, nb), np.uint8)
    out[:, :, 0:2] = s["d"].reshape(n_rows, sb * 8, 2)
    if t == GGMLType.Q4_0:
        out[:, :, 2:18] = bm(s["qs"], 16).reshape(n_rows, sb * 8, 16) ^ 0x80
    else:
        out[:, :, 2:34] = bm(s["qs"], 32).reshape(n_rows, sb * 8, 32)
    return np.ascontiguousarray(out[:, : k // blk]).reshape(-1)
