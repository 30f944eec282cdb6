"""Device weight loader: GGUF -> repacked quant streams in HBM.

Every projection is uploaded as a `DevQMat` (csrc/kernels/qmat.h) laid out for the fused GEMV:
  * q/k/v rows concatenated into one matrix when they share a quant type (one QKV launch);
  * phi2 q/k rows re-ordered inside each head so NEOX rotary pairs (i, i + n_rot/2) become
    adjacent rows (the GEMV epilogue only rotates adjacent pairs) -- q.k dot products unchanged;
  * gate/up rows interleaved (row 2j = gate j, 2j+1 = up j) so SiLU-GLU fuses into the epilogue;
  * tensor-parallel shards cut on head / row / 256-weight-block boundaries;
  * MoE experts stacked [X][N][K] so the kernel offsets to the routed expert on device.
Types without a native kernel (Q4_1/Q5_0/Q5_1/F16/BF16/F32 projections) are requantised to Q8_0 at
load -- documented precision upgrade for those files, never a silent fallback.
Host staging goes through the native repack (`_C.GGUFMap.repack`, multi-threaded over the mmap).
"""
from __future__ import annotations

import os
from dataclasses import dataclass, field

import numpy as np
import torch

from ..gguf import GGMLType, read_gguf
from ..gguf.constants import BLOCK_GEOMETRY
from ..models.config import ROPE_NEOX, ModelConfig
from ..quant import REPACK_STREAMS, dequantize, quantize, repack_row_bytes
from ..ops import has_native, native

NATIVE_QTYPES = (GGMLType.Q4_0, GGMLType.Q8_0, GGMLType.Q4_K, GGMLType.Q5_K, GGMLType.Q6_K)


def stream_bytes(qtype: int, K: int) -> list[int]:
    """Per-row bytes of each device stream (layout v2, quant.repack)."""
    return repack_row_bytes(qtype, K)


@dataclass
class DevQMat:
    qtype: int
    N: int
    K: int
    streams: list[torch.Tensor] = field(default_factory=list)
    # Q6_K only, GPU: codes widened to signed int8 at load for the batch-1 GEMV (qmat.h QT_Q6_K8)
    wide: torch.Tensor | None = None
    # GPU, continuous batching: layout M copy for the matrix-core batched decode GEMV (gemv_mfma.hip)
    mt: torch.Tensor | None = None

    @property
    def tup(self) -> tuple:
        p = [s.data_ptr() for s in self.streams] + [0] * (4 - len(self.streams))
        t = (p[0], p[1], p[2], p[3], self.N, self.K, int(self.qtype))
        wide = self.wide.data_ptr() if self.wide is not None else 0
        if self.mt is not None:
            return t + (wide, self.mt.data_ptr())
        return t + (wide,) if self.wide is not None else t

    def build_mfma_layout(self) -> int:
        """Layout M copy (gemv_mfma.hip `repack_m`, built on the device from the v2 streams) for the
        batched decode GEMV; returns its bytes (0: this quant type has no layout M)."""
        from ..ops import native, stream_handle
        if self.mt is not None:
            return self.mt.numel()
        n = native().mfma_layout_bytes(int(self.qtype), self.N, self.K)
        if n:
            self.mt = torch.empty(n, dtype=torch.uint8, device=self.streams[0].device)
            native().repack_m(self.tup, self.mt.data_ptr(), stream_handle())
        return n

    @property
    def nbytes(self) -> int:
        return sum(s.numel() for s in self.streams)


def _np_repack_rows(src: np.ndarray, qtype: int, K_src: int, rows: np.ndarray, dst_rows: np.ndarray,
                    kb0: int, kb1: int, dst: list[np.ndarray], K_out: int = 0) -> None:
    """numpy twin of csrc/gguf/gguf.cpp repack_rows (CPU-only environments / tests). K_out > K: the
    destination rows are K_out wide (zero super-blocks past K, every stream's stride grown to match)."""
    from ..quant import repack
    blk, nb = BLOCK_GEOMETRY[GGMLType(qtype)]
    b = src.reshape(-1, K_src // blk, nb)[rows][:, kb0:kb1]
    K = (kb1 - kb0) * blk
    st = repack(b.reshape(-1), qtype, len(rows), K)
    sb, sbo = (K + 255) // 256, (max(K, K_out) + 255) // 256
    for i, n in enumerate(REPACK_STREAMS[GGMLType(qtype)]):
        a = st[n]
        if sbo > sb:  # per-row streams are [8 pieces][SB][w] (codes) or [SB][w] (scales): pad the SB axis
            w = a.shape[1] // sb
            piece_major = n in ("qs", "ql", "qh")
            if piece_major:
                a3 = a.reshape(len(rows), 8, sb, w // 8)
                a = np.concatenate([a3, np.zeros((len(rows), 8, sbo - sb, w // 8), a.dtype)], 2).reshape(len(rows), -1)
            else:
                a = np.concatenate([a, np.zeros((len(rows), (sbo - sb) * w), a.dtype)], 1)
        dst[i].reshape(-1, a.shape[1])[dst_rows] = a


class WeightSource:
    """Reads tensors from a GGUF file (native mmap + repack when built, numpy otherwise)."""

    def __init__(self, path: str):
        self.path = path
        self.g = read_gguf(path)
        self.cfg = ModelConfig.from_gguf_metadata(self.g.metadata)
        self.nat = native().GGUFMap(path) if has_native() else None
        self.threads = min(16, os.cpu_count() or 4)
        self._requant: dict[str, np.ndarray] = {}

    def info(self, name: str):
        return self.g.tensors[name]

    def has(self, name: str) -> bool:
        return name in self.g.tensors

    def f32(self, name: str) -> np.ndarray:
        return np.ascontiguousarray(self.g.array(name), dtype=np.float32).reshape(-1)

    def qtype_of(self, name: str) -> int:
        t = self.info(name).ggml_type
        return int(t) if t in NATIVE_QTYPES else int(GGMLType.Q8_0)

    def _requantized(self, name: str) -> np.ndarray:
        if name not in self._requant:
            t = self.info(name)
            x = dequantize(self.g.raw(name), t.ggml_type, t.n_elements)
            self._requant[name] = quantize(x, GGMLType.Q8_0)
        return self._requant[name]

    def repack_into(self, name: str, K_src: int, rows: np.ndarray, dst_rows: np.ndarray, kb0: int, kb1: int,
                    dst: list[np.ndarray], K_out: int = 0) -> None:
        t = self.info(name)
        rows = np.ascontiguousarray(rows, dtype=np.int64)
        dst_rows = np.ascontiguousarray(dst_rows, dtype=np.int64)
        if t.ggml_type in NATIVE_QTYPES:
            if self.nat is not None:
                self.nat.repack(name, rows, dst_rows, K_src, kb0, kb1, [d.ctypes.data for d in dst], self.threads,
                                K_out)
                if hasattr(self.nat, "release"):
                    self.nat.release(name)  # the blob's pages leave RSS as soon as their copy exists
            else:
                _np_repack_rows(self.g.raw(name), int(t.ggml_type), K_src, rows, dst_rows, kb0, kb1, dst, K_out)
        else:
            src = self._requantized(name)
            if self.nat is not None:
                native().repack_ptr(src.ctypes.data, int(GGMLType.Q8_0), K_src, rows, dst_rows, kb0, kb1,
                                    [d.ctypes.data for d in dst], self.threads, K_out)
            else:
                _np_repack_rows(src, int(GGMLType.Q8_0), K_src, rows, dst_rows, kb0, kb1, dst, K_out)


_HUGE = 2 << 20


def host_buffer(nbytes: int, device) -> np.ndarray:
    """Zeroed uint8 host buffer for one weight stream. On the CPU backend the streams ARE the serving
    weights: they are placed on 2 MiB-aligned transparent huge pages (madvise), so the hardware
    prefetchers of the streaming int8 GEMM are not stopped at every 4 KiB page boundary and the
    1.6 GB of Phi-2 costs ~800 TLB entries instead of ~400k."""
    if str(device) != "cpu" or nbytes < _HUGE:
        return np.zeros(nbytes, np.uint8)
    raw = np.empty(nbytes + _HUGE, np.uint8)  # large np.empty: fresh anonymous mapping, untouched
    off = (-raw.ctypes.data) % _HUGE
    buf = raw[off:off + nbytes]  # fresh anonymous pages read as zero; every byte is then repacked
    try:
        import ctypes
        libc = ctypes.CDLL(None, use_errno=True)
        span = (nbytes + _HUGE - 1) // _HUGE * _HUGE
        libc.madvise(ctypes.c_void_p(buf.ctypes.data), ctypes.c_size_t(min(span, raw.nbytes - off)), 14)  # MADV_HUGEPAGE
    except (OSError, AttributeError):  # pragma: no cover - non-Linux
        pass
    return buf


def build_qmat(src: WeightSource, parts: list[tuple[str, np.ndarray, np.ndarray]], N: int, K_src: int,
               kb: tuple[int, int] | None, device, expert_rows: int = 0, widen: bool = False,
               k_pad: int = 0) -> DevQMat:
    """parts: (tensor, source rows, destination rows). All parts must share one device qtype.
    k_pad > K: the matrix is stored (and presented to the kernels) with K = k_pad, zero weights past the
    real K (the consumer's activation columns past it are zero too: DeviceWeights.ffn_pad)."""
    qts = {src.qtype_of(p[0]) for p in parts}
    if len(qts) != 1:
        raise ValueError(f"mixed quant types in one matrix: {qts}")
    qt = qts.pop()
    blk = BLOCK_GEOMETRY[GGMLType(qt)][0]
    kb0, kb1 = kb if kb is not None else (0, K_src // blk)
    K = max((kb1 - kb0) * blk, k_pad)
    sb = stream_bytes(qt, K)
    host = [host_buffer(N * b, device) for b in sb]
    for name, rows, drows in parts:
        src.repack_into(name, K_src, rows, drows, kb0, kb1, host, K)
    streams = [torch.from_numpy(h).to(device) for h in host]
    m = DevQMat(qt, expert_rows or N, K, streams)
    # opt-in (OMX_Q6K_WIDEN=1): Q6_K projections (down, V, O) get int8-widened codes for the batch-1
    # GEMV. Measured in the engine it loses: down 13.2 -> 14.6 us, the +30 % bytes cost more than the
    # 6-bit unpack it saves (profiles/r2_gemv/engine_widened_step.txt); kept as a tested knob
    if (widen and qt == int(GGMLType.Q6_K) and not expert_rows and str(device).startswith("cuda")
            and os.environ.get("OMX_Q6K_WIDEN", "0") == "1"):
        from ..ops import native, stream_handle
        m.wide = torch.empty(N * ((K + 255) // 256) * 256, dtype=torch.uint8, device=device)
        native().widen_q6k(m.tup, m.wide.data_ptr(), stream_handle())
    return m


def neox_pair_perm(D: int, n_rot: int) -> np.ndarray:
    """Row order inside one head that makes NEOX pairs (i, i + n_rot/2) adjacent."""
    half = n_rot // 2
    p = []
    for i in range(half):
        p += [i, i + half]
    return np.array(p + list(range(n_rot, D)), np.int64)


def rope_inv_freq(n_rot: int, base: float) -> np.ndarray:
    i = np.arange(n_rot // 2, dtype=np.float64)
    return (base ** (-2.0 * i / n_rot)).astype(np.float32)


def ffn_pad(F: int, device, tp: int, moe: bool) -> int:
    """Zero columns appended to ffn_down's K on the GPU (tp == 1, dense FFN) so its layout-v2 piece runs
    start on 256-B boundaries: piece t of a row sits at byte (t * SB + sb) * 16, so with SB % 8 != 0 every
    16-lane run of the decode GEMV straddles an extra 128-B line. Llama-2-7B's 11008 = 43 super-blocks is
    padded to 48 (+11.6 % storage; the r5 probe: down Q6_K 13.1 -> 10.9 us, Q4_K 8.9 -> 8.2 us at the padded
    K, profiles/r5_decode/align_full_*.log). OMX_FFN_PAD: auto (<= 12.5 % growth, SB % 8 != 0), force
    (any SB % 16 != 0; tests), 0 (off)."""
    mode = os.environ.get("OMX_FFN_PAD", "auto").strip().lower()
    if mode in ("0", "off") or tp != 1 or moe or not str(device).startswith("cuda"):
        return 0
    sb = (F + 255) // 256
    sb16 = (sb + 15) // 16 * 16
    if mode == "force":
        return sb16 * 256 - F if sb % 16 else 0
    if sb % 8 and sb16 * 8 <= sb * 9:
        return sb16 * 256 - F
    return 0


class DeviceWeights:
    """All weights of one model (one TP rank) resident on `device`."""

    def __init__(self, path: str, device: str | torch.device = "cuda", tp_rank: int = 0, tp_size: int = 1):
        self.src = src = WeightSource(path)
        cfg = self.full_cfg = src.cfg
        self.device = device
        self.tp_rank, self.tp_size = tp_rank, tp_size
        T, r = tp_size, tp_rank
        E, H, Hkv, D, F, V = cfg.n_embd, cfg.n_head, cfg.n_head_kv, cfg.head_dim, cfg.n_ff, cfg.n_vocab
        if H % T or Hkv % T or V % T:
            raise ValueError(f"tp={T} must divide heads ({H}/{Hkv}) and vocab ({V})")
        # FFN rows per rank: whole 256-weight super-blocks of the down projection's K, split as evenly
        # as they go -- Llama-2-7B's n_ff = 11008 is 43 super-blocks, so TP=2 ranks hold 22 / 21
        # (Megatron row-parallel needs no equal split: the all-reduce sums E-wide partials)
        f_unit = 256 if F % 256 == 0 else 32
        nbf = F // f_unit
        if F % f_unit or nbf < T or (cfg.n_expert and F % T):
            raise ValueError(f"tp={T} cannot split n_ff={F} on quant-block boundaries")
        f0, f1 = (r * nbf // T) * f_unit, ((r + 1) * nbf // T) * f_unit
        self.f_range = (f0, f1)
        Hl, Hkvl, Fl, Vl = H // T, Hkv // T, (f1 - f0) if not cfg.n_expert else F // T, V // T
        self.cfg = cfg
        self.ffn_pad = ffn_pad(Fl, device, T, bool(cfg.n_expert))
        # the executor's FFN width: the padded K of ffn_down (the gate/up rows stay Fl; the activation
        # columns past Fl are never written, so they stay zero, like the padded weights)
        self.local = dict(E=E, H=Hl, Hkv=Hkvl, D=D, F=Fl + self.ffn_pad, V=Vl)
        dev = device
        t = lambda a: torch.from_numpy(np.array(a, np.float32)).to(dev)  # noqa: E731
        phi = cfg.arch == "phi2"
        perm = neox_pair_perm(D, cfg.n_rot) if cfg.rope_mode == ROPE_NEOX else np.arange(D, dtype=np.int64)

        def head_rows(h0: int, nh: int, permute: bool) -> np.ndarray:
            base = (np.arange(h0, h0 + nh, dtype=np.int64)[:, None] * D)
            return (base + (perm if permute else np.arange(D))[None, :]).reshape(-1)

        def kblocks(K_full: int, name: str) -> tuple[int, int]:
            blk = BLOCK_GEOMETRY[GGMLType(src.qtype_of(name))][0]
            nb = K_full // blk
            if K_full == F and not cfg.n_expert:  # row-parallel over the (possibly uneven) FFN split
                if f0 % blk or f1 % blk:
                    raise ValueError(f"{name}: FFN split {f0}:{f1} not on {blk}-weight blocks")
                return (f0 // blk, f1 // blk)
            if nb % T:
                raise ValueError(f"{name}: {nb} blocks of {blk} not divisible by tp={T}")
            return (r * nb // T, (r + 1) * nb // T)

        ar = lambda n, off=0: np.arange(off, off + n, dtype=np.int64)  # noqa: E731
        self.tok_embd = build_qmat(src, [("token_embd.weight", ar(V), ar(V))], V, E, None, dev)
        self.layers = []
        Eq, Ekv = Hl * D, Hkvl * D
        for i in range(cfg.n_layer):
            b = f"blk.{i}."
            L: dict = {}
            if phi:
                qkv = b + "attn_qkv.weight"
                rq = head_rows(r * Hl, Hl, True)
                rk = E + head_rows(r * Hkvl, Hkvl, True)
                rv = E + Hkv * D + head_rows(r * Hkvl, Hkvl, False)
                rows = np.concatenate([rq, rk, rv])
                L["wqk"] = build_qmat(src, [(qkv, rows, ar(len(rows)))], Eq + 2 * Ekv, E, None, dev)
                L["qkv_bias"] = t(src.f32(b + "attn_qkv.bias")[rows])
                L["attn_norm"] = t(src.f32(b + "attn_norm.weight"))
                L["attn_norm_b"] = t(src.f32(b + "attn_norm.bias"))
                L["wo"] = build_qmat(src, [(b + "attn_output.weight", ar(E), ar(E))], E, E,
                                     kblocks(E, b + "attn_output.weight"), dev, widen=True)
                L["bo"] = t(src.f32(b + "attn_output.bias")) if r == 0 else None
                L["wgu"] = build_qmat(src, [(b + "ffn_up.weight", ar(Fl, f0), ar(Fl))], Fl, E, None, dev)
                L["bup"] = t(src.f32(b + "ffn_up.bias")[f0:f1])
                L["wdown"] = build_qmat(src, [(b + "ffn_down.weight", ar(E), ar(E))], E, F,
                                        kblocks(F, b + "ffn_down.weight"), dev, widen=True,
                                        k_pad=Fl + self.ffn_pad)
                L["bdown"] = t(src.f32(b + "ffn_down.bias")) if r == 0 else None
            else:
                rq = head_rows(r * Hl, Hl, cfg.rope_mode == ROPE_NEOX)
                rk = head_rows(r * Hkvl, Hkvl, cfg.rope_mode == ROPE_NEOX)
                rv = head_rows(r * Hkvl, Hkvl, False)
                nq, nk, nv = b + "attn_q.weight", b + "attn_k.weight", b + "attn_v.weight"
                if src.qtype_of(nq) == src.qtype_of(nk) == src.qtype_of(nv):
                    L["wqk"] = build_qmat(src, [(nq, rq, ar(Eq)), (nk, rk, ar(Ekv, Eq)), (nv, rv, ar(Ekv, Eq + Ekv))],
                                          Eq + 2 * Ekv, E, None, dev)
                else:
                    L["wqk"] = build_qmat(src, [(nq, rq, ar(Eq)), (nk, rk, ar(Ekv, Eq))], Eq + Ekv, E, None, dev)
                    L["wv"] = build_qmat(src, [(nv, rv, ar(Ekv))], Ekv, E, None, dev, widen=True)
                L["attn_norm"] = t(src.f32(b + "attn_norm.weight"))
                L["ffn_norm"] = t(src.f32(b + "ffn_norm.weight"))
                Eq_full = cfg.n_embd_q  # O projection K = H * head_dim (Gemma: != E)
                L["wo"] = build_qmat(src, [(b + "attn_output.weight", ar(E), ar(E))], E, Eq_full,
                                     kblocks(Eq_full, b + "attn_output.weight"), dev, widen=True)
                if cfg.n_expert:
                    X = cfg.n_expert
                    L["router"] = build_qmat(src, [(b + "ffn_gate_inp.weight", ar(X), ar(X))], X, E, None, dev)
                    gparts = []
                    for e in range(X):
                        loc = ar(Fl, e * F + r * Fl)
                        gparts.append((b + "ffn_gate_exps.weight", loc, e * 2 * Fl + 2 * ar(Fl)))
                        gparts.append((b + "ffn_up_exps.weight", loc, e * 2 * Fl + 2 * ar(Fl) + 1))
                    L["gu_exps"] = build_qmat(src, gparts, X * 2 * Fl, E, None, dev, expert_rows=2 * Fl)
                    L["down_exps"] = build_qmat(src, [(b + "ffn_down_exps.weight", ar(X * E), ar(X * E))], X * E, F,
                                                kblocks(F, b + "ffn_down_exps.weight"), dev, expert_rows=E)
                else:
                    ng, nu = b + "ffn_gate.weight", b + "ffn_up.weight"
                    loc = ar(Fl, f0)
                    L["wgu"] = build_qmat(src, [(ng, loc, 2 * ar(Fl)), (nu, loc, 2 * ar(Fl) + 1)], 2 * Fl, E, None, dev)
                    L["wdown"] = build_qmat(src, [(b + "ffn_down.weight", ar(E), ar(E))], E, F,
                                            kblocks(F, b + "ffn_down.weight"), dev, widen=True,
                                            k_pad=Fl + self.ffn_pad)
            self.layers.append(L)
        self.out_norm = t(src.f32("output_norm.weight"))
        self.out_norm_b = t(src.f32("output_norm.bias")) if src.has("output_norm.bias") else None
        out_name = "output.weight" if src.has("output.weight") else "token_embd.weight"  # tied embeddings
        self.lm_head = build_qmat(src, [(out_name, ar(Vl, r * Vl), ar(Vl))], Vl, E, None, dev)
        self.lm_bias = t(src.f32("output.bias")[r * Vl:(r + 1) * Vl]) if src.has("output.bias") else None
        self.inv_freq = t(rope_inv_freq(cfg.n_rot, cfg.rope_base))
        self.lm_c1 = self.lm_c2 = None
        if phi and T == 1 and str(dev).startswith("cuda") and os.environ.get("OMX_X8_LN", "1") != "0":
            self._ln_consts()
        # the GGUF mapping (and any requantised copies) is no longer needed: dropping it releases the
        # file's resident pages (a CPU server would otherwise hold the blob twice in RSS)
        self.src = None

    def _ln_consts(self) -> None:
        """Phi-2 int8 decode chain (executor.cpp ln8): the LayerNorm constants c1 = W . ln_w and
        c2 = W . ln_b of every LayerNorm'd consumer (QKV and FFN up with attn_norm, the LM head with
        output_norm), so the GEMV computes W . LN(x) = rstd * (W . (x * ln_w) - mu * c1) + c2 from the
        producer's int8 image of x * ln_w. W is this matrix as stored (fp16-dequantised on the device,
        gemm.hip's dequant_f16), the dot products in fp32."""
        from ..ops import stream_handle
        C = native()
        dev = self.device

        def consts(q: "DevQMat", w: torch.Tensor, b: torch.Tensor | None):
            buf = torch.empty(q.N, q.K, dtype=torch.float16, device=dev)
            C.dequant_f16(q.tup, buf.data_ptr(), stream_handle(), 0)
            c1 = torch.empty(q.N, dtype=torch.float32, device=dev)
            c2 = torch.zeros(q.N, dtype=torch.float32, device=dev)
            for r0 in range(0, q.N, 8192):
                blk = buf[r0:r0 + 8192].float()
                c1[r0:r0 + 8192] = blk @ w
                if b is not None:
                    c2[r0:r0 + 8192] = blk @ b
            return c1, c2

        for L in self.layers:
            L["c1_qkv"], L["c2_qkv"] = consts(L["wqk"], L["attn_norm"], L["attn_norm_b"])
            L["c1_up"], L["c2_up"] = consts(L["wgu"], L["attn_norm"], L["attn_norm_b"])
        if self.out_norm_b is not None:
            self.lm_c1, self.lm_c2 = consts(self.lm_head, self.out_norm, self.out_norm_b)

    def build_mfma_layouts(self) -> int:
        """Layout M copies of every dense projection (+ LM head) for continuous-batching decode steps
        on the matrix cores; MoE expert stacks keep the routed int8 GEMV. Returns the bytes added."""
        n = self.lm_head.build_mfma_layout()
        for L in self.layers:
            for k, v in L.items():
                if isinstance(v, DevQMat) and k not in ("gu_exps", "down_exps"):
                    n += v.build_mfma_layout()
        return n

    @property
    def nbytes(self) -> int:
        n = self.tok_embd.nbytes + self.lm_head.nbytes
        for L in self.layers:
            for v in L.values():
                if isinstance(v, DevQMat):
                    n += v.nbytes
        return n
