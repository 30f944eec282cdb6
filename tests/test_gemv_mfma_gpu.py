"""GPU numerics of the batched matrix-core decode GEMV (csrc/kernels/gemv_mfma.hip, layout M) against
a plain fp32 PyTorch GEMV on the dequantised weights: every quant type with a layout M, B = 2..16,
K with and without super-block padding, partial row tiles, and the fused prologue / epilogues."""
import math

import numpy as np
import pytest
import torch

from ollama_operator_amd.gguf import GGMLType
from test_kernels_gpu import QM, C, S, gemv, rel

pytestmark = pytest.mark.gpu

MB_TYPES = [GGMLType.Q4_0, GGMLType.Q8_0, GGMLType.Q4_K, GGMLType.Q6_K]


class QMM(QM):
    """QM plus its layout M copy (built on the device from the v2 streams by repack_m)."""

    def __init__(self, qt, N, K, seed=0, zero_mt=False):
        super().__init__(qt, N, K, seed)
        n = C().mfma_layout_bytes(int(qt), N, K)
        assert n > 0
        self.mt = torch.zeros(n, dtype=torch.uint8, device="cuda")
        if not zero_mt:
            C().repack_m(self.tup, self.mt.data_ptr(), S())
        self.tup = self.tup + (0, self.mt.data_ptr())


@pytest.mark.parametrize("qt", MB_TYPES)
@pytest.mark.parametrize("B", [3, 4, 7, 16])
@pytest.mark.parametrize("K", [256, 2080, 4096, 11008])
def test_mb_store(qt, B, K):
    if K == 2080 and qt in (GGMLType.Q4_K, GGMLType.Q6_K):
        K = 2304  # K-quants: whole super-blocks; 2080 = 65 Q4_0/Q8_0 blocks exercises the padding
    if K == 11008 and B > 6:
        B = 6  # > 6 fp16 rows of K = 11008 exceed the block's LDS: that shape keeps the int8 GEMV
    N = 400  # 25 row tiles, the last one partial
    m = QMM(qt, N, K, seed=K + B)
    x = torch.randn(B, K, device="cuda")
    y = torch.zeros(B, N, device="cuda")
    gemv(m, x, y=y)
    ref = x @ m.w.T
    assert rel(y, ref) < 4e-3, (qt, B, K)


@pytest.mark.parametrize("qt", MB_TYPES)
def test_mb_path_is_taken(qt):
    """A zeroed layout M copy must zero the output: the batched step reads layout M, not v2."""
    m = QMM(qt, 64, 512, seed=1, zero_mt=True)
    x = torch.randn(4, 512, device="cuda")
    y = torch.full((4, 64), 7.0, device="cuda")
    gemv(m, x, y=y)
    assert float(y.abs().max()) == 0.0
    C().set_mb_enable(0)  # the int8 GEMV ignores layout M
    try:
        gemv(m, x, y=y)
    finally:
        C().set_mb_enable(1)
    assert rel(y, x @ m.w.T) < 1e-2


@pytest.mark.parametrize("qt", [GGMLType.Q4_K, GGMLType.Q6_K, GGMLType.Q4_0])
@pytest.mark.parametrize("B", [3, 16])
def test_mb_rmsnorm_add_bias(qt, B):
    N, K = 512, 4096
    m = QMM(qt, N, K, seed=3 + B)
    x = torch.randn(B, K, device="cuda") * 3
    nw = torch.rand(K, device="cuda") + 0.5
    bias = torch.randn(N, device="cuda")
    y0 = torch.randn(B, N, device="cuda")
    y = y0.clone()
    gemv(m, x, norm=1, nw=nw, epi=1, y=y, bias=bias)
    xn = x * torch.rsqrt(x.pow(2).mean(-1, keepdim=True) + 1e-5) * nw
    ref = y0 + xn @ m.w.T + bias
    assert rel(y - y0, ref - y0) < 4e-3


@pytest.mark.parametrize("epi", [2, 5])
def test_mb_glu(epi):
    F, K, B = 344, 4096, 5
    m = QMM(GGMLType.Q4_K, 2 * F, K, seed=5)
    x = torch.randn(B, K, device="cuda")
    nw = torch.rand(K, device="cuda") + 0.5
    y = torch.zeros(B, F, device="cuda")
    gemv(m, x, norm=1, nw=nw, epi=epi, y=y)
    xn = x * torch.rsqrt(x.pow(2).mean(-1, keepdim=True) + 1e-5) * nw
    gu = xn @ m.w.T
    if epi == 2:
        act = torch.nn.functional.silu(gu[:, 0::2])
    else:
        g = gu[:, 0::2]
        act = 0.5 * g * (1 + torch.tanh(math.sqrt(2 / math.pi) * (g + 0.044715 * g ** 3)))
    ref = act * gu[:, 1::2]
    assert rel(y, ref) < 5e-3


def test_mb_qkv_matches_int8_gemv():
    """The RoPE + paged KV scatter epilogue from the matrix-core kernel against the int8 GEMV."""
    H, Hkv, D, n_rot, K, B, bs = 8, 2, 128, 128, 1024, 6, 16
    Eq, Ekv = H * D, Hkv * D
    N = Eq + 2 * Ekv
    m = QMM(GGMLType.Q4_K, N, K, seed=9)
    x = torch.randn(B, K, device="cuda")
    nw = torch.rand(K, device="cuda") + 0.5
    inv = (10000.0 ** (-torch.arange(0, n_rot // 2, dtype=torch.float64) * 2 / n_rot)).float().cuda()
    pos = torch.tensor([0, 17, 40, 3, 99, 250], device="cuda", dtype=torch.int32)
    slot = torch.tensor([5, 3 * bs + 1, 7 * bs + 15, 2 * bs, 9 * bs + 3, 11 * bs + 7], device="cuda", dtype=torch.int32)
    outs = []
    for on in (1, 0):
        q = torch.zeros(B, Eq, device="cuda")
        kc = torch.zeros(12, Hkv, bs, D, device="cuda", dtype=torch.float16)
        vc = torch.zeros_like(kc)
        extra = dict(pos=pos.data_ptr(), slot=slot.data_ptr(), kc=kc.data_ptr(), vc=vc.data_ptr(),
                     inv_freq=inv.data_ptr(), Eq=Eq, Ekv=Ekv, D=D, n_rot=n_rot, n_kv=Hkv, bs=bs)
        C().set_mb_enable(on)
        try:
            gemv(m, x, norm=1, nw=nw, epi=4, y=q, extra=extra)
        finally:
            C().set_mb_enable(1)
        torch.cuda.synchronize()
        outs.append((q.clone(), kc.float().clone(), vc.float().clone()))
    for a, b in zip(outs[0], outs[1]):
        assert b.abs().sum() > 0
        assert rel(a, b) < 1.5e-2


def test_mb_layout_bytes():
    assert C().mfma_layout_bytes(int(GGMLType.Q4_K), 4096, 4096) == 256 * 16 * 2304
    assert C().mfma_layout_bytes(int(GGMLType.Q6_K), 4000, 11008) == 250 * 43 * 3360
    assert C().mfma_layout_bytes(int(GGMLType.Q8_0), 17, 288) == 2 * 2 * 4352
    assert C().mfma_layout_bytes(int(GGMLType.Q5_K), 4096, 4096) == 0


@pytest.mark.parametrize("B", [3, 4, 8, 16])
def test_mb_engine_batched_decode(tiny_models, B):
    """Engine level: a continuous-batching step with layout M equals the int8-GEMV step."""
    from ollama_operator_amd.engine.runner import Runner
    g = Runner(tiny_models["tiny-llama"], device="cuda", max_batch=32, max_seqs=16, ctx=256)
    assert g.mfma_bytes > 0
    assert g.exe.exe.mb_chain  # every projection takes the fp16 matrix-core chain
    rng = np.random.default_rng(B)
    prompts = [[1] + [int(v) for v in rng.integers(3, 500, 10 + 7 * b)] for b in range(B)]
    sids = []
    for p in prompts:
        sid = g.new_sequence()
        g.prefill(sid, p)
        sids.append(sid)
    V = g.cfg.n_vocab
    outs = []
    for on in (1, 0):
        C().set_mb_enable(on)
        try:
            g.set_tokens(list(range(7, 7 + B)))
            g.decode_batch(sids, [len(p) for p in prompts])
            torch.cuda.synchronize()
        finally:
            C().set_mb_enable(1)
        outs.append(g.logits[:B, :V].float().cpu().clone())
    assert rel(outs[0], outs[1]) < 2e-2


def f16_rows(x, ld, zero_rows=1):
    """fp16 activation buffer [B + zero_rows][ld] (row B..: zeros) as the chain buffers are laid out."""
    B, K = x.shape
    out = torch.zeros(B + zero_rows, ld, device="cuda", dtype=torch.float16)
    out[:B, :K] = x.half()
    return out


@pytest.mark.parametrize("qt", MB_TYPES)
@pytest.mark.parametrize("B,K", [(3, 4096), (5, 4096), (16, 2048), (4, 11008), (9, 11008)])
def test_mb_fp16_input_with_rms_partials(qt, B, K):
    """Consumer side of the chain: activations fp16(x * norm_w) from global memory, the RMSNorm scale
    from per-16-row sum-of-squares partials (as a producer's epilogue leaves them)."""
    N = 400
    m = QMM(qt, N, K, seed=K + B + 7)
    x = torch.randn(B, K, device="cuda") * 2
    nw = torch.rand(K, device="cuda") + 0.5
    ld = (K + 255) // 256 * 256
    x16 = f16_rows(x * nw, ld)
    parts = torch.zeros(16, K // 16, device="cuda")  # [batch row][16-row tile] as producers write them
    parts[:B] = x.pow(2).reshape(B, K // 16, 16).sum(-1)
    y = torch.zeros(B, N, device="cuda")
    gemv(m, x, norm=1, nw=nw, y=y, extra=dict(x16=x16.data_ptr(), ld16=ld, zrow16=B, xstat=parts.data_ptr(),
                                              xstat_n=K // 16))
    xn = x * torch.rsqrt(x.pow(2).mean(-1, keepdim=True) + 1e-5) * nw
    assert rel(y, xn @ m.w.T) < 4e-3, (qt, B, K)


@pytest.mark.parametrize("B", [3, 12])
def test_mb_residual_emission(B):
    """Producer side: the EPI_ADD epilogue also emits fp16(new resid * next norm_w) and the per-tile
    sum-of-squares partials of the new residual."""
    N, K = 1024, 4096
    m = QMM(GGMLType.Q4_K, N, K, seed=B)
    x = torch.randn(B, K, device="cuda")
    resid0 = torch.randn(B, N, device="cuda") * 4
    resid = resid0.clone()
    nw_next = torch.rand(N, device="cuda") + 0.5
    e16 = torch.zeros(B + 1, N, device="cuda", dtype=torch.float16)
    st = torch.full((16, N // 16), -1.0, device="cuda")
    gemv(m, x, epi=1, y=resid, extra=dict(emit16=e16.data_ptr(), ld_emit=N, emit_nw=nw_next.data_ptr(),
                                          emit_stat=st.data_ptr()))
    ref = resid0 + x @ m.w.T
    assert rel(resid, ref) < 4e-3
    assert rel(e16[:B].float(), (resid * nw_next)) < 1e-3
    assert float(e16[B].abs().max()) == 0.0
    got = st[:B].sum(1)
    assert torch.allclose(got, resid.pow(2).sum(-1), rtol=1e-4)
    assert float((st[B:] + 1).abs().max()) == 0.0  # rows >= B untouched


def test_mb_chain_matches_fused_norm():
    """producer (O-style residual add + emission) -> consumer (RMSNorm'd GEMV on the fp16 emission)
    equals the consumer reading the fp32 residual with its own fused RMSNorm."""
    B, E, F = 6, 4096, 512
    mo = QMM(GGMLType.Q4_K, E, E, seed=21)
    mg = QMM(GGMLType.Q6_K, F, E, seed=22)
    a = torch.randn(B, E, device="cuda")
    resid = torch.randn(B, E, device="cuda") * 3
    nw = torch.rand(E, device="cuda") + 0.5
    e16 = torch.zeros(B + 1, E, device="cuda", dtype=torch.float16)
    st = torch.zeros(16, E // 16, device="cuda")
    gemv(mo, a, epi=1, y=resid, extra=dict(emit16=e16.data_ptr(), ld_emit=E, emit_nw=nw.data_ptr(),
                                           emit_stat=st.data_ptr()))
    y_chain = torch.zeros(B, F, device="cuda")
    gemv(mg, resid, norm=1, nw=nw, y=y_chain, extra=dict(x16=e16.data_ptr(), ld16=E, zrow16=B, xstat=st.data_ptr(),
                                                         xstat_n=E // 16))
    y_lds = torch.zeros(B, F, device="cuda")
    gemv(mg, resid, norm=1, nw=nw, y=y_lds)
    assert rel(y_chain, y_lds) < 2e-3


def test_mb_glu_fp16_output():
    F, K, B = 344, 4096, 7
    m = QMM(GGMLType.Q4_K, 2 * F, K, seed=31)
    x = torch.randn(B, K, device="cuda")
    h16 = torch.zeros(B + 1, F, device="cuda", dtype=torch.float16)
    y = torch.zeros(B, F, device="cuda")
    gemv(m, x, epi=2, y=y, extra=dict(y16=h16.data_ptr(), ld16y=F))
    gu = x @ m.w.T
    ref = torch.nn.functional.silu(gu[:, 0::2]) * gu[:, 1::2]
    assert rel(h16[:B].float(), ref) < 5e-3
    assert float(y.abs().max()) == 0.0  # the fp16 output replaces the fp32 one


@pytest.mark.parametrize("qt", [GGMLType.Q4_0, GGMLType.Q4_K])
def test_mb_chain_range_scale(qt):
    """A residual past fp16's range (random-init 32-layer stacks reach ~6e4 by layer 21; Mistral-7B at
    B = 4 went NaN there): the producer stores row b times 2^-e_b, e_b from the RMS of the residual
    before its add (emit_prev), writes 2^e_b after the partials, and the consumer folds it back in
    (xscale). Rows with an old RMS below 8 keep e = 0 (bit-identical to the unscaled emission)."""
    B, E, F = 5, 4096, 512
    n = E // 16
    mo = QMM(qt, E, E, seed=41)
    mg = QMM(GGMLType.Q6_K, F, E, seed=42)
    a = torch.randn(B, E, device="cuda")
    mag = torch.tensor([1.0, 3e2, 4e3, 3e4, 9e4], device="cuda")[:, None]
    resid = torch.randn(B, E, device="cuda") * mag
    prev = torch.zeros(16 * n + 16, device="cuda")  # partials of the residual before the add
    prev[:B * n] = resid.pow(2).reshape(B, n, 16).sum(-1).reshape(-1)
    rms_old = resid.pow(2).mean(-1).sqrt()
    nw = torch.rand(E, device="cuda") + 0.5
    e16 = torch.zeros(B + 1, E, device="cuda", dtype=torch.float16)
    st = torch.zeros(16 * n + 16, device="cuda")
    gemv(mo, a, epi=1, y=resid, extra=dict(emit16=e16.data_ptr(), ld_emit=E, emit_nw=nw.data_ptr(),
                                           emit_stat=st.data_ptr(), emit_prev=prev.data_ptr(), emit_prev_n=n,
                                           emit_scale=st[16 * n:].data_ptr()))
    torch.cuda.synchronize()
    scale = st[16 * n:16 * n + B]
    want = torch.clamp(torch.floor(torch.log2(rms_old)) - 2, 0, 30).exp2()
    assert torch.equal(scale, want), (scale, want)
    assert bool(torch.isfinite(e16[:B].float()).all())
    assert rel(e16[:B].float() * scale[:, None], resid * nw) < 1e-3
    y_chain = torch.zeros(B, F, device="cuda")
    gemv(mg, resid, norm=1, nw=nw, y=y_chain, extra=dict(x16=e16.data_ptr(), ld16=E, zrow16=B, xstat=st.data_ptr(),
                                                         xstat_n=n, xscale=st[16 * n:].data_ptr()))
    y_lds = torch.zeros(B, F, device="cuda")
    gemv(mg, resid, norm=1, nw=nw, y=y_lds)
    for b in range(B):
        assert rel(y_chain[b], y_lds[b]) < 2e-3, b


def test_mb_engine_batched_decode_large_residual(tmp_path, monkeypatch):
    """Engine level: a residual stream far past fp16's range (the token embeddings scaled by 1e7) decodes
    a layout-M batch with finite logits that match the fp32-activation batch step."""
    from ollama_operator_amd.engine.runner import Runner
    from ollama_operator_amd.gguf.constants import FileType
    from ollama_operator_amd.models.config import ModelConfig, preset
    from ollama_operator_amd.models.random_init import write_random_gguf
    p = str(tmp_path / "m.gguf")
    write_random_gguf(p, preset("tiny-llama"), FileType.MOSTLY_Q4_0, seed=5)
    monkeypatch.setattr(ModelConfig, "embed_scale", property(lambda self: 1e7))
    g = Runner(p, device="cuda", max_batch=32, max_seqs=4, ctx=256)
    assert g.exe.exe.mb_chain
    B = 4
    sids = []
    for b in range(B):
        sid = g.new_sequence()
        g.prefill(sid, [1] + [3 + 7 * b + i for i in range(12)])
        sids.append(sid)
    V = g.cfg.n_vocab
    outs = []
    for on in (1, 0):
        C().reset_launch_counts()
        C().set_mb_enable(on)
        try:
            g.set_tokens(list(range(7, 7 + B)))
            g.decode_batch(sids, [13] * B)
            torch.cuda.synchronize()
        finally:
            C().set_mb_enable(1)
        assert (C().launch_counts()["gemv_mb"] > 0) == bool(on)
        outs.append(g.logits[:B, :V].float().cpu().clone())
    assert float(g.resid[:B].abs().max()) > 1e5  # the rows did outgrow fp16
    assert bool(torch.isfinite(outs[0]).all())
    assert rel(outs[0], outs[1]) < 2e-2
