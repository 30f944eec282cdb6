"""GPU numerics: every HIP kernel against a plain fp32 PyTorch reference of the same op."""
import math

import numpy as np
import pytest
import torch

from ollama_operator_amd.gguf import GGMLType
from ollama_operator_amd.quant import dequantize, quantize, random_blocks, repack

pytestmark = pytest.mark.gpu

QTYPES = [GGMLType.Q4_0, GGMLType.Q8_0, GGMLType.Q4_K, GGMLType.Q5_K, GGMLType.Q6_K]
STREAMS = {GGMLType.Q4_K: ["qs", "meta"], GGMLType.Q5_K: ["qs", "meta", "qh"], GGMLType.Q6_K: ["ql", "qh", "sc", "d"],
           GGMLType.Q4_0: ["qs", "d"], GGMLType.Q8_0: ["qs", "d"]}


def C():
    from ollama_operator_amd.ops import native
    return native()


def S():
    return torch.cuda.current_stream().cuda_stream


class QM:
    def __init__(self, qt, N, K, seed=0):
        rng = np.random.default_rng(seed)
        raw = random_blocks(qt, N, K, rng)
        self.w = torch.from_numpy(dequantize(raw, qt, N * K).reshape(N, K)).cuda()
        st = repack(raw, qt, N, K)
        self.streams = [torch.from_numpy(np.ascontiguousarray(st[n])).cuda() for n in STREAMS[qt]]
        p = [s.data_ptr() for s in self.streams] + [0] * (4 - len(self.streams))
        self.tup = (p[0], p[1], p[2], p[3], N, K, int(qt))


def rel(a, b):
    return float((a - b).norm() / (b.norm() + 1e-12))


def gemv(m, x, norm=0, nw=None, nb=None, epi=0, y=None, bias=None, row_offset=0, extra=None, eps=1e-5):
    B, K = x.shape
    p = lambda t: t.data_ptr() if t is not None else 0  # noqa: E731
    C().gemv(m.tup, B, p(x), K, norm, p(nw), p(nb), eps, epi, p(y), y.shape[1], p(bias), row_offset,
             extra or {}, S())


@pytest.mark.parametrize("qt", QTYPES)
@pytest.mark.parametrize("B", [1, 3, 6])
@pytest.mark.parametrize("K", [256, 4096, 11008])
def test_gemv_store(qt, B, K):
    if K == 11008 and qt in (GGMLType.Q4_0, GGMLType.Q8_0):
        K = 11008  # multiple of 32 as well
    N = 384
    m = QM(qt, N, K, seed=K + B)
    x = torch.randn(B, K, device="cuda")
    y = torch.zeros(B, N, device="cuda")
    gemv(m, x, y=y)
    ref = x @ m.w.T
    assert rel(y, ref) < 1e-2


@pytest.mark.parametrize("qt", [GGMLType.Q4_K, GGMLType.Q5_K, GGMLType.Q6_K])
def test_gemv_rmsnorm_add_bias(qt):
    N, K, B = 512, 2048, 2
    m = QM(qt, N, K, seed=3)
    x = torch.randn(B, K, device="cuda") * 3
    nw = torch.rand(K, device="cuda") + 0.5
    bias = torch.randn(N, device="cuda")
    y0 = torch.randn(B, N, device="cuda")
    y = y0.clone()
    gemv(m, x, norm=1, nw=nw, epi=1, y=y, bias=bias)
    xn = x * torch.rsqrt(x.pow(2).mean(-1, keepdim=True) + 1e-5) * nw
    ref = y0 + xn @ m.w.T + bias
    assert rel(y - y0, ref - y0) < 1e-2


def test_gemv_layernorm_gelu():
    N, K, B = 512, 2560, 1
    m = QM(GGMLType.Q4_0, N, K, seed=4)
    x = torch.randn(B, K, device="cuda") + 0.3
    nw, nb = torch.rand(K, device="cuda") + 0.5, torch.randn(K, device="cuda") * 0.1
    bias = torch.randn(N, device="cuda") * 0.1
    y = torch.zeros(B, N, device="cuda")
    gemv(m, x, norm=2, nw=nw, nb=nb, epi=3, y=y, bias=bias)
    xn = torch.nn.functional.layer_norm(x, (K,), nw, nb, 1e-5)
    h = xn @ m.w.T + bias
    ref = 0.5 * h * (1 + torch.tanh(math.sqrt(2 / math.pi) * (h + 0.044715 * h ** 3)))
    assert rel(y, ref) < 1e-2


def test_gemv_glu():
    F, K, B = 256, 1024, 4
    m = QM(GGMLType.Q4_K, 2 * F, K, seed=5)
    x = torch.randn(B, K, device="cuda")
    y = torch.zeros(B, F, device="cuda")
    gemv(m, x, epi=2, y=y)
    gu = x @ m.w.T
    ref = torch.nn.functional.silu(gu[:, 0::2]) * gu[:, 1::2]
    assert rel(y, ref) < 1.5e-2


@pytest.mark.parametrize("ks", [1, 2, 3, 4])
@pytest.mark.parametrize("qt,K", [(GGMLType.Q4_K, 11008), (GGMLType.Q6_K, 11008), (GGMLType.Q4_K, 4096),
                                  (GGMLType.Q5_K, 11008), (GGMLType.Q5_K, 4096),
                                  (GGMLType.Q8_0, 2560), (GGMLType.Q6_K, 1024)])
def test_gemv_flight_k_split(qt, K, ks):
    """The decode kernel's in-block K split (KS groups of 4 waves on the same rows, partial sums
    meeting in LDS) against fp32 torch, with the RMSNorm prologue and the pairwise GLU epilogue."""
    F = 200  # 400 rows: the last 16-row tile is partial
    m = QM(qt, 2 * F, K, seed=K + ks)
    x = torch.randn(1, K, device="cuda")
    nw = torch.rand(K, device="cuda") + 0.5
    y = torch.zeros(1, F, device="cuda")
    C().set_gemv_tuning(0, 0, 0, ks)
    try:
        gemv(m, x, norm=1, nw=nw, epi=2, y=y)
    finally:
        C().set_gemv_tuning(0, 0, 0, 0)
    xn = x * torch.rsqrt(x.pow(2).mean(-1, keepdim=True) + 1e-5) * nw
    gu = xn @ m.w.T
    ref = torch.nn.functional.silu(gu[:, 0::2]) * gu[:, 1::2]
    assert rel(y, ref) < 1.5e-2


@pytest.mark.parametrize("D,n_rot", [(128, 128), (80, 32), (64, 64)])
def test_gemv_qkv_rope_kv_scatter(D, n_rot):
    H, Hkv, K, B, bs = 4, 2, 512, 3, 16
    Eq, Ekv = H * D, Hkv * D
    N = Eq + 2 * Ekv
    m = QM(GGMLType.Q4_K if K % 256 == 0 else GGMLType.Q8_0, N, K, seed=D)
    x = torch.randn(B, K, device="cuda")
    q = torch.zeros(B, Eq, device="cuda")
    nblk = 8
    kc = torch.zeros(nblk, Hkv, bs, D, device="cuda", dtype=torch.float16)
    vc = torch.zeros_like(kc)
    pos = torch.tensor([0, 17, 40], device="cuda", dtype=torch.int32)
    slot = torch.tensor([5, 3 * bs + 1, 7 * bs + 15], device="cuda", dtype=torch.int32)
    inv = (10000.0 ** (-torch.arange(0, n_rot // 2, dtype=torch.float64) * 2 / n_rot)).float().cuda()
    extra = dict(pos=pos.data_ptr(), slot=slot.data_ptr(), kc=kc.data_ptr(), vc=vc.data_ptr(), inv_freq=inv.data_ptr(),
                 Eq=Eq, Ekv=Ekv, D=D, n_rot=n_rot, n_kv=Hkv, bs=bs)
    gemv(m, x, epi=4, y=q, extra=extra)
    y = x @ m.w.T

    def rope(t, nh):
        t = t.view(B, nh, D).clone()
        ang = pos.double()[:, None] * inv.double()[None, :]
        c, s = torch.cos(ang).float()[:, None, :], torch.sin(ang).float()[:, None, :]
        a, b = t[..., 0:n_rot:2].clone(), t[..., 1:n_rot:2].clone()
        t[..., 0:n_rot:2] = a * c - b * s
        t[..., 1:n_rot:2] = a * s + b * c
        return t
    assert rel(q.view(B, H, D), rope(y[:, :Eq], H)) < 1e-2
    kr = rope(y[:, Eq:Eq + Ekv], Hkv)
    vr = y[:, Eq + Ekv:].view(B, Hkv, D)
    for b in range(B):
        blk, off = int(slot[b]) // bs, int(slot[b]) % bs
        assert rel(kc[blk, :, off].float(), kr[b]) < 1.2e-2
        assert rel(vc[blk, :, off].float(), vr[b]) < 1.2e-2


@pytest.mark.parametrize("D", [64, 80, 96, 112, 128])
@pytest.mark.parametrize("G,hpb", [(1, 0), (2, 0), (4, 0), (4, 1), (4, 4), (8, 0), (8, 1), (8, 2), (8, 8), (3, 0)])
@pytest.mark.parametrize("splits", [1, 5])
def test_attention_paged(D, G, hpb, splits):
    """Decode attention vs fp32 torch; hpb = query heads per block (GQA group split over blocks)."""
    C().set_attn_tuning(256, hpb)
    try:
        _attention_paged(D, G, splits)
    finally:
        C().set_attn_tuning(256, 0)


def _attention_paged(D, G, splits):
    Hkv, bs, NQ = 2, 16, 3
    H = Hkv * G
    lens = [1, 37, 200]
    max_blocks = 16
    nblk = 64
    torch.manual_seed(0)
    kc = (torch.randn(nblk, Hkv, bs, D, device="cuda")).half()
    vc = (torch.randn(nblk, Hkv, bs, D, device="cuda")).half()
    bt = torch.randperm(nblk, device="cuda")[:NQ * max_blocks].view(NQ, max_blocks).int()
    q = torch.randn(NQ, H * D, device="cuda")
    qlen = torch.tensor(lens, device="cuda", dtype=torch.int32)
    out = torch.zeros(NQ, H * D, device="cuda")
    ws = torch.zeros(max(1, C().attention_ws_floats(NQ, H, D, splits)), device="cuda")
    cnt = torch.zeros(NQ * H, device="cuda", dtype=torch.int32)
    scale = 1 / math.sqrt(D)
    for rep in range(3):  # tickets must re-arm themselves between launches
        out.zero_()
        C().attention(q.data_ptr(), H * D, kc.data_ptr(), vc.data_ptr(), bt.data_ptr(), max_blocks, 0,
                      qlen.data_ptr(), NQ, H, Hkv, D, bs, scale, 0, out.data_ptr(), H * D, ws.data_ptr(), splits,
                      cnt.data_ptr(), S())
    assert int(cnt.abs().sum()) == 0
    for i, n in enumerate(lens):
        t = torch.arange(n, device="cuda")
        kk = kc[bt[i][t // bs].long(), :, t % bs].float().repeat_interleave(G, 1)
        vv = vc[bt[i][t // bs].long(), :, t % bs].float().repeat_interleave(G, 1)
        s = torch.einsum("hd,thd->ht", q[i].view(H, D), kk) * scale
        ref = torch.einsum("ht,thd->hd", torch.softmax(s, -1), vv).reshape(-1)
        assert rel(out[i], ref) < 2e-3


@pytest.mark.parametrize("D", [64, 80, 128])
@pytest.mark.parametrize("G", [1, 4])
@pytest.mark.parametrize("start,NQ,window", [(0, 16, 0), (37, 100, 0), (0, 300, 0), (5, 130, 64)])
def test_attention_prefill_mfma(D, G, start, NQ, window):
    """MFMA flash prefill (attn_prefill_kernel): one sequence, queries at contiguous positions
    start..start+NQ-1 (a prompt chunk after `start` cached tokens), causal (+ sliding window)."""
    Hkv, bs = 2, 16
    H = Hkv * G
    total = start + NQ
    max_blocks = (total + bs - 1) // bs
    nblk = max_blocks + 8
    torch.manual_seed(1)
    kc = torch.randn(nblk, Hkv, bs, D, device="cuda").half()
    vc = torch.randn(nblk, Hkv, bs, D, device="cuda").half()
    bt = torch.randperm(nblk, device="cuda")[:max_blocks].view(1, max_blocks).int()
    q = torch.randn(NQ, H * D, device="cuda")
    qlen = torch.arange(start + 1, start + NQ + 1, device="cuda", dtype=torch.int32)
    qseq = torch.zeros(NQ, device="cuda", dtype=torch.int32)
    out = torch.zeros(NQ, H * D, device="cuda")
    scale = 1 / math.sqrt(D)
    C().attention(q.data_ptr(), H * D, kc.data_ptr(), vc.data_ptr(), bt.data_ptr(), max_blocks, qseq.data_ptr(),
                  qlen.data_ptr(), NQ, H, Hkv, D, bs, scale, window, out.data_ptr(), H * D, 0, 1, 0, S(),
                  prefill=1)
    torch.cuda.synchronize()
    t = torch.arange(total, device="cuda")
    kk = kc[bt[0][t // bs].long(), :, t % bs].float().repeat_interleave(G, 1)  # [T][H][D]
    vv = vc[bt[0][t // bs].long(), :, t % bs].float().repeat_interleave(G, 1)
    s = torch.einsum("qhd,thd->hqt", q.view(NQ, H, D), kk) * scale
    pos = torch.arange(start, start + NQ, device="cuda")[:, None]
    mask = t[None, :] <= pos
    if window:
        mask &= t[None, :] >= (pos + 1 - window)
    s = s.masked_fill(~mask[None], float("-inf"))
    ref = torch.einsum("hqt,thd->qhd", torch.softmax(s, -1), vv).reshape(NQ, -1)
    assert rel(out, ref) < 3e-3


@pytest.mark.parametrize("qt", QTYPES)
def test_embed_and_dequant_f16(qt):
    V, E = 64, 512
    m = QM(qt, V, E, seed=9)
    rows = torch.tensor([0, 5, 63, 5], device="cuda", dtype=torch.int32)
    out = torch.zeros(4, E, device="cuda")
    C().embed_rows(m.tup, rows.data_ptr(), 4, out.data_ptr(), E, S())
    torch.testing.assert_close(out, m.w[rows.long()], rtol=1e-5, atol=1e-6)
    h = torch.zeros(V, E, device="cuda", dtype=torch.float16)
    C().dequant_f16(m.tup, h.data_ptr(), S())
    torch.testing.assert_close(h.float(), m.w, rtol=1e-3, atol=1e-4)


def _sample_args(B, V, logits, **kw):
    d = dict(temperature=torch.full((B,), kw.get("temperature", 0.8)), top_k=torch.full((B,), kw.get("top_k", 40), dtype=torch.int32),
             top_p=torch.full((B,), kw.get("top_p", 0.9)), min_p=torch.full((B,), kw.get("min_p", 0.0)),
             repeat_penalty=torch.full((B,), kw.get("repeat_penalty", 1.0)), presence_penalty=torch.zeros(B),
             frequency_penalty=torch.zeros(B), repeat_last_n=torch.full((B,), 64, dtype=torch.int32),
             seed=torch.tensor([kw.get("seed", 7)] * B, dtype=torch.int64), step=torch.zeros(B, dtype=torch.int32),
             history=torch.zeros(B, 64, dtype=torch.int32), hist_count=torch.zeros(B, dtype=torch.int32),
             out=torch.zeros(B, dtype=torch.int32))
    if kw.get("fast"):
        d["ws"] = torch.full((B, -(-V // 1024) * 128), float("nan"))
        d["counters"] = torch.zeros(B, dtype=torch.int32)
    d = {k: v.cuda() for k, v in d.items()}
    ptrs = {k: v.data_ptr() for k, v in d.items()}
    ptrs.update(logits=logits.data_ptr(), B=B, V=V, ld=V, hist_cap=64)
    return d, ptrs


@pytest.mark.parametrize("V", [32000, 50257, 1000])
@pytest.mark.parametrize("top_k,top_p,min_p", [(40, 0.9, 0.0), (1, 1.0, 0.0), (64, 0.95, 0.05), (7, 1.0, 0.0),
                                               (65, 0.9, 0.0), (0, 0.9, 0.0)])
def test_sampling_multiblock_matches_host(V, top_k, top_p, min_p):
    """The multi-block sampler (per-wave bitonic top-64, LDS tree, ticket hand-off; top_k outside
    1..64 falls back to the single-block selection in the last block) against the host reference,
    token for token: penalties with repeated history tokens, ties broken by the lower index, and
    three consecutive calls on the same tickets."""
    from ollama_operator_amd.engine.sampling import SamplingOptions, sample_host
    B = 3
    torch.manual_seed(V + top_k)
    base = torch.randn(B, V, device="cuda") * 2
    base[1] = torch.round(base[1] * 2) / 2  # heavy ties
    hist = [[5, 17, 5, 900, 17, 5], [], [3, 3, 3, 999]]
    o = SamplingOptions(temperature=0.7, top_k=top_k, top_p=top_p, min_p=min_p, repeat_penalty=1.3,
                        presence_penalty=0.2, frequency_penalty=0.1, repeat_last_n=64)
    for temperature in (0.7, 0.0):
        lg = base.clone()
        d, p = _sample_args(B, V, lg, fast=True, temperature=temperature, top_k=top_k, top_p=top_p, min_p=min_p,
                            repeat_penalty=1.3, seed=11)
        d["presence_penalty"].fill_(0.2)
        d["frequency_penalty"].fill_(0.1)
        for b in range(B):
            d["history"][b, :len(hist[b])] = torch.tensor(hist[b], dtype=torch.int32) if hist[b] else 0
            d["hist_count"][b] = len(hist[b])
        o.temperature = temperature
        hs = [list(h) for h in hist]
        for step in range(3):
            lg.copy_(base)
            C().sample(p, S())
            torch.cuda.synchronize()
            for b in range(B):
                want = sample_host(base[b].cpu().numpy(), hs[b], o, 11, step)
                assert int(d["out"][b]) == want, (b, step, temperature)
                hs[b].append(want)
        assert int(d["counters"].abs().sum()) == 0  # tickets re-armed


def test_sampling_greedy_and_seeded():
    from ollama_operator_amd.engine.sampling import SamplingOptions, sample_host
    B, V = 3, 32000
    torch.manual_seed(1)
    logits = torch.randn(B, V, device="cuda") * 3
    ref_argmax = logits.argmax(-1)
    d, p = _sample_args(B, V, logits.clone(), temperature=0.0)
    C().sample(p, S())
    assert torch.equal(d["out"].long(), ref_argmax)
    out = torch.zeros(B, dtype=torch.int32, device="cuda")
    C().argmax(logits.data_ptr(), B, V, V, out.data_ptr(), S())
    assert torch.equal(out.long(), ref_argmax)
    for seed in [1, 2, 3]:
        lg = logits.clone()
        d, p = _sample_args(B, V, lg, seed=seed)
        C().sample(p, S())
        o = SamplingOptions(temperature=0.8, top_k=40, top_p=0.9, repeat_penalty=1.0)
        for b in range(B):
            assert int(d["out"][b]) == sample_host(logits[b].cpu().numpy(), [], o, seed, 0)
        assert int(d["step"][0]) == 1 and int(d["hist_count"][0]) == 1


def test_repeat_penalty_changes_argmax():
    B, V = 1, 1000
    logits = torch.zeros(B, V, device="cuda")
    logits[0, 10] = 2.0
    logits[0, 11] = 1.9
    d, p = _sample_args(B, V, logits, temperature=0.0, repeat_penalty=1.1)
    d["history"][0, :3] = torch.tensor([10, 10, 5], dtype=torch.int32)
    d["hist_count"][0] = 3
    C().sample(p, S())
    assert int(d["out"][0]) == 11


@pytest.mark.parametrize("qt", QTYPES)
@pytest.mark.parametrize("B", [2, 4, 5, 8, 15])
@pytest.mark.parametrize("K,norm", [(4096, 1), (4096, 0), (11008, 0), (2560, 2), (8192, 1)])
def test_gemv_batch_rows(qt, B, K, norm):
    """Continuous-batching GEMV (gemv_batch.hip: BT rows per block, register or x-first LDS
    prologue) against fp32 torch, with no norm / RMSNorm / LayerNorm prologues and a residual add."""
    N = 400  # partial last 16-row tile
    m = QM(qt, N, K, seed=K + 7 * B + norm)
    x = torch.randn(B, K, device="cuda") + 0.2
    nw = torch.rand(K, device="cuda") + 0.5 if norm else None
    nb = torch.randn(K, device="cuda") * 0.1 if norm == 2 else None
    y0 = torch.randn(B, N, device="cuda")
    y = y0.clone()
    gemv(m, x, norm=norm, nw=nw, nb=nb, epi=1, y=y)
    if norm == 1:
        xn = x * torch.rsqrt(x.pow(2).mean(-1, keepdim=True) + 1e-5) * nw
    elif norm == 2:
        xn = torch.nn.functional.layer_norm(x, (K,), nw, nb, 1e-5)
    else:
        xn = x
    ref = xn @ m.w.T
    assert rel(y - y0, ref) < 1e-2


@pytest.mark.parametrize("K", [4096, 11008])
@pytest.mark.parametrize("B", [1, 3])
def test_gemv_q6k_widened(K, B):
    """Q6_K with load-time int8-widened codes (qmat.h QT_Q6_K8): the batch-1 GEMV reads the widened
    stream, batched rows the 6-bit streams; both against fp32 torch (store and residual-add)."""
    N = 512
    m = QM(GGMLType.Q6_K, N, K, seed=K + 7)
    wide = torch.empty(N * (K // 256) * 256, dtype=torch.uint8, device="cuda")
    C().widen_q6k(m.tup, wide.data_ptr(), S())
    m.tup = m.tup + (wide.data_ptr(),)
    x = torch.randn(B, K, device="cuda")
    y = torch.zeros(B, N, device="cuda")
    gemv(m, x, y=y)
    torch.cuda.synchronize()
    assert rel(y, x @ m.w.T) < 1e-2
    res = torch.randn(B, N, device="cuda")
    y2 = res.clone()
    gemv(m, x, epi=1, y=y2)
    torch.cuda.synchronize()
    assert rel(y2, res + x @ m.w.T) < 1e-2


@pytest.mark.parametrize("qt", [GGMLType.Q8_0, GGMLType.Q4_K, GGMLType.Q6_K])
@pytest.mark.parametrize("B,X,k", [(1, 8, 2), (5, 8, 2), (3, 16, 4), (2, 60, 6)])
def test_moe_router_fused(qt, B, X, k):
    """Fused RMSNorm + router logits + top-k softmax (moe.hip moe_router) against fp32 torch."""
    K = 1024
    m = QM(qt, X, K, seed=X + k)
    x = torch.randn(B, K, device="cuda")
    nw = torch.rand(K, device="cuda") + 0.5
    ids = torch.full((B, k), -1, device="cuda", dtype=torch.int32)
    w = torch.zeros(B, k, device="cuda")
    C().moe_router(m.tup, B, x.data_ptr(), K, nw.data_ptr(), 1e-5, k, ids.data_ptr(), w.data_ptr(), S())
    xn = x * torch.rsqrt(x.pow(2).mean(-1, keepdim=True) + 1e-5) * nw
    logits = xn @ m.w.T
    top, idx = torch.topk(logits, k, dim=-1)
    ref_w = torch.softmax(top, dim=-1)
    assert torch.equal(ids.long(), idx), (ids, idx)
    assert torch.allclose(w, ref_w, atol=1e-5)
