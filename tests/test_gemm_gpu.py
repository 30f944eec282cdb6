"""GPU numerics of the prefill MFMA dequant GEMM paths: the same `gemv` entry with an fp16 activation
workspace and B >= GEMM_MIN_B, against a plain fp32 PyTorch reference on the dequantised weights.
path "dq": the stream-order kernel (csrc/kernels/gemm_dq.hip, the default from 128 rows); "old": the
128 x 128 natural-order tile (gemm.hip, below 128 rows); "lib": hipBLASLt (the oracle / A-B baseline).
Covers every quant type, partial M/N tiles, K padding (Q4_0/Q8_0 with K % 256 != 0), split-K and
every fused epilogue."""
import math

import pytest
import torch

from ollama_operator_amd.gguf import GGMLType
from test_kernels_gpu import QM, QTYPES, C, S, rel

pytestmark = pytest.mark.gpu


def gemm(m, x, norm=0, nw=None, nb=None, epi=0, y=None, bias=None, extra=None, eps=1e-5, split=True, lib=False,
         path="old"):
    """split=True gives the kernel a split-K workspace (small M then runs split-K + finalize).
    lib=True: the hipBLASLt path (dequantised fp16 weight scratch + fp32 slab) from M = 16 on.
    path: "dq" enables the stream-order kernel (gemm_dq.hip, B >= 128), "old" disables it."""
    B, K = x.shape
    Kp = (K + 255) // 256 * 256
    xws = torch.empty(B * Kp, device="cuda", dtype=torch.float16)
    gws = torch.empty(8 << 20, device="cuda")
    p = lambda t: t.data_ptr() if t is not None else 0  # noqa: E731
    d = dict(extra or {})
    d["xws"], d["xws_elems"] = xws.data_ptr(), xws.numel()
    if split or lib:
        d["gws"], d["gws_elems"] = gws.data_ptr(), gws.numel()
    keep = []
    if lib:
        w16 = torch.full((m.w.shape[0] * K,), float("nan"), device="cuda", dtype=torch.float16)
        yws = torch.full((B * m.w.shape[0],), float("nan"), device="cuda")
        keep += [w16, yws]
        d.update(w16ws=w16.data_ptr(), w16_elems=w16.numel(), yws=yws.data_ptr(), yws_elems=yws.numel())
    old, old_dq = C().gemm_lib_min_m(), C().dq_gemm_enabled()
    C().set_gemm_lib_min_m(16 if lib else 0)
    C().set_dq_gemm(1 if path == "dq" else 0)
    C().reset_launch_counts()
    try:
        C().gemv(m.tup, B, p(x), K, norm, p(nw), p(nb), eps, epi, p(y), y.shape[1], p(bias), 0, d, S())
        torch.cuda.synchronize()
    finally:
        C().set_gemm_lib_min_m(old)
        C().set_dq_gemm(int(old_dq))
    n = C().launch_counts()
    if lib:  # the library path really ran: the fp32 slab holds the raw products
        assert not torch.isnan(keep[1]).any()
        assert n["gemm_lib"] == 1, n
    elif path == "dq":  # the stream-order kernel ran, not a silent fallback to the tile kernel
        assert n["dq_gemm"] == 1 and n["gemm_tile"] == 0, n
    elif B >= 16:
        assert n["gemm_tile"] == 1 and n["dq_gemm"] == 0, n


@pytest.mark.parametrize("qt", QTYPES)
@pytest.mark.parametrize("B", [16, 40, 130])
@pytest.mark.parametrize("K", [256, 4096, 11008, 288])
@pytest.mark.parametrize("split", [True, False])
def test_gemm_store(qt, B, K, split):
    if K == 288 and qt in (GGMLType.Q4_K, GGMLType.Q5_K, GGMLType.Q6_K):
        pytest.skip("k-quant rows are whole super-blocks")
    N = 384 + 64  # partial N tile
    m = QM(qt, N, K, seed=K + B)
    x = torch.randn(B, K, device="cuda")
    y = torch.zeros(B, N, device="cuda")
    gemm(m, x, y=y, split=split)
    assert rel(y, x @ m.w.T) < 1e-2


def test_gemm_rmsnorm_add_bias():
    N, K, B = 512, 2048, 33
    m = QM(GGMLType.Q4_K, N, K, seed=3)
    x = torch.randn(B, K, device="cuda") * 3
    nw = torch.rand(K, device="cuda") + 0.5
    bias = torch.randn(N, device="cuda")
    y0 = torch.randn(B, N, device="cuda")
    y = y0.clone()
    gemm(m, x, norm=1, nw=nw, epi=1, y=y, bias=bias)
    xn = x * torch.rsqrt(x.pow(2).mean(-1, keepdim=True) + 1e-5) * nw
    ref = y0 + xn @ m.w.T + bias
    assert rel(y - y0, ref - y0) < 1e-2


def test_gemm_layernorm_gelu():
    N, K, B = 512, 2560, 20
    m = QM(GGMLType.Q4_0, N, K, seed=4)
    x = torch.randn(B, K, device="cuda") + 0.3
    nw, nb = torch.rand(K, device="cuda") + 0.5, torch.randn(K, device="cuda") * 0.1
    bias = torch.randn(N, device="cuda") * 0.1
    y = torch.zeros(B, N, device="cuda")
    gemm(m, x, norm=2, nw=nw, nb=nb, epi=3, y=y, bias=bias)
    xn = torch.nn.functional.layer_norm(x, (K,), nw, nb, 1e-5)
    h = xn @ m.w.T + bias
    ref = 0.5 * h * (1 + torch.tanh(math.sqrt(2 / math.pi) * (h + 0.044715 * h ** 3)))
    assert rel(y, ref) < 1e-2


@pytest.mark.parametrize("qt", [GGMLType.Q4_K, GGMLType.Q5_K, GGMLType.Q6_K])
def test_gemm_glu(qt):
    F, K, B = 320, 1024, 50
    m = QM(qt, 2 * F, K, seed=5)
    x = torch.randn(B, K, device="cuda")
    y = torch.zeros(B, F, device="cuda")
    gemm(m, x, epi=2, y=y)
    gu = x @ m.w.T
    ref = torch.nn.functional.silu(gu[:, 0::2]) * gu[:, 1::2]
    assert rel(y, ref) < 1.5e-2


@pytest.mark.parametrize("D,n_rot", [(128, 128), (80, 32)])
def test_gemm_qkv_rope_kv_scatter(D, n_rot):
    H, Hkv, K, B, bs = 4, 2, 512, 24, 16
    Eq, Ekv = H * D, Hkv * D
    N = Eq + 2 * Ekv
    m = QM(GGMLType.Q4_K, N, K, seed=D)
    x = torch.randn(B, K, device="cuda")
    q = torch.zeros(B, Eq, device="cuda")
    nblk = 4
    kc = torch.zeros(nblk, Hkv, bs, D, device="cuda", dtype=torch.float16)
    vc = torch.zeros_like(kc)
    pos = torch.arange(B, device="cuda", dtype=torch.int32) + 7
    slot = torch.arange(B, device="cuda", dtype=torch.int32) + 9  # distinct slots across 3 blocks
    inv = (10000.0 ** (-torch.arange(0, n_rot // 2, dtype=torch.float64) * 2 / n_rot)).float().cuda()
    extra = dict(pos=pos.data_ptr(), slot=slot.data_ptr(), kc=kc.data_ptr(), vc=vc.data_ptr(), inv_freq=inv.data_ptr(),
                 Eq=Eq, Ekv=Ekv, D=D, n_rot=n_rot, n_kv=Hkv, bs=bs)
    gemm(m, x, epi=4, y=q, extra=extra)
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


def test_gemm_matches_batched_gemv():
    """Both B > 1 paths of the same matrix agree (GEMM fp16 vs GEMV int8-dot activations)."""
    N, K, B = 1024, 4096, 64
    m = QM(GGMLType.Q4_K, N, K, seed=11)
    x = torch.randn(B, K, device="cuda")
    y1 = torch.zeros(B, N, device="cuda")
    y2 = torch.zeros(B, N, device="cuda")
    gemm(m, x, y=y1)
    C().gemv(m.tup, B, x.data_ptr(), K, 0, 0, 0, 1e-5, 0, y2.data_ptr(), N, 0, 0, {}, S())
    torch.cuda.synchronize()
    assert rel(y1, y2) < 1e-2


# ---- large-M library path (gemm.hip gemm_lib -> blas.cpp hipBLASLt) ---------------------------------
@pytest.mark.parametrize("qt", QTYPES)
@pytest.mark.parametrize("B,K", [(16, 256), (130, 4096), (300, 288), (64, 11008)])
def test_gemm_lib_store(qt, B, K):
    if K % 256 and qt in (GGMLType.Q4_K, GGMLType.Q5_K, GGMLType.Q6_K):
        pytest.skip("k-quant rows are whole super-blocks")
    N = 384 + 64
    m = QM(qt, N, K, seed=K + B + 1)
    x = torch.randn(B, K, device="cuda")
    y = torch.zeros(B, N, device="cuda")
    gemm(m, x, y=y, lib=True)
    assert rel(y, x @ m.w.T) < 1e-2


def test_gemm_lib_rmsnorm_add_bias():
    N, K, B = 512, 2048, 96
    m = QM(GGMLType.Q6_K, N, K, seed=13)
    x = torch.randn(B, K, device="cuda") * 3
    nw = torch.rand(K, device="cuda") + 0.5
    bias = torch.randn(N, device="cuda")
    y0 = torch.randn(B, N, device="cuda")
    y = y0.clone()
    gemm(m, x, norm=1, nw=nw, epi=1, y=y, bias=bias, lib=True)
    xn = x * torch.rsqrt(x.pow(2).mean(-1, keepdim=True) + 1e-5) * nw
    ref = y0 + xn @ m.w.T + bias
    assert rel(y - y0, ref - y0) < 1e-2


def test_gemm_lib_glu():
    F, K, B = 320, 1024, 257
    m = QM(GGMLType.Q4_K, 2 * F, K, seed=15)
    x = torch.randn(B, K, device="cuda")
    y = torch.zeros(B, F, device="cuda")
    gemm(m, x, epi=2, y=y, lib=True)
    gu = x @ m.w.T
    ref = torch.nn.functional.silu(gu[:, 0::2]) * gu[:, 1::2]
    assert rel(y, ref) < 1.5e-2


def test_gemm_lib_matches_fused():
    """Both prefill paths compute the same product (fp16 operands, fp32 accumulation)."""
    N, K, B = 1024, 4096, 512
    m = QM(GGMLType.Q4_K, N, K, seed=17)
    x = torch.randn(B, K, device="cuda")
    y1 = torch.zeros(B, N, device="cuda")
    y2 = torch.zeros(B, N, device="cuda")
    gemm(m, x, y=y1, split=False)
    gemm(m, x, y=y2, lib=True)
    assert rel(y1, y2) < 2e-3


# ---- stream-order dequant GEMM (gemm_dq.hip) --------------------------------------------------------
@pytest.mark.parametrize("qt", QTYPES)
@pytest.mark.parametrize("B,N", [(128, 448), (300, 448), (600, 2304), (160, 5120)])
@pytest.mark.parametrize("K", [256, 4096, 288])
@pytest.mark.parametrize("split", [True, False])
def test_dq_store(qt, B, N, K, split):
    if K == 288 and qt in (GGMLType.Q4_K, GGMLType.Q5_K, GGMLType.Q6_K):
        pytest.skip("k-quant rows are whole super-blocks")
    m = QM(qt, N, K, seed=K + B + N)
    x = torch.randn(B, K, device="cuda")
    y = torch.zeros(B, N, device="cuda")
    gemm(m, x, y=y, split=split, path="dq")
    assert rel(y, x @ m.w.T) < 1e-2


@pytest.mark.parametrize("qt", [GGMLType.Q4_K, GGMLType.Q6_K])
def test_dq_long_k(qt):
    N, K, B = 4096, 11008, 256  # Llama-2-7B down projection shape, one M tile, split-K
    m = QM(qt, N, K, seed=21)
    x = torch.randn(B, K, device="cuda")
    y = torch.zeros(B, N, device="cuda")
    gemm(m, x, y=y, path="dq")
    assert rel(y, x @ m.w.T) < 1e-2


def test_dq_rmsnorm_add_bias():
    N, K, B = 512, 2048, 200
    m = QM(GGMLType.Q4_K, N, K, seed=23)
    x = torch.randn(B, K, device="cuda") * 3
    nw = torch.rand(K, device="cuda") + 0.5
    bias = torch.randn(N, device="cuda")
    y0 = torch.randn(B, N, device="cuda")
    y = y0.clone()
    gemm(m, x, norm=1, nw=nw, epi=1, y=y, bias=bias, path="dq")
    xn = x * torch.rsqrt(x.pow(2).mean(-1, keepdim=True) + 1e-5) * nw
    ref = y0 + xn @ m.w.T + bias
    assert rel(y - y0, ref - y0) < 1e-2


def test_dq_layernorm_gelu():
    N, K, B = 512, 2560, 150
    m = QM(GGMLType.Q4_0, N, K, seed=24)
    x = torch.randn(B, K, device="cuda") + 0.3
    nw, nb = torch.rand(K, device="cuda") + 0.5, torch.randn(K, device="cuda") * 0.1
    bias = torch.randn(N, device="cuda") * 0.1
    y = torch.zeros(B, N, device="cuda")
    gemm(m, x, norm=2, nw=nw, nb=nb, epi=3, y=y, bias=bias, path="dq")
    xn = torch.nn.functional.layer_norm(x, (K,), nw, nb, 1e-5)
    h = xn @ m.w.T + bias
    ref = 0.5 * h * (1 + torch.tanh(math.sqrt(2 / math.pi) * (h + 0.044715 * h ** 3)))
    assert rel(y, ref) < 1e-2


@pytest.mark.parametrize("qt", [GGMLType.Q4_K, GGMLType.Q5_K, GGMLType.Q6_K, GGMLType.Q8_0])
def test_dq_glu(qt):
    F, K, B = 320, 1024, 270
    m = QM(qt, 2 * F, K, seed=25)
    x = torch.randn(B, K, device="cuda")
    y = torch.zeros(B, F, device="cuda")
    gemm(m, x, epi=2, y=y, path="dq")
    gu = x @ m.w.T
    ref = torch.nn.functional.silu(gu[:, 0::2]) * gu[:, 1::2]
    assert rel(y, ref) < 1.5e-2


def test_dq_qkv_rope_kv_scatter():
    D, n_rot, H, Hkv, K, B, bs = 128, 128, 4, 2, 512, 140, 16
    Eq, Ekv = H * D, Hkv * D
    N = Eq + 2 * Ekv
    m = QM(GGMLType.Q4_K, N, K, seed=26)
    x = torch.randn(B, K, device="cuda")
    q = torch.zeros(B, Eq, device="cuda")
    nblk = (B + 9 + bs - 1) // bs
    kc = torch.zeros(nblk, Hkv, bs, D, device="cuda", dtype=torch.float16)
    vc = torch.zeros_like(kc)
    pos = torch.arange(B, device="cuda", dtype=torch.int32) + 7
    slot = torch.arange(B, device="cuda", dtype=torch.int32) + 9
    inv = (10000.0 ** (-torch.arange(0, n_rot // 2, dtype=torch.float64) * 2 / n_rot)).float().cuda()
    extra = dict(pos=pos.data_ptr(), slot=slot.data_ptr(), kc=kc.data_ptr(), vc=vc.data_ptr(), inv_freq=inv.data_ptr(),
                 Eq=Eq, Ekv=Ekv, D=D, n_rot=n_rot, n_kv=Hkv, bs=bs)
    gemm(m, x, epi=4, y=q, extra=extra, path="dq")
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
    for b in range(0, B, 7):
        blk, off = int(slot[b]) // bs, int(slot[b]) % bs
        assert rel(kc[blk, :, off].float(), kr[b]) < 1.2e-2
        assert rel(vc[blk, :, off].float(), vr[b]) < 1.2e-2


def test_dq_matches_library():
    """The hand-written kernel and hipBLASLt compute the same product (fp16 operands, fp32 accumulate;
    only the summation order differs)."""
    N, K, B = 1024, 4096, 512
    m = QM(GGMLType.Q4_K, N, K, seed=27)
    x = torch.randn(B, K, device="cuda")
    y1 = torch.zeros(B, N, device="cuda")
    y2 = torch.zeros(B, N, device="cuda")
    gemm(m, x, y=y1, split=False, path="dq")
    gemm(m, x, y=y2, lib=True)
    assert rel(y1, y2) < 2e-3
