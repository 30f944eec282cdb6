"""GPU numerics of the wave-specialised decode GEMV (csrc/kernels/gemv_ws.hip: loader waves stream the
weights into LDS with global_load_lds, compute waves consume them) against fp32 torch, for every
quant type, prologue and epilogue it serves, plus the engine end to end with it switched on."""
import math

import pytest
import torch

from ollama_operator_amd.gguf import GGMLType
from tests.test_kernels_gpu import QM, QTYPES, C, gemv, rel

pytestmark = pytest.mark.gpu


@pytest.fixture
def ws_on():
    C().set_gemv_tuning(ws=1)
    yield
    C().set_gemv_tuning(ws=0)


@pytest.mark.parametrize("qt", QTYPES)
@pytest.mark.parametrize("K", [256, 4096, 11008])
@pytest.mark.parametrize("N", [400, 4096])
def test_ws_store(ws_on, qt, K, N):
    m = QM(qt, N, K, seed=K + N)
    x = torch.randn(1, K, device="cuda")
    y = torch.zeros(1, N, device="cuda")
    for _ in range(3):  # the LDS handshake re-initialises every launch
        gemv(m, x, y=y)
    assert rel(y, x @ m.w.T) < 1e-2


@pytest.mark.parametrize("qt", [GGMLType.Q4_K, GGMLType.Q5_K, GGMLType.Q6_K, GGMLType.Q8_0])
def test_ws_rmsnorm_add_bias(ws_on, qt):
    N, K = 1000, 4096
    m = QM(qt, N, K, seed=3)
    x = torch.randn(1, K, device="cuda") * 3
    nw = torch.rand(K, device="cuda") + 0.5
    bias = torch.randn(N, device="cuda")
    y0 = torch.randn(1, N, device="cuda")
    y = y0.clone()
    gemv(m, x, norm=1, nw=nw, epi=1, y=y, bias=bias)
    xn = x * torch.rsqrt(x.pow(2).mean(-1, keepdim=True) + 1e-5) * nw
    ref = y0 + xn @ m.w.T + bias
    assert rel(y - y0, ref - y0) < 1e-2


def test_ws_layernorm_gelu(ws_on):
    N, K = 2000, 2560
    m = QM(GGMLType.Q4_0, N, K, seed=4)
    x = torch.randn(1, K, device="cuda") + 0.3
    nw, nb = torch.rand(K, device="cuda") + 0.5, torch.randn(K, device="cuda") * 0.1
    bias = torch.randn(N, device="cuda") * 0.1
    y = torch.zeros(1, N, device="cuda")
    gemv(m, x, norm=2, nw=nw, nb=nb, epi=3, y=y, bias=bias)
    h = torch.nn.functional.layer_norm(x, (K,), nw, nb, 1e-5) @ m.w.T + bias
    ref = 0.5 * h * (1 + torch.tanh(math.sqrt(2 / math.pi) * (h + 0.044715 * h ** 3)))
    assert rel(y, ref) < 1e-2


@pytest.mark.parametrize("qt,K", [(GGMLType.Q4_K, 4096), (GGMLType.Q6_K, 11008), (GGMLType.Q4_K, 11008)])
def test_ws_glu(ws_on, qt, K):
    F = 1100  # 2200 rows: several tiles per compute wave, the last one partial
    m = QM(qt, 2 * F, K, seed=5)
    x = torch.randn(1, K, device="cuda")
    nw = torch.rand(K, device="cuda") + 0.5
    y = torch.zeros(1, F, device="cuda")
    gemv(m, x, norm=1, nw=nw, epi=2, y=y)
    gu = (x * torch.rsqrt(x.pow(2).mean(-1, keepdim=True) + 1e-5) * nw) @ m.w.T
    ref = torch.nn.functional.silu(gu[:, 0::2]) * gu[:, 1::2]
    assert rel(y, ref) < 1.5e-2


def test_ws_qkv_rope_kv_scatter(ws_on):
    D, n_rot, H, Hkv, K, bs = 128, 128, 8, 2, 1024, 16
    Eq, Ekv = H * D, Hkv * D
    m = QM(GGMLType.Q4_K, Eq + 2 * Ekv, K, seed=D)
    x = torch.randn(1, K, device="cuda")
    q = torch.zeros(1, Eq, device="cuda")
    kc = torch.zeros(8, Hkv, bs, D, device="cuda", dtype=torch.float16)
    vc = torch.zeros_like(kc)
    pos = torch.tensor([37], device="cuda", dtype=torch.int32)
    slot = torch.tensor([3 * bs + 5], device="cuda", dtype=torch.int32)
    inv = (10000.0 ** (-torch.arange(0, n_rot // 2, dtype=torch.float64) * 2 / n_rot)).float().cuda()
    bias = torch.randn(Eq + 2 * Ekv, device="cuda") * 0.1
    extra = dict(pos=pos.data_ptr(), slot=slot.data_ptr(), kc=kc.data_ptr(), vc=vc.data_ptr(), inv_freq=inv.data_ptr(),
                 Eq=Eq, Ekv=Ekv, D=D, n_rot=n_rot, n_kv=Hkv, bs=bs)
    gemv(m, x, epi=4, y=q, bias=bias, extra=extra)
    y = x @ m.w.T + bias

    def rope(t, nh):
        t = t.view(1, nh, D).clone()
        ang = pos.double()[:, None] * inv.double()[None, :]
        c, s = torch.cos(ang).float()[:, None, :], torch.sin(ang).float()[:, None, :]
        a, b = t[..., 0:n_rot:2].clone(), t[..., 1:n_rot:2].clone()
        t[..., 0:n_rot:2] = a * c - b * s
        t[..., 1:n_rot:2] = a * s + b * c
        return t
    assert rel(q.view(1, H, D), rope(y[:, :Eq], H)) < 1e-2
    assert rel(kc[3, :, 5].float(), rope(y[:, Eq:Eq + Ekv], Hkv)[0]) < 1.2e-2
    assert rel(vc[3, :, 5].float(), y[:, Eq + Ekv:].view(Hkv, D)) < 1.2e-2


def test_ws_wide_matrix_falls_back(ws_on):
    """More row tiles per compute wave than the kernel preloads epilogue operands for: the launcher
    declines and the flight kernel serves the call (still correct)."""
    N, K = 80000, 256
    m = QM(GGMLType.Q4_K, N, K, seed=9)
    x = torch.randn(1, K, device="cuda")
    y = torch.zeros(1, N, device="cuda")
    gemv(m, x, y=y)
    assert rel(y, x @ m.w.T) < 1e-2


@pytest.mark.parametrize("name", ["tiny-llama", "tiny-phi2", "tiny-llama-q8", "tiny-llama-q5km", "tiny-gemma"])
def test_ws_engine_vs_torch(tiny_models, name, ws_on):
    """Decode steps through the executor (dual q,k Q4_K / v Q6_K QKV side included) with the
    wave-specialised GEMV against the torch twin."""
    from ollama_operator_amd.engine.runner import Runner
    path = tiny_models[name]
    g = Runner(path, device="cuda", max_batch=8, max_seqs=2, ctx=128)
    c = Runner(path, device="cpu", max_batch=8, max_seqs=2, ctx=128)
    sg, sc = g.new_sequence(), c.new_sequence()
    g.prefill(sg, [1, 17, 42, 99])
    c.prefill(sc, [1, 17, 42, 99])
    V = g.cfg.n_vocab
    for t in [8, 9, 10, 11]:
        g.prefill(sg, [t])
        c.prefill(sc, [t])
        assert rel(g.logits[0, :V].cpu(), c.logits[0, :V]) < 3e-2
