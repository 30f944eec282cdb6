"""Batch-1 int8 activation chain (csrc/kernels/gemv8.hip) against fp32 PyTorch references: the
consumer reads a producer-written int8 image (+ RMS partials) and must equal the fp32 GEMV of the
normed input; producers (residual-add, GLU) must write the same outputs as the fp32 path AND an image
that decodes to the next input. The int8 activation rounding (per 16 elements) bounds the error."""
import numpy as np
import pytest
import torch

from ollama_operator_amd.gguf import GGMLType

from test_kernels_gpu import QM, C, S, rel

pytestmark = pytest.mark.gpu

EPI_STORE, EPI_ADD, EPI_GLU, EPI_QKV, EPI_GEGLU = 0, 1, 2, 4, 5


def make_image(x: torch.Tensor, nw: torch.Tensor | None = None):
    """Host-side reference encoder of the image layout (ops.h x8_bytes): int8(x * nw) per 16-group,
    {d, d * sum(q)} per slot, pad slot 16 of every super-block, trailing dummy; + RMS partials of x."""
    K = x.numel()
    xs = (x * nw if nw is not None else x).float().cpu().numpy()
    SB = (K + 255) // 256
    slots = C().x8_slots(K)
    q = np.zeros((slots, 16), np.int8)
    f = np.zeros((slots, 2), np.float32)
    for gi in range(K // 16):
        v = xs[16 * gi:16 * gi + 16]
        amax = np.abs(v).max()
        d = np.float32(amax / 127.0)
        qq = np.rint(v * (127.0 / amax)).astype(np.int32) if amax > 0 else np.zeros(16, np.int32)
        slot = (gi // 16) * 17 + gi % 16
        q[slot] = qq.astype(np.int8)
        f[slot] = (d, d * qq.sum())
    img = np.concatenate([q.reshape(-1).view(np.uint8), f.reshape(-1).view(np.uint8)])
    assert img.nbytes == C().x8_bytes(K) and SB * 17 < slots
    st = (x.float().reshape(-1, 16) ** 2).sum(1).cpu()
    return torch.from_numpy(img).cuda(), torch.cat([st, torch.zeros(4)]).cuda()


def decode_image(img: torch.Tensor, K: int) -> torch.Tensor:
    slots = C().x8_slots(K)
    a = img.cpu().numpy()
    q = a[:slots * 16].view(np.int8).reshape(slots, 16).astype(np.float32)
    f = a[slots * 16:].view(np.float32).reshape(slots, 2)
    out = np.zeros(K, np.float32)
    for gi in range(K // 16):
        slot = (gi // 16) * 17 + gi % 16
        out[16 * gi:16 * gi + 16] = q[slot] * f[slot, 0]
    return torch.from_numpy(out)


def call(m, B, x, y, epi, ops, ldy=None):
    C().reset_launch_counts()
    C().gemv(m.tup, B, x.data_ptr() if x is not None else 0, m.tup[5], 0, 0, 0, 1e-5, epi, y.data_ptr(),
             ldy or y.shape[-1], 0, 0, ops, S())
    n = C().launch_counts()  # the int8-chain kernel ran, not the fp32-prologue fallback
    assert n["gemv8_row1" if B == 1 else "gemv8_rows"] == 1 and n["gemv_flight"] == 0, n


@pytest.mark.parametrize("qt", [GGMLType.Q4_K, GGMLType.Q6_K, GGMLType.Q4_0, GGMLType.Q8_0, GGMLType.Q5_K])
@pytest.mark.parametrize("K", [4096, 11008, 8192])
def test_consumer_rms_store(qt, K):
    """K = 4096: an RMSNorm'd input (QKV / gate_up / LM head shape); K = 11008: the un-normed GLU output
    (down's input, in-block K split over 3 wave groups); K = 8192 over > 512 row tiles: two super-blocks
    per lane, unsplit, four image words per thread (Llama-2-70B's QKV / LM head)."""
    N = {4096: 1024, 11008: 512, 8192: 8320}[K]
    m = QM(qt, N, K, seed=K + int(qt))
    x = torch.randn(K, device="cuda") * 2
    rms = K != 11008
    nw = torch.rand(K, device="cuda") + 0.5 if rms else None
    img, st = make_image(x, nw)
    y = torch.zeros(1, N, device="cuda")
    ops = {"x8": img.data_ptr()}
    if rms:
        ops["x8_stat"] = st.data_ptr()
    call(m, 1, None, y, EPI_STORE, ops)
    xn = x * torch.rsqrt(x.pow(2).mean() + 1e-5) * nw if rms else x
    ref = (xn @ m.w.T)[None]
    assert rel(y, ref) < 1.5e-2


@pytest.mark.parametrize("qt", [GGMLType.Q4_K, GGMLType.Q6_K])
def test_residual_producer_emits_next_input(qt):
    """O / down shape: EPI_ADD into the residual, image of (new resid * next norm w) + partials."""
    N, K = 4096, 11008
    m = QM(qt, N, K, seed=5)
    h = torch.randn(K, device="cuda")
    img_in, _ = make_image(h)
    resid0 = torch.randn(1, N, device="cuda") * 4
    resid = resid0.clone()
    nw = torch.rand(N, device="cuda") + 0.5
    out = torch.zeros(C().x8_bytes(N), dtype=torch.uint8, device="cuda")
    st = torch.zeros(N // 16 + 4, device="cuda")
    call(m, 1, None, resid, EPI_ADD, {"x8": img_in.data_ptr(), "emit8": out.data_ptr(),
                                      "emit8_nw": nw.data_ptr(), "emit8_stat": st.data_ptr()})
    ref = resid0 + (h @ m.w.T)[None]
    assert rel(resid - resid0, ref - resid0) < 1.5e-2
    # the emitted image decodes to (new resid * nw) within int8 rounding, partials = group sums of squares
    dec = decode_image(out, N)
    want = (resid[0] * nw).cpu()
    assert rel(dec, want) < 1e-2
    assert torch.allclose(st[:N // 16].cpu(), (resid[0].cpu().reshape(-1, 16) ** 2).sum(1), rtol=1e-4, atol=1e-3)


@pytest.mark.parametrize("act", [EPI_GLU, EPI_GEGLU])
def test_glu_producer_emits_down_input(act):
    """gate_up shape (interleaved gate/up rows): h written to y and emitted as down's image."""
    F, K = 11008, 4096
    m = QM(GGMLType.Q4_K, 2 * F, K, seed=9)
    x = torch.randn(K, device="cuda")
    nw = torch.rand(K, device="cuda") + 0.5
    img, st = make_image(x, nw)
    y = torch.zeros(1, F, device="cuda")
    out = torch.zeros(C().x8_bytes(F), dtype=torch.uint8, device="cuda")
    call(m, 1, None, y, act, {"x8": img.data_ptr(), "x8_stat": st.data_ptr(), "emit8": out.data_ptr()})
    xn = x * torch.rsqrt(x.pow(2).mean() + 1e-5) * nw
    gu = xn @ m.w.T
    g, u = gu[0::2], gu[1::2]
    hact = torch.nn.functional.silu(g) if act == EPI_GLU else torch.nn.functional.gelu(g, approximate="tanh")
    ref = hact * u
    assert rel(y[0], ref) < 2e-2
    assert rel(decode_image(out, F), y[0].cpu()) < 1e-2


@pytest.mark.parametrize("qt,K", [(GGMLType.Q4_0, 28672), (GGMLType.Q4_K, 28672), (GGMLType.Q6_K, 20480)])
@pytest.mark.parametrize("emit", [False, True])
def test_wide_k_down_two_superblocks_per_lane(qt, K, emit):
    """Llama-2-70B ffn_down (K = 28672 = 112 super-blocks): two super-blocks per lane at a 4-way in-block
    K split (Q4_0 / Q4_K; Q6_K at a 3-way split, K <= 24576); the residual add with the next RMSNorm'd
    image, or the plain store of a TP partial."""
    N = 512
    m = QM(qt, N, K, seed=21 + int(qt))
    h = torch.randn(K, device="cuda")
    img_in, _ = make_image(h)
    resid0 = torch.randn(1, N, device="cuda") * 4
    resid = resid0.clone()
    ops = {"x8": img_in.data_ptr()}
    if emit:
        nw = torch.rand(N, device="cuda") + 0.5
        out = torch.zeros(C().x8_bytes(N), dtype=torch.uint8, device="cuda")
        st = torch.zeros(N // 16 + 4, device="cuda")
        ops.update(emit8=out.data_ptr(), emit8_nw=nw.data_ptr(), emit8_stat=st.data_ptr())
    call(m, 1, None, resid, EPI_ADD if emit else EPI_STORE, ops)
    ref = (h @ m.w.T)[None]
    got = resid - resid0 if emit else resid
    assert rel(got, ref) < 1.5e-2
    if emit:
        assert rel(decode_image(out, N), (resid[0] * nw).cpu()) < 1e-2


@pytest.mark.parametrize("qt", [GGMLType.Q4_0, GGMLType.Q4_K, GGMLType.Q6_K])
@pytest.mark.parametrize("N,K,mode", [(2560, 10240, 2), (4096, 11008, 2), (512, 13824, 0)])
def test_k_split_across_blocks(qt, N, K, mode):
    """K-split down projections with two blocks per row tile (GemvParams::kb): forced on Phi-2 / 7B shapes,
    the auto rule at 13B's K (Q6_K). Residual add + emitted image match the fp32 reference and the tile
    tickets re-arm (the same launch three times)."""
    m = QM(qt, N, K, seed=31 + int(qt))
    h = torch.randn(K, device="cuda")
    img_in, _ = make_image(h)
    nw = torch.rand(N, device="cuda") + 0.5
    kb_ws = torch.zeros(2 * N + 64, device="cuda")
    kb_cnt = torch.zeros((N + 15) // 16, dtype=torch.int32, device="cuda")
    C().set_gemv8_kb(mode)
    try:
        for _ in range(3):
            resid0 = torch.randn(1, N, device="cuda") * 4
            resid = resid0.clone()
            out = torch.zeros(C().x8_bytes(N), dtype=torch.uint8, device="cuda")
            st = torch.zeros(N // 16 + 4, device="cuda")
            call(m, 1, None, resid, EPI_ADD, {"x8": img_in.data_ptr(), "emit8": out.data_ptr(), "emit8_nw": nw.data_ptr(),
                                              "emit8_stat": st.data_ptr(), "kb_ws": kb_ws.data_ptr(),
                                              "kb_cnt": kb_cnt.data_ptr()})
            torch.cuda.synchronize()
            assert rel(resid - resid0, (h @ m.w.T)[None]) < 1.5e-2
            assert rel(decode_image(out, N), (resid[0] * nw).cpu()) < 1e-2
            assert int(kb_cnt.abs().sum()) == 0
    finally:
        C().set_gemv8_kb(0)


@pytest.mark.parametrize("S_", [1, 2, 4])
def test_merge_producer(S_):
    """O projection: deferred flash-decode partial slabs (or a plain fp32 row) in, residual + image out."""
    N, K, D = 4096, 4096, 128
    m = QM(GGMLType.Q4_K, N, K, seed=11)
    nh = K // D
    acc = torch.randn(S_, K, device="cuda")
    mx = torch.randn(S_, nh, device="cuda")
    l = torch.rand(S_, nh, device="cuda") + 0.5
    if S_ > 1:
        ml = torch.stack([mx, l], -1).contiguous()
        wgt = torch.exp(mx - mx.max(0).values)  # [S, nh]
        x = (acc.view(S_, nh, D) * wgt[..., None]).sum(0) / (wgt * l).sum(0)[:, None]
        x = x.reshape(K)
        ops = {"merge_S": S_, "merge_ml": ml.data_ptr(), "merge_D": D}
    else:
        x = acc[0]
        ops = {}
    resid0 = torch.randn(1, N, device="cuda")
    resid = resid0.clone()
    nw = torch.rand(N, device="cuda") + 0.5
    out = torch.zeros(C().x8_bytes(N), dtype=torch.uint8, device="cuda")
    st = torch.zeros(N // 16 + 4, device="cuda")
    ops.update(emit8=out.data_ptr(), emit8_nw=nw.data_ptr(), emit8_stat=st.data_ptr())
    call(m, 1, acc, resid, EPI_ADD, ops)
    ref = resid0 + (x @ m.w.T)[None]
    assert rel(resid - resid0, ref - resid0) < 1.5e-2
    assert rel(decode_image(out, N), (resid[0] * nw).cpu()) < 1e-2


def test_engine_x8_chain_on_and_matches_torch(tmp_path):
    """Llama Q4_K_M batch-1 decode through the executor: the chain is on (every emitter covered) and
    teacher-forced decode steps (graph replays of the decode path, where the chain runs) track the fp32
    torch twin's logits."""
    from ollama_operator_amd.engine.runner import Runner
    from ollama_operator_amd.gguf.constants import FileType
    from ollama_operator_amd.models.config import preset
    from ollama_operator_amd.models.random_init import write_random_gguf
    p = str(tmp_path / "m.gguf")
    write_random_gguf(p, preset("tiny-llama"), FileType.MOSTLY_Q4_K_M, seed=4, quantize_from_float=True)
    g = Runner(p, device="cuda:0", max_batch=16, max_seqs=1, ctx=256)
    assert g.exe.exe.x8_on == 1
    c = Runner(p, device="cpu", max_batch=16, max_seqs=1, ctx=256, cpu_backend="torch")
    prompt = [1, 17, 33, 49, 65]
    sg, sc = g.new_sequence(), c.new_sequence()
    g.prefill(sg, prompt)
    c.prefill(sc, prompt)
    V = g.cfg.n_vocab
    L = g.cfg.n_layer
    for i, t in enumerate([8, 9, 10, 11, 12]):
        g.set_tokens([t])
        eager = i == 4  # the last step eagerly: launch counters count enqueues, a graph replay enqueues none
        g.use_graphs = not eager
        C().reset_launch_counts()
        g.decode_step(sg)
        torch.cuda.synchronize()
        if eager:
            n = C().launch_counts()
            # every projection of every layer on the int8 chain (QKV, O, gate_up, down; LM head); only
            # layer 0's QKV reads the embedding rows through the fp32 prologue
            assert n["gemv8_row1"] + n["gemv8_dual"] >= 4 * L and n["gemv_flight"] <= 1, n
        g.kv.seqs[sg].tokens.append(t)
        c.prefill(sc, [t])
        assert rel(g.logits[0, :V].cpu(), c.logits[0, :V]) < 3e-2


@pytest.mark.parametrize("ftype", ["MOSTLY_Q4_0", "MOSTLY_Q4_K_M"])
def test_engine_phi2_ln_chain_matches_torch(tmp_path, ftype):
    """Phi-2 batch-1 decode on the LayerNorm form of the int8 chain (executor.cpp ln8): down emits
    x * ln_w with per-group sums and sums of squares, QKV / FFN up / the LM head apply
    rstd * (dot - mu * c1) + c2 (engine/weights.py _ln_consts), FFN up emits gelu(.) for down.
    Teacher-forced decode steps track the fp32 torch twin; with the chain off (OMX_X8_LN=0) the fp32
    LayerNorm prologue path gives the same logits."""
    import os
    from ollama_operator_amd.engine.runner import Runner
    from ollama_operator_amd.gguf.constants import FileType
    from ollama_operator_amd.models.config import preset
    from ollama_operator_amd.models.random_init import write_random_gguf
    p = str(tmp_path / "phi.gguf")
    write_random_gguf(p, preset("tiny-phi2"), getattr(FileType, ftype), seed=6, quantize_from_float=True)
    g = Runner(p, device="cuda:0", max_batch=16, max_seqs=1, ctx=256)
    assert g.exe.exe.x8_on == 1
    os.environ["OMX_X8_LN"] = "0"
    try:
        g0 = Runner(p, device="cuda:0", max_batch=16, max_seqs=1, ctx=256)
    finally:
        del os.environ["OMX_X8_LN"]
    assert g0.exe.exe.x8_on == 0
    c = Runner(p, device="cpu", max_batch=16, max_seqs=1, ctx=256, cpu_backend="torch")
    prompt = [1, 17, 33, 49, 65]
    sg, s0, sc = g.new_sequence(), g0.new_sequence(), c.new_sequence()
    for r, sid in ((g, sg), (g0, s0), (c, sc)):
        r.prefill(sid, prompt)
    V = g.cfg.n_vocab
    L = g.cfg.n_layer
    for i, t in enumerate([8, 9, 10, 11, 12]):
        eager = i == 4
        outs = []
        for r, sid in ((g, sg), (g0, s0)):
            r.set_tokens([t])
            r.use_graphs = not eager
            C().reset_launch_counts()
            r.decode_step(sid)
            torch.cuda.synchronize()
            if eager and r is g:
                n = C().launch_counts()
                # QKV + FFN up (one dual launch) and O + down (one pair launch, gemv8_pair.hip, when both
                # have the same quant type) of every layer plus the LM head on the chain
                assert n["gemv8_dual"] == L, n
                if ftype == "MOSTLY_Q4_0":
                    assert n["gemv8_pair"] == L and n["gemv_flight"] == 0, n
                else:  # per layer: the pair, or O apart (fp32 rows at this length: gemv.hip) and down on gemv8
                    assert n["gemv8_pair"] + n["gemv_flight"] == L, n
            r.kv.seqs[sid].tokens.append(t)
            outs.append(r.logits[0, :V].float().cpu().clone())
        c.prefill(sc, [t])
        assert rel(outs[0], c.logits[0, :V]) < 3e-2, i
        assert rel(outs[0], outs[1]) < 2e-2, i


def test_engine_phi2_pair_deferred_splits(tmp_path):
    """Phi-2 Q4_0 decode with O + ffn_down in one launch (gemv8_pair.hip) at lengths in every deferred split
    bucket (the pair kernel merges 1 / 2 / 4 / 8 attention slabs itself): logits track the fp32 torch twin
    and every layer took the pair launch."""
    from ollama_operator_amd.engine.runner import Runner
    from ollama_operator_amd.gguf.constants import FileType
    from ollama_operator_amd.models.config import preset
    from ollama_operator_amd.models.random_init import write_random_gguf
    p = str(tmp_path / "phi.gguf")
    write_random_gguf(p, preset("tiny-phi2", ctx_len=2048), FileType.MOSTLY_Q4_0, seed=8, quantize_from_float=True)
    g = Runner(p, device="cuda:0", max_batch=64, max_seqs=1, ctx=1100)
    assert g.exe.exe.x8_on == 1 and g._defer_ok
    g.use_graphs = False  # launch counters count enqueues
    c = Runner(p, device="cpu", max_batch=64, max_seqs=1, ctx=1100, cpu_backend="torch")
    rng = np.random.default_rng(5)
    V, L = g.cfg.n_vocab, g.cfg.n_layer
    seen = set()
    for n_keys in (60, 200, 400, 900):
        toks = [1] + [int(x) for x in rng.integers(3, 500, n_keys - 1)]
        seen.add(g.decode_splits(n_keys + 1))
        sg, sc = g.new_sequence(), c.new_sequence()
        g.prefill(sg, toks)
        c.prefill(sc, toks + [77])
        g.d_tokens[0] = 77
        C().reset_launch_counts()
        g.decode_step(sg, n_keys)
        torch.cuda.synchronize()
        n = C().launch_counts()
        assert n["gemv8_pair"] == L and n["gemv_flight"] == 0, (n_keys, n)
        assert rel(g.logits[0, :V].float().cpu(), c.logits[0, :V]) < 3e-2, n_keys
        g.free_sequence(sg)
        c.free_sequence(sc)
    assert seen == {1, 2, 4, 8}


def images(xs, nw=None):
    """B rows -> the batched image buffer (row b at b * x8_bytes(K)) and RMS partials (stride x8_stat_ld)."""
    K = xs.shape[1]
    ld = C().x8_stat_ld(K)
    imgs, sts = [], torch.zeros(xs.shape[0] * ld + 4, device="cuda")
    for b in range(xs.shape[0]):
        img, st = make_image(xs[b], nw)
        imgs.append(img)
        sts[b * ld:b * ld + K // 16] = st[:K // 16]
    return torch.cat(imgs), sts


@pytest.mark.parametrize("B", [2, 3, 4])
def test_batched_rows_consumer_and_producers(B):
    """Every chain kernel with B rows: RMS consumer (QKV / gate_up / head shape), GLU producer, residual
    producer (down, K split over 3 wave groups) and the O projection on plain fp32 attention rows -- each
    row equal to its own fp32 reference, emitted images per row."""
    E, F = 4096, 11008
    x = torch.randn(B, E, device="cuda") * 2
    nw = torch.rand(E, device="cuda") + 0.5
    img, st = images(x, nw)
    xn = x * torch.rsqrt(x.pow(2).mean(1, keepdim=True) + 1e-5) * nw
    # consumer (store)
    m = QM(GGMLType.Q4_K, 1024, E, seed=31)
    y = torch.zeros(B, 1024, device="cuda")
    call(m, B, None, y, EPI_STORE, {"x8": img.data_ptr(), "x8_stat": st.data_ptr()})
    assert rel(y, xn @ m.w.T) < 1.5e-2
    # GLU producer: h rows + down's images
    mg = QM(GGMLType.Q4_K, 2 * F, E, seed=32)
    h = torch.zeros(B, F, device="cuda")
    himg = torch.zeros(B * C().x8_bytes(F), dtype=torch.uint8, device="cuda")
    call(mg, B, None, h, EPI_GLU, {"x8": img.data_ptr(), "x8_stat": st.data_ptr(), "emit8": himg.data_ptr()})
    gu = xn @ mg.w.T
    assert rel(h, torch.nn.functional.silu(gu[:, 0::2]) * gu[:, 1::2]) < 2e-2
    nbF = C().x8_bytes(F)
    for b in range(B):
        assert rel(decode_image(himg[b * nbF:(b + 1) * nbF], F), h[b].cpu()) < 1e-2, b
    # residual producer (down): K = 11008 split over 3 wave groups
    for qd in (GGMLType.Q4_K, GGMLType.Q6_K):
        md = QM(qd, E, F, seed=33)
        resid0 = torch.randn(B, E, device="cuda") * 4
        resid = resid0.clone()
        nw2 = torch.rand(E, device="cuda") + 0.5
        out = torch.zeros(B * C().x8_bytes(E), dtype=torch.uint8, device="cuda")
        ld = C().x8_stat_ld(E)
        sto = torch.zeros(B * ld + 4, device="cuda")
        call(md, B, None, resid, EPI_ADD, {"x8": himg.data_ptr(), "emit8": out.data_ptr(), "emit8_nw": nw2.data_ptr(),
                                           "emit8_stat": sto.data_ptr()})
        hq = torch.stack([decode_image(himg[b * nbF:(b + 1) * nbF], F) for b in range(B)]).cuda()
        assert rel(resid - resid0, hq @ md.w.T) < 1.5e-2, qd
        nbE = C().x8_bytes(E)
        for b in range(B):
            assert rel(decode_image(out[b * nbE:(b + 1) * nbE], E), (resid[b] * nw2).cpu()) < 1e-2, (qd, b)
            assert torch.allclose(sto[b * ld:b * ld + E // 16].cpu(), (resid[b].cpu().reshape(-1, 16) ** 2).sum(1),
                                  rtol=1e-4, atol=1e-3), (qd, b)
    # O projection: plain fp32 attention rows in (int8-quantised in the prologue), residual + image out
    mo = QM(GGMLType.Q4_K, E, E, seed=34)
    a = torch.randn(B, E, device="cuda")
    resid0 = torch.randn(B, E, device="cuda")
    resid = resid0.clone()
    out = torch.zeros(B * C().x8_bytes(E), dtype=torch.uint8, device="cuda")
    sto = torch.zeros(B * C().x8_stat_ld(E) + 4, device="cuda")
    call(mo, B, a, resid, EPI_ADD, {"emit8": out.data_ptr(), "emit8_nw": nw.data_ptr(), "emit8_stat": sto.data_ptr()})
    assert rel(resid - resid0, a @ mo.w.T) < 1.5e-2


@pytest.mark.parametrize("B", [2, 3, 4])
def test_engine_batched_x8_chain_matches_single(tiny_models, B, monkeypatch):
    """Continuous-batching decode steps of B = 2..4 rows on the int8 chain (one weight read for all rows)
    against each sequence's own batch-1 step."""
    from ollama_operator_amd.engine.runner import Runner
    monkeypatch.setenv("OMX_X8_BATCH", "4")
    g = Runner(tiny_models["tiny-llama"], device="cuda", max_batch=32, max_seqs=8, ctx=256)
    assert g.exe.exe.x8_bmax == 4
    rng = np.random.default_rng(B)
    prompts = [[1] + [int(x) for x in rng.integers(3, 500, n)] for n in (5, 40, 17, 90)[:B]]
    sids = []
    for p in prompts:
        sid = g.new_sequence()
        g.prefill(sid, p)
        sids.append(sid)
    V = g.cfg.n_vocab
    nxt = [7, 8, 9, 10][:B]
    g.set_tokens(nxt)
    g.decode_batch(sids, [len(p) for p in prompts])
    torch.cuda.synchronize()
    batched = g.logits[:B, :V].float().cpu().clone()
    assert torch.isfinite(batched).all()
    for b, (sid, p) in enumerate(zip(sids, prompts)):
        g.set_tokens([nxt[b]])
        g.decode_batch([sid], [len(p)])
        torch.cuda.synchronize()
        assert rel(batched[b], g.logits[0, :V].float().cpu()) < 3e-2, b


@pytest.mark.parametrize("qd", [GGMLType.Q4_0, GGMLType.Q4_K, GGMLType.Q6_K])
@pytest.mark.parametrize("F", [14336, 13824])
def test_batched_rows_down_ks4(qd, F):
    """2 batch rows on the residual producer at K = 14336 (Mistral-7B / Llama-3-8B down: 56 super-blocks,
    the in-block K split over 4 wave groups, 1024-thread blocks) and K = 13824 (Llama-2-13B: 54, the
    balanced 14 / 14 / 14 / 12 split)"""
    B, E = 2, 4096
    h = torch.randn(B, F, device="cuda")
    nbF = C().x8_bytes(F)
    himg = torch.zeros(B * nbF, dtype=torch.uint8, device="cuda")
    for b in range(B):
        img, _ = make_image(h[b])
        himg[b * nbF:(b + 1) * nbF] = img
    md = QM(qd, E, F, seed=35)
    resid0 = torch.randn(B, E, device="cuda") * 4
    resid = resid0.clone()
    nw2 = torch.rand(E, device="cuda") + 0.5
    out = torch.zeros(B * C().x8_bytes(E), dtype=torch.uint8, device="cuda")
    ld = C().x8_stat_ld(E)
    sto = torch.zeros(B * ld + 4, device="cuda")
    call(md, B, None, resid, EPI_ADD, {"x8": himg.data_ptr(), "emit8": out.data_ptr(), "emit8_nw": nw2.data_ptr(),
                                       "emit8_stat": sto.data_ptr()})
    torch.cuda.synchronize()
    hq = torch.stack([decode_image(himg[b * nbF:(b + 1) * nbF], F) for b in range(B)]).cuda()
    assert rel(resid - resid0, hq @ md.w.T) < 1.5e-2, qd
    nbE = C().x8_bytes(E)
    for b in range(B):
        assert rel(decode_image(out[b * nbE:(b + 1) * nbE], E), (resid[b] * nw2).cpu()) < 1e-2, (qd, b)


@pytest.mark.parametrize("qt", [GGMLType.Q4_K, GGMLType.Q6_K, GGMLType.Q4_0])
@pytest.mark.parametrize("B,K", [(1, 5120), (3, 5120), (4, 5120), (1, 8192), (2, 8192)])
def test_plain_o_projection_k_split(qt, B, K):
    """O projection on plain fp32 attention rows at 4096 < K <= 8192 (Llama-2-13B: H * D = 5120): the
    quantising prologue over a block split in 2 wave groups. Before, such an O left the whole model off
    the int8 chain (Llama-2-13B decoded on the fp32 GEMVs at 308 tok/s)."""
    E = 5120
    mo = QM(qt, E, K, seed=K + B)
    a = torch.randn(B, K, device="cuda")
    resid0 = torch.randn(B, E, device="cuda")
    resid = resid0.clone()
    nw = torch.rand(E, device="cuda") + 0.5
    nbE, ld = C().x8_bytes(E), C().x8_stat_ld(E)
    out = torch.zeros(B * nbE, dtype=torch.uint8, device="cuda")
    sto = torch.zeros(B * ld + 4, device="cuda")
    call(mo, B, a, resid, EPI_ADD, {"emit8": out.data_ptr(), "emit8_nw": nw.data_ptr(), "emit8_stat": sto.data_ptr()})
    torch.cuda.synchronize()
    assert rel(resid - resid0, a @ mo.w.T) < 1.5e-2
    for b in range(B):
        assert rel(decode_image(out[b * nbE:(b + 1) * nbE], E), (resid[b] * nw).cpu()) < 1e-2, b


def test_engine_x8_chain_covers_13b_shapes(tmp_path, monkeypatch):
    """A 2-layer model with Llama-2-13B's widths (E = 5120, 40 heads, F = 13824) decodes on the int8
    chain and matches the fp32 torch twin."""
    from ollama_operator_amd.engine.runner import Runner
    from ollama_operator_amd.gguf.constants import FileType
    from ollama_operator_amd.models.config import preset
    from ollama_operator_amd.models.random_init import write_random_gguf
    import dataclasses
    cfg = dataclasses.replace(preset("llama2-13b", ctx_len=512), n_layer=2, n_vocab=512)
    p = str(tmp_path / "m.gguf")
    write_random_gguf(p, cfg, FileType.MOSTLY_Q4_K_M, seed=3, quantize_from_float=True)
    monkeypatch.setenv("OMX_DEFER_KSPLIT", "1")  # opt-in: K = 5120, the int8-chain O merges the deferred slabs
    g = Runner(p, device="cuda:0", max_batch=64, max_seqs=1, ctx=512)
    assert g.exe.exe.x8_on == 1 and g._defer_ok
    g.use_graphs = False  # launch counters count enqueues
    c = Runner(p, device="cpu", max_batch=64, max_seqs=1, ctx=512, cpu_backend="torch")
    prompt = [1] + [(11 * i + 3) % 500 for i in range(1, 20)]
    sids = {id(r): r.new_sequence() for r in (g, c)}
    for r in (g, c):
        r.prefill(sids[id(r)], prompt)
    V = g.cfg.n_vocab
    for t in (5, 6):
        C().reset_launch_counts()
        g.set_tokens([t])
        g.decode_step(sids[id(g)])
        torch.cuda.synchronize()
        n = C().launch_counts()
        # every projection on the chain (layer 0's QKV reads the embedding's image; a q,k / v pair of
        # different quant types takes the two-super-blocks-per-lane dual launch); the 512-row LM head may
        # take either path
        assert n["gemv8_row1"] + n["gemv8_dual"] >= 4 * 2 and n["gemv_flight"] <= 1, sorted(n.items())
        g.kv.seqs[sids[id(g)]].tokens.append(t)
        c.prefill(sids[id(c)], [t])
        assert rel(g.logits[0, :V].float().cpu(), c.logits[0, :V]) < 3e-2
    # past 128 / 256 keys: 2 / 4 deferred attention splits, merged in the O GEMV's prologue at a 2-way K split
    for r in (g, c):
        r.free_sequence(sids[id(r)])
    rng = np.random.default_rng(9)
    for n_keys in (200, 400):
        toks = [1] + [int(x) for x in rng.integers(3, 500, n_keys - 1)]
        sg, sc = g.new_sequence(), c.new_sequence()
        g.prefill(sg, toks)
        c.prefill(sc, toks + [77])
        g.d_tokens[0] = 77
        assert g.decode_splits(n_keys + 1) in (2, 4)
        C().reset_launch_counts()
        g.decode_step(sg, n_keys)
        torch.cuda.synchronize()
        n = C().launch_counts()
        assert n["gemv_flight"] <= 1, n
        assert rel(g.logits[0, :V].float().cpu(), c.logits[0, :V]) < 3e-2, n_keys
        g.free_sequence(sg)
        c.free_sequence(sc)


@pytest.mark.parametrize("B", [1, 2])
@pytest.mark.parametrize("qt", [GGMLType.Q4_K, GGMLType.Q4_0])
def test_glu_producer_two_superblocks_per_lane(B, qt):
    """gate_up at K = 5120 (Llama-2-13B): 1728 row tiles take two super-blocks per lane and two tiles
    per block (NSB = 2, J = 2); h rows and down's images per row."""
    E, F = 5120, 13824
    x = torch.randn(B, E, device="cuda") * 2
    nw = torch.rand(E, device="cuda") + 0.5
    img, st = images(x, nw)
    xn = x * torch.rsqrt(x.pow(2).mean(1, keepdim=True) + 1e-5) * nw
    mg = QM(qt, 2 * F, E, seed=36 + B)
    h = torch.zeros(B, F, device="cuda")
    nbF = C().x8_bytes(F)
    himg = torch.zeros(B * nbF, dtype=torch.uint8, device="cuda")
    call(mg, B, None, h, EPI_GLU, {"x8": img.data_ptr(), "x8_stat": st.data_ptr(), "emit8": himg.data_ptr()})
    torch.cuda.synchronize()
    gu = xn @ mg.w.T
    assert rel(h, torch.nn.functional.silu(gu[:, 0::2]) * gu[:, 1::2]) < 2e-2
    for b in range(B):
        assert rel(decode_image(himg[b * nbF:(b + 1) * nbF], F), h[b].cpu()) < 1e-2, b
