"""GPU: the native executor (HIP kernels) against the torch twin on the same repacked weights."""
import numpy as np
import pytest
import torch

from ollama_operator_amd.engine.runner import Runner
from ollama_operator_amd.engine.sampling import SamplingOptions
from ollama_operator_amd.ops import native

pytestmark = pytest.mark.gpu


def rel(a, b):
    return float((a - b).norm() / (b.norm() + 1e-12))


@pytest.mark.parametrize("name", ["tiny-llama", "tiny-mixtral", "tiny-phi2", "tiny-llama-q8", "tiny-llama-q40",
                                  "tiny-llama-q5km", "tiny-mixtral-q5ks", "tiny-gemma", "tiny-orca"])
def test_native_vs_torch_teacher_forced(tiny_models, name):
    path = tiny_models[name]
    g = Runner(path, device="cuda", max_batch=8, max_seqs=2, ctx=128)
    c = Runner(path, device="cpu", max_batch=8, max_seqs=2, ctx=128)
    sg, sc = g.new_sequence(), c.new_sequence()
    toks = [1, 17, 42, 99, 7, 300, 12, 5, 77, 200, 3]
    g.prefill(sg, toks)
    c.prefill(sc, toks)
    V = g.cfg.n_vocab
    assert rel(g.logits[0, :V].cpu(), c.logits[0, :V]) < 3e-2
    for t in [8, 9, 10]:  # single-token steps (decode shape)
        g.prefill(sg, [t])
        c.prefill(sc, [t])
        assert rel(g.logits[0, :V].cpu(), c.logits[0, :V]) < 3e-2


def test_graph_decode_matches_eager(tiny_models):
    path = tiny_models["tiny-llama"]
    o = SamplingOptions(temperature=0.7, top_k=20, top_p=0.95, seed=99)
    a = Runner(path, device="cuda", max_batch=8, max_seqs=2, ctx=128, use_graphs=True)
    b = Runner(path, device="cuda", max_batch=8, max_seqs=2, ctx=128, use_graphs=False, weights=a.w)
    ta = list(a.generate(a.new_sequence(), [1, 2, 3, 4], o, max_tokens=24))
    tb = list(b.generate(b.new_sequence(), [1, 2, 3, 4], o, max_tokens=24))
    assert ta == tb
    assert len(ta) == 24


def test_long_context_splits(tiny_models):
    """Prefill past several KV blocks and attention splits; compare with the torch twin."""
    path = tiny_models["tiny-llama"]
    g = Runner(path, device="cuda", max_batch=32, max_seqs=1, ctx=256)
    c = Runner(path, device="cpu", max_batch=32, max_seqs=1, ctx=256)
    rng = np.random.default_rng(0)
    toks = [int(x) for x in rng.integers(3, 500, 150)]
    sg, sc = g.new_sequence(), c.new_sequence()
    g.prefill(sg, toks)
    c.prefill(sc, toks)
    V = g.cfg.n_vocab
    assert rel(g.logits[0, :V].cpu(), c.logits[0, :V]) < 3e-2


@pytest.mark.parametrize("name", ["tiny-llama", "tiny-mixtral", "tiny-phi2", "tiny-llama-q8", "tiny-llama-q40",
                                  "tiny-llama-q5km", "tiny-mixtral-q5ks", "tiny-gemma", "tiny-orca"])
def test_prefill_gemm_path_vs_torch(tiny_models, name):
    """Prompts >= GEMM_MIN_B take the MFMA GEMM path (and, for Mixtral, the device-sorted grouped
    expert GEMM with the routing-weighted scatter); logits must match the torch twin."""
    path = tiny_models[name]
    g = Runner(path, device="cuda", max_batch=64, max_seqs=2, ctx=160)
    c = Runner(path, device="cpu", max_batch=64, max_seqs=2, ctx=160)
    rng = np.random.default_rng(1)
    toks = [1] + [int(x) for x in rng.integers(3, 500, 69)]
    sg, sc = g.new_sequence(), c.new_sequence()
    g.prefill(sg, toks)
    c.prefill(sc, toks)
    V = g.cfg.n_vocab
    assert rel(g.logits[0, :V].cpu(), c.logits[0, :V]) < 3e-2
    g.prefill(sg, [5])  # then a decode-shaped step on the KV the GEMM path wrote
    c.prefill(sc, [5])
    assert rel(g.logits[0, :V].cpu(), c.logits[0, :V]) < 3e-2


@pytest.mark.parametrize("name", ["tiny-llama", "tiny-mixtral", "tiny-phi2", "tiny-llama-q8", "tiny-llama-q40",
                                  "tiny-llama-q5km", "tiny-gemma", "tiny-orca"])
def test_prefill_dq_path_vs_torch(tiny_models, name, monkeypatch):
    """Prompts >= 128 tokens take the stream-order dequant GEMM (gemm_dq.hip, the default prefill path;
    no fp16 weight copy exists): logits must match the torch twin, before and after a decode step on the
    KV it wrote."""
    C = native()
    assert C.dq_gemm_enabled() and (C.gemm_lib_min_m() == 0 or C.gemm_lib_min_m() > 230)
    path = tiny_models[name]
    g = Runner(path, device="cuda", max_batch=256, max_seqs=2, ctx=256)
    c = Runner(path, device="cpu", max_batch=256, max_seqs=2, ctx=256)
    rng = np.random.default_rng(4)
    toks = [1] + [int(x) for x in rng.integers(3, 500, 229)]
    sg, sc = g.new_sequence(), c.new_sequence()
    C.reset_launch_counts()
    g.prefill(sg, toks)
    n = C.launch_counts()  # every dense projection ran on the dq kernel, none fell back to the tile GEMM
    assert n["dq_gemm"] >= 2 * g.cfg.n_layer and n["gemm_tile"] == 0 and n["gemm_lib"] == 0, n
    c.prefill(sc, toks)
    V = g.cfg.n_vocab
    assert rel(g.logits[0, :V].cpu(), c.logits[0, :V]) < 3e-2
    g.prefill(sg, [5])
    c.prefill(sc, [5])
    assert rel(g.logits[0, :V].cpu(), c.logits[0, :V]) < 3e-2


def test_moe_prefill_experts_on_library_by_default(tiny_models):
    """MoE prefill: from moe_lib_min_m() routed pairs (default 256) each expert's GEMM runs on hipBLASLt
    over its per-call dequantised weights (gemm.hip moe_gemm_lib) while every dense projection stays on
    the hand-written kernel (gemm_lib_min_m() == 0): the expert scratch is used and logits match."""
    C = native()
    assert C.gemm_lib_min_m() == 0 and C.moe_lib_min_m() > 0
    path = tiny_models["tiny-mixtral"]
    g = Runner(path, device="cuda", max_batch=256, max_seqs=2, ctx=256)
    c = Runner(path, device="cpu", max_batch=256, max_seqs=2, ctx=256)
    assert g.w16 is not None
    g.w16.fill_(float("nan"))
    rng = np.random.default_rng(8)
    toks = [1] + [int(x) for x in rng.integers(3, 500, 199)]  # 400 pairs at top-2
    sg, sc = g.new_sequence(), c.new_sequence()
    C.reset_launch_counts()
    g.prefill(sg, toks)
    torch.cuda.synchronize()
    n = C.launch_counts()
    assert not torch.isnan(g.w16).all() and n["gemm_lib"] == 0 and n["dq_gemm"] >= 2 * g.cfg.n_layer, n
    c.prefill(sc, toks)
    V = g.cfg.n_vocab
    assert rel(g.logits[0, :V].cpu(), c.logits[0, :V]) < 3e-2


@pytest.mark.parametrize("name", ["tiny-llama", "tiny-mixtral", "tiny-gemma", "tiny-phi2"])
def test_prefill_library_path_vs_torch(tiny_models, name, monkeypatch):
    """The hipBLASLt prefill path (gemm.hip gemm_lib; for Mixtral per-expert GEMMs over the sorted
    rows with the GLU / routing-weighted scatter epilogues, moe_gemm_lib) forced from 16 rows: logits
    must match the torch twin, and the dequantised-weight scratch must have been used (per-call
    dequantisation: no resident fp16 copies)."""
    C = native()
    old = C.gemm_lib_min_m()
    C.set_gemm_lib_min_m(16)
    try:
        path = tiny_models[name]
        # max_batch 128: 70 prompt rows run on the 128-row bucket's plan padded (rows 70..127 unused)
        g = Runner(path, device="cuda", max_batch=128, max_seqs=2, ctx=160)
        c = Runner(path, device="cpu", max_batch=64, max_seqs=2, ctx=160)
        assert g.w16 is not None
        g.w16.fill_(float("nan"))
        rng = np.random.default_rng(2)
        toks = [1] + [int(x) for x in rng.integers(3, 500, 69)]
        sg, sc = g.new_sequence(), c.new_sequence()
        g.prefill(sg, toks)
        c.prefill(sc, toks)
        torch.cuda.synchronize()
        assert not torch.isnan(g.w16).all()  # some matrix went through the library path
        V = g.cfg.n_vocab
        assert rel(g.logits[0, :V].cpu(), c.logits[0, :V]) < 3e-2
        g.prefill(sg, [5])
        c.prefill(sc, [5])
        assert rel(g.logits[0, :V].cpu(), c.logits[0, :V]) < 3e-2
    finally:
        C.set_gemm_lib_min_m(old)


@pytest.mark.parametrize("name", ["tiny-llama", "tiny-phi2"])
def test_deferred_split_merge_decode(tmp_path, monkeypatch, name):
    """B == 1 decode at lengths in every split bucket: the deferred merge (attention leaves S partial
    slabs, the O GEMV prologue merges them) must match the in-launch merge and the torch twin."""
    from ollama_operator_amd.gguf.constants import FileType
    from ollama_operator_amd.models.config import preset
    from ollama_operator_amd.models.random_init import write_random_gguf
    path = str(tmp_path / "long.gguf")
    write_random_gguf(path, preset(name, ctx_len=2048), FileType.MOSTLY_Q4_K_M, seed=5, quantize_from_float=True)
    g = Runner(path, device="cuda", max_batch=64, max_seqs=1, ctx=1100)
    monkeypatch.setenv("OMX_DEFER_MERGE", "0")
    g0 = Runner(path, device="cuda", max_batch=64, max_seqs=1, ctx=1100, weights=g.w)
    assert g._defer_ok and not g0._defer_ok
    c = Runner(path, device="cpu", max_batch=64, max_seqs=1, ctx=1100)
    rng = np.random.default_rng(3)
    V = g.cfg.n_vocab
    seen = set()
    for L in (100, 200, 400, 900, 1050):
        toks = [1] + [int(x) for x in rng.integers(3, 500, L - 1)]
        seen.add(g.decode_splits(L + 1))
        outs = []
        for r in (g, g0, c):
            sid = r.new_sequence()
            r.prefill(sid, toks)
            if r.is_gpu:
                r.d_tokens[0] = 77
                r.decode_step(sid, L)
                torch.cuda.synchronize()
                outs.append(r.logits[0, :V].float().cpu().clone())
            else:
                r.prefill(sid, [77])
                outs.append(r.logits[0, :V].clone())
            r.free_sequence(sid)
        assert rel(outs[0], outs[1]) < 2e-3, L
        assert rel(outs[0], outs[2]) < 3e-2, L
    assert seen == {1, 2, 4, 8}  # 1050 keys: 8 deferred splits of 132 (OMX_DEFER_LONG, default on)
    monkeypatch.setenv("OMX_DEFER_S4_MAX", "3072")
    monkeypatch.delenv("OMX_DEFER_MERGE")
    g4 = Runner(path, device="cuda", max_batch=64, max_seqs=1, ctx=1100, weights=g.w)
    # the opt-in 4-split bucket: up to 768 keys per split between 1024 and 3072 keys, 8 splits beyond
    assert [g4.decode_splits(n) for n in (1000, 1050, 2049, 3072, 3073, 4096)] == [8, 4, 4, 4, 8, 8]
    sid = g4.new_sequence()
    toks = [1] + [int(x) for x in rng.integers(3, 500, 1049)]
    g4.prefill(sid, toks)
    g4.d_tokens[0] = 77
    g4.decode_step(sid, 1050)
    torch.cuda.synchronize()
    out4 = g4.logits[0, :V].float().cpu().clone()
    sc = c.new_sequence()
    c.prefill(sc, toks + [77])
    assert rel(out4, c.logits[0, :V]) < 3e-2


@pytest.mark.parametrize("name", ["tiny-llama", "tiny-mixtral", "tiny-phi2", "tiny-gemma"])
def test_batched_decode_matches_single(tiny_models, name):
    """Continuous batching step (B rows of different sequences/lengths, batched GEMV + multi-sequence
    paged attention) against each sequence's own B == 1 decode step."""
    path = tiny_models[name]
    g = Runner(path, device="cuda", max_batch=32, max_seqs=8, ctx=256)
    rng = np.random.default_rng(11)
    prompts = [[1] + [int(x) for x in rng.integers(3, 500, n)] for n in (5, 40, 17, 90)]
    sids = []
    for p in prompts:
        sid = g.new_sequence()
        g.prefill(sid, p)
        sids.append(sid)
    V = g.cfg.n_vocab
    nxt = [7, 8, 9, 10]
    g.set_tokens(nxt)
    g.decode_batch(sids, [len(p) for p in prompts])
    torch.cuda.synchronize()
    batched = g.logits[:4, :V].float().cpu().clone()
    for b, (sid, p) in enumerate(zip(sids, prompts)):
        g.set_tokens([nxt[b]])
        g.decode_batch([sid], [len(p)])  # rewrites the same KV position: same input token
        torch.cuda.synchronize()
        assert rel(batched[b], g.logits[0, :V].float().cpu()) < 3e-2, b


@pytest.mark.parametrize("mfma", [0, 1])
def test_scheduler_concurrent_gpu(tiny_models, mfma):
    """mfma = 0: the int8 GEMV serves every batch size with the same per-row arithmetic, so a seeded
    request gives the same tokens whatever rows it shares steps with (batch invariance). mfma = 1: steps
    of 3..16 rows run on the matrix cores (fp16 activations, a different summation order from the
    1-2 row int8 GEMV), so a request's stream may depend on the batch composition -- as in llama.cpp's
    batched decode; the streams must still be valid and of the requested lengths."""
    import threading
    from ollama_operator_amd.engine.scheduler import BatchScheduler
    from ollama_operator_amd.ops import native
    native().set_mb_enable(mfma)
    try:
        _scheduler_concurrent(tiny_models, invariant=not mfma)
    finally:
        native().set_mb_enable(1)


def _scheduler_concurrent(tiny_models, invariant):
    import threading
    from ollama_operator_amd.engine.scheduler import BatchScheduler
    g = Runner(tiny_models["tiny-llama"], device="cuda", max_batch=32, max_seqs=8, ctx=256)
    g.warmup()
    g.capture_batch_graphs(4)
    sch = BatchScheduler(g, max_parallel=4)
    out = [None] * 6
    lens = [30, 12, 25, 40, 5, 18]

    def work(i):
        out[i] = list(sch.submit([1, 10 + i, 20 + i], SamplingOptions(temperature=0.7, seed=i), lens[i]))

    def run_all():
        th = [threading.Thread(target=work, args=(i,)) for i in range(6)]
        for t in th:
            t.start()
        for t in th:
            t.join(60)
        return [list(o) for o in out]

    first = run_all()
    again = run_all()  # same requests, different row composition/timing: seeded sampling is per row
    sch.close()
    assert [len(o) for o in first] == lens
    assert sch.max_batch_seen >= 2
    assert all(0 <= t < g.cfg.n_vocab for o in first for t in o)
    assert [len(o) for o in again] == lens
    if not invariant:
        return
    assert again == first
    # parity with solo generation (B == 1 path): same seeded stream; the batched GEMV sums in a
    # different order, so allow a late divergence on a near-tie but require the opening tokens agree
    s = Runner(tiny_models["tiny-llama"], device="cuda", max_batch=32, max_seqs=2, ctx=256)
    for i in range(6):
        sid = s.new_sequence()
        solo = list(s.generate(sid, [1, 10 + i, 20 + i], SamplingOptions(temperature=0.7, seed=i), max_tokens=lens[i]))
        s.free_sequence(sid)
        k = min(4, lens[i])
        assert solo[:k] == first[i][:k], i
        assert sum(a == b for a, b in zip(solo, first[i])) >= lens[i] // 2, i


def test_interleaved_admission_gpu(tiny_models):
    """A burst admitted while a row decodes (scheduler chunk = 16): each chunk's forward carries the
    running row's decode token (mixed prefill + decode segments through the MFMA flash / split decode
    attention). Streams complete at their lengths, the running row kept stepping during the admission,
    and each burst request's first token matches its solo prefill."""
    from ollama_operator_amd.engine.scheduler import BatchScheduler
    g = Runner(tiny_models["tiny-llama"], device="cuda", max_batch=32, max_seqs=8, ctx=256)
    g.warmup()
    g.capture_batch_graphs(4)
    sch = BatchScheduler(g, max_parallel=4, chunk=16)
    p1, p2 = [1] + list(range(40, 80)), [1] + list(range(100, 133))
    g0 = sch.submit([1, 5, 9], SamplingOptions(temperature=0.7, seed=1), 40)
    head = [next(g0), next(g0)]
    with sch.cv:
        g1 = sch.submit(p1, SamplingOptions(temperature=0), 10)
        g2 = sch.submit(p2, SamplingOptions(temperature=0), 10)
    out = [head + list(g0), list(g1), list(g2)]
    sch.close()
    assert [len(o) for o in out] == [40, 10, 10]
    assert all(0 <= t < g.cfg.n_vocab for o in out for t in o)
    assert sch.interleaved_chunks >= (40 + 33) // 16
    s = Runner(tiny_models["tiny-llama"], device="cuda", max_batch=64, max_seqs=2, ctx=256)
    for p, o in ((p1, out[1]), (p2, out[2])):
        sid = s.new_sequence()
        solo = list(s.generate(sid, p, SamplingOptions(temperature=0), max_tokens=2))
        s.free_sequence(sid)
        assert solo[0] == o[0]


@pytest.mark.parametrize("name", ["tiny-llama", "tiny-mixtral"])
def test_admit_many_gpu_matches_sequential(tiny_models, name):
    """Queued requests prefilled together (Runner.admit_many: one forward over every prompt row,
    multi-sequence paged attention) against each request's own prefill."""
    g = Runner(tiny_models[name], device="cuda", max_batch=64, max_seqs=6, ctx=128)
    V = g.cfg.n_vocab
    rng = np.random.default_rng(6)
    prompts = [[1] + [int(x) for x in rng.integers(3, 500, n)] for n in (9, 23, 4)]
    o = SamplingOptions(temperature=0)
    ref = []
    for p in prompts:
        sid = g.new_sequence()
        g.admit(sid, 0, p, o, p, 0)
        torch.cuda.synchronize()
        ref.append(g.logits[0, :V].float().cpu().clone())
        g.free_sequence(sid)
    sids = [g.new_sequence() for _ in prompts]
    g.admit_many([(sid, 0, p, o, p, 0) for sid, p in zip(sids, prompts)])
    torch.cuda.synchronize()
    for i, lg in enumerate(ref):
        assert rel(g.logits[i, :V].float().cpu(), lg) < 2e-2, i


@pytest.mark.parametrize("group", [2, 4])
def test_grouped_decode_graph_matches_single_steps(tiny_models, monkeypatch, group):
    """generate() replays `group` decode steps per graph (OMX_DECODE_GROUP): the same tokens as one step
    per replay, for a generation length that is not a multiple of the group and crosses KV pages."""
    path = tiny_models["tiny-llama"]
    o = SamplingOptions(temperature=0.7, top_k=20, top_p=0.95, seed=7)
    monkeypatch.setenv("OMX_DECODE_GROUP", "1")
    a = Runner(path, device="cuda", max_batch=8, max_seqs=2, ctx=128)
    monkeypatch.setenv("OMX_DECODE_GROUP", str(group))
    b = Runner(path, device="cuda", max_batch=8, max_seqs=2, ctx=128, weights=a.w)
    b.warmup()
    assert b.decode_group == group
    prompt = [1, 9, 8, 7, 6, 5]
    ta = list(a.generate(a.new_sequence(), prompt, o, max_tokens=37))
    tb = list(b.generate(b.new_sequence(), prompt, o, max_tokens=37))
    assert ta == tb and len(ta) == 37
    assert any(k[2] == group for k in b.graphs), "no grouped graph was replayed"


@pytest.mark.parametrize("name", ["tiny-llama", "tiny-llama-q40", "tiny-llama-q8"])
def test_ffn_down_k_padding(tiny_models, monkeypatch, name):
    """ffn_down stored with a padded K (weights.py ffn_pad, zero super-blocks; the GLU image and the fp32
    / fp16 activation rows carry zeros there): prefill logits and greedy decode match the unpadded
    model on the int8 chain, the fp32 GEMV and the prefill GEMM paths."""
    path = tiny_models[name]
    monkeypatch.setenv("OMX_FFN_PAD", "0")
    a = Runner(path, device="cuda", max_batch=64, max_seqs=2, ctx=128)
    monkeypatch.setenv("OMX_FFN_PAD", "force")
    b = Runner(path, device="cuda", max_batch=64, max_seqs=2, ctx=128)
    assert a.w.ffn_pad == 0 and b.w.ffn_pad > 0
    assert b.w.layers[0]["wdown"].K == a.w.layers[0]["wdown"].K + b.w.ffn_pad
    V = a.cfg.n_vocab
    toks = [1] + list(range(3, 40))  # 39 rows: the prefill GEMM path
    for r in (a, b):
        r._sid = r.new_sequence()
        r.prefill(r._sid, toks)
    assert rel(b.logits[0, :V].cpu(), a.logits[0, :V].cpu()) < 1e-3
    o = SamplingOptions(temperature=0)
    ta = list(a.generate(a.new_sequence(), [1, 5, 6, 7], o, max_tokens=12))
    tb = list(b.generate(b.new_sequence(), [1, 5, 6, 7], o, max_tokens=12))
    assert ta == tb


@pytest.mark.parametrize("ring", [0, 1])
@pytest.mark.parametrize("name", ["tiny-llama", "tiny-llama-q40", "tiny-llama-q8", "tiny-llama-q5km", "tiny-phi2"])
def test_prefill_dq_ring_and_glds_kernels(tiny_models, name, ring):
    """Both editions of the hand-written prefill GEMM (gemm_dq_impl.h: the register-ring default and the
    glds kernel, set_dq_ring) over 240 prompt rows (128- and 256-row tiles with a partial last tile,
    split-K for the narrow shapes): logits match the torch twin and every dense projection ran on the dq
    kernel."""
    C = native()
    C.set_dq_ring(ring)
    try:
        path = tiny_models[name]
        g = Runner(path, device="cuda", max_batch=256, max_seqs=2, ctx=256)
        c = Runner(path, device="cpu", max_batch=256, max_seqs=2, ctx=256)
        rng = np.random.default_rng(11)
        toks = [1] + [int(x) for x in rng.integers(3, 500, 239)]
        sg, sc = g.new_sequence(), c.new_sequence()
        C.reset_launch_counts()
        g.prefill(sg, toks)
        n = C.launch_counts()
        assert n["dq_gemm"] >= 2 * g.cfg.n_layer and n["gemm_lib"] == 0, n
        c.prefill(sc, toks)
        V = g.cfg.n_vocab
        assert rel(g.logits[0, :V].cpu(), c.logits[0, :V]) < 3e-2
    finally:
        C.set_dq_ring(1)
