"""CPU: the runner (repacked weights + paged KV + torch executor) against the fp32 GGUF reference.
Covers the loader's row transforms (QKV fusion, NEOX pairing, gate/up interleave, MoE stacking)."""
import numpy as np
import pytest
import torch

from ollama_operator_amd.engine.runner import Runner
from ollama_operator_amd.engine.sampling import SamplingOptions
from ollama_operator_amd.gguf import read_gguf
from ollama_operator_amd.models.reference import KVCacheRef, ReferenceModel

MODELS = ["tiny-llama", "tiny-mixtral", "tiny-phi2", "tiny-llama-q8", "tiny-llama-q40", "tiny-llama-q5km", "tiny-orca"]


@pytest.mark.parametrize("name", MODELS)
def test_prefill_logits_match_reference(tiny_models, name):
    path = tiny_models[name]
    ref = ReferenceModel(read_gguf(path))
    toks = [1, 17, 42, 99, 7, 300, 12]
    want = ref.forward(torch.tensor(toks), KVCacheRef(ref.cfg, 64), start=0)[-1]
    r = Runner(path, device="cpu", max_batch=4, max_seqs=2, ctx=64)
    sid = r.new_sequence()
    r.prefill(sid, toks)  # 7 tokens in chunks of 4 -> exercises multi-chunk causal prefill
    got = r.logits[0, :ref.cfg.n_vocab]
    np.testing.assert_allclose(got.numpy(), want.numpy(), rtol=2e-3, atol=2e-3)


@pytest.mark.parametrize("name", ["tiny-llama", "tiny-phi2", "tiny-mixtral"])
def test_greedy_generation_matches_reference(tiny_models, name):
    path = tiny_models[name]
    ref = ReferenceModel(read_gguf(path))
    prompt = [1, 5, 9, 33]
    cache = KVCacheRef(ref.cfg, 64)
    lg = ref.forward(torch.tensor(prompt), cache)[-1]
    want = []
    for _ in range(6):
        t = int(lg.argmax())
        want.append(t)
        lg = ref.forward(torch.tensor([t]), cache)[-1]
    r = Runner(path, device="cpu", max_batch=4, max_seqs=2, ctx=64)
    sid = r.new_sequence()
    got = list(r.generate(sid, prompt, SamplingOptions(temperature=0, repeat_penalty=1.0), max_tokens=6))
    assert got == want
    # second turn extends the first: prefix reused, result identical to a fresh run
    prompt2 = prompt + got + [11, 12]
    got2 = list(r.generate(sid, prompt2, SamplingOptions(temperature=0, repeat_penalty=1.0), max_tokens=3))
    r2 = Runner(path, device="cpu", max_batch=4, max_seqs=2, ctx=64, weights=r.w)
    sid2 = r2.new_sequence()
    fresh = list(r2.generate(sid2, prompt2, SamplingOptions(temperature=0, repeat_penalty=1.0), max_tokens=3))
    assert got2 == fresh


def test_seeded_sampling_reproducible(tiny_models):
    r = Runner(tiny_models["tiny-llama"], device="cpu", max_batch=4, max_seqs=2, ctx=64)
    o = SamplingOptions(temperature=0.9, top_k=40, top_p=0.9, seed=1234)
    a = list(r.generate(r.new_sequence(), [1, 2, 3], o, max_tokens=8))
    b = list(r.generate(r.new_sequence(), [1, 2, 3], o, max_tokens=8))
    assert a == b


def test_admit_many_matches_sequential_admits(tiny_models):
    """Several requests prefilled in one forward (independent rows, multi-sequence paged attention)
    give each the logits its own prefill gives."""
    import numpy as np
    from ollama_operator_amd.engine.runner import Runner
    from ollama_operator_amd.engine.sampling import SamplingOptions
    r = Runner(tiny_models["tiny-llama"], device="cpu", max_batch=64, max_seqs=6, ctx=128)
    V = r.cfg.n_vocab
    rng = np.random.default_rng(4)
    prompts = [[1] + [int(x) for x in rng.integers(3, 500, n)] for n in (9, 23, 4)]
    o = SamplingOptions(temperature=0)
    ref = []
    for p in prompts:
        sid = r.new_sequence()
        r.admit(sid, 0, p, o, p, 0)
        ref.append((r.logits[0, :V].clone(), int(r.s_out[0])))
        r.free_sequence(sid)
    sids = [r.new_sequence() for _ in prompts]
    firsts = r.admit_many([(sid, 0, p, o, p, 0) for sid, p in zip(sids, prompts)])
    for i, (lg, tok) in enumerate(ref):
        assert float((r.logits[i, :V] - lg).norm() / lg.norm()) < 1e-4
        assert firsts[i] == tok
    for sid, p in zip(sids, prompts):
        assert r.kv.seqs[sid].tokens == p


def test_unsupported_head_dim_fails_at_load(tmp_path):
    """A head dim no attention kernel serves is refused when the model loads (it used to load and then
    skip attention on the GPU): 132 is past 128 and far below 256."""
    from ollama_operator_amd.gguf.constants import FileType
    from ollama_operator_amd.models.config import UnsupportedArchitecture, preset
    from ollama_operator_amd.models.random_init import write_random_gguf
    p = str(tmp_path / "bad.gguf")
    write_random_gguf(p, preset("tiny-llama", n_embd=264, n_head=2, n_head_kv=2, n_rot=132, n_embd_head=132),
                      FileType.MOSTLY_Q8_0, seed=1)
    with pytest.raises(UnsupportedArchitecture):
        Runner(p, device="cpu", max_batch=4, max_seqs=1, ctx=32)


def test_kv_cache_type_env(tiny_models, monkeypatch):
    """OMX_KV_CACHE_TYPE / OLLAMA_KV_CACHE_TYPE select the GPU KV element type (fp8 for the 8-bit settings,
    f16 otherwise); the CPU backends always keep fp16 rows."""
    from ollama_operator_amd.engine.runner import kv_cache_type
    for env, val, want in (("OMX_KV_CACHE_TYPE", "fp8", "fp8"), ("OLLAMA_KV_CACHE_TYPE", "q8_0", "fp8"),
                           ("OLLAMA_KV_CACHE_TYPE", "q4_0", "f16"), ("OLLAMA_KV_CACHE_TYPE", "F16", "f16")):
        monkeypatch.delenv("OMX_KV_CACHE_TYPE", raising=False)
        monkeypatch.delenv("OLLAMA_KV_CACHE_TYPE", raising=False)
        monkeypatch.setenv(env, val)
        assert kv_cache_type() == want, (env, val)
    monkeypatch.setenv("OMX_KV_CACHE_TYPE", "fp8")
    r = Runner(tiny_models["tiny-llama"], device="cpu", max_batch=8, max_seqs=1, ctx=64)
    assert not r.kv8 and r.kc[0].dtype == torch.float16


@pytest.mark.parametrize("backend", ["torch", "native"])
def test_close_releases_runner_after_gc_freeze(tiny_models, backend):
    """warmup() freezes the objects alive after load (gc.freeze), and Runner <->
    NativeExec point at each other; close() must break that cycle so the unloaded model's buffers go
    (the server's unload path: ModelManager._unload -> Runner.close)."""
    import gc
    import weakref
    from ollama_operator_amd.ops.cpu import cpu_module
    if backend == "native" and cpu_module() is None:
        pytest.skip("native CPU backend not built")
    r = Runner(tiny_models["tiny-llama"], device="cpu", max_batch=4, max_seqs=2, ctx=64, cpu_backend=backend)
    sid = r.new_sequence()
    r.prefill(sid, [1, 2, 3])
    ref, kc = weakref.ref(r), weakref.ref(r.kc[0])
    gc.collect()
    gc.freeze()
    try:
        r.close()
        assert r.exe is None and r.kc is None
        del r
        gc.collect()
        assert ref() is None, "runner still alive after close()"
        assert kc() is None, "KV cache still alive after close()"
    finally:
        gc.unfreeze()
