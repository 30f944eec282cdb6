"""fp8 (OCP e4m3fn) KV cache (OMX_KV_CACHE_TYPE=fp8): the QKV epilogues store K / V as one byte per
element and the decode / MFMA-prefill attention kernels widen them on load
(csrc/kernels/attention.hip load_krow8 / the prefill staging). Checked against the fp32 torch twin (fp16
KV) and the fp16-KV GPU run of the same model: prefill through the MFMA flash path (>= 16 rows), decode
at lengths that cover the single-block, deferred-split and in-launch-merge attention."""
import pytest
import torch

from ollama_operator_amd.engine.runner import Runner
from ollama_operator_amd.gguf.constants import FileType
from ollama_operator_amd.models.config import preset
from ollama_operator_amd.models.random_init import write_random_gguf
from ollama_operator_amd.ops import native

pytestmark = pytest.mark.gpu


def rel(a, b):
    return float((a - b).norm() / (b.norm() + 1e-12))


@pytest.mark.parametrize("name", ["tiny-llama-d128", "tiny-llama-d128-gqa", "tiny-gemma", "tiny-orca", "tiny-llama"])
@pytest.mark.parametrize("plen,defer", [(40, "1"), (700, "1"), (700, "0")])
def test_fp8_kv_matches_torch(tmp_path, monkeypatch, name, plen, defer):
    """defer = 0: long decode through the in-launch split merge instead of the O-prologue merge"""
    monkeypatch.setenv("OMX_DEFER_MERGE", defer)
    ft = FileType.MOSTLY_Q4_0 if name == "tiny-orca" else FileType.MOSTLY_Q4_K_M
    p = str(tmp_path / "m.gguf")
    write_random_gguf(p, preset(name, ctx_len=1024), ft, seed=11, quantize_from_float=True)
    monkeypatch.setenv("OMX_KV_CACHE_TYPE", "fp8")
    g8 = Runner(p, device="cuda:0", max_batch=256, max_seqs=1, ctx=1024)
    assert g8.kv8 and g8.kc[0].dtype == torch.uint8
    monkeypatch.setenv("OMX_KV_CACHE_TYPE", "f16")
    g16 = Runner(p, device="cuda:0", max_batch=256, max_seqs=1, ctx=1024, weights=g8.w)
    assert not g16.kv8 and g16.kc[0].dtype == torch.float16
    c = Runner(p, device="cpu", max_batch=256, max_seqs=1, ctx=1024, cpu_backend="torch")
    prompt = [1] + [(7 * i + 5) % 500 for i in range(1, plen)]
    V = c.cfg.n_vocab
    sids = {}
    C = native()
    for r in (g8, g16, c):
        sids[id(r)] = r.new_sequence()
        if r.is_gpu:
            C.reset_launch_counts()
        r.prefill(sids[id(r)], prompt)
        if r.is_gpu:
            torch.cuda.synchronize()
            assert C.launch_counts()["attn_prefill"] >= r.cfg.n_layer  # the MFMA flash path ran
    assert rel(g8.logits[0, :V].float().cpu(), c.logits[0, :V]) < 8e-2
    for t in (8, 9, 10):
        for r in (g8, g16, c):
            if r.is_gpu:
                r.set_tokens([t])
                r.decode_step(sids[id(r)])
                torch.cuda.synchronize()
                r.kv.seqs[sids[id(r)]].tokens.append(t)
            else:
                r.prefill(sids[id(r)], [t])
        ref = c.logits[0, :V]
        e8, e16 = rel(g8.logits[0, :V].float().cpu(), ref), rel(g16.logits[0, :V].float().cpu(), ref)
        assert e16 < 3e-2, e16
        assert e8 < 8e-2, (e8, e16)
