"""The fused batch-1 attention + O projection launch (csrc/kernels/attn_o.hip: split attention blocks
whose last split per KV group merges and writes O's int8 image; O blocks that request their weights
before waiting on the hand-off) against the fp32 torch twin, teacher-forced through the decode graphs,
with the launch asserted to have run for every layer and no hand-off timeout."""
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


@pytest.mark.parametrize("name,ft", [("tiny-llama-d128", FileType.MOSTLY_Q4_K_M),
                                     ("tiny-llama-d128", FileType.MOSTLY_Q4_0),
                                     ("tiny-llama-d128-gqa", FileType.MOSTLY_Q4_K_M)])
@pytest.mark.parametrize("plen,kps", [(40, 128), (200, 128), (400, 128), (300, 16)])
def test_attn_o_matches_torch(tmp_path, monkeypatch, name, ft, plen, kps):
    """kps = 16: up to 8 key splits per group at these lengths (the split merge inside the launch)"""
    monkeypatch.setenv("OMX_ATTN_O", "1")  # opt-in (measured slower than the split launches)
    monkeypatch.setenv("OMX_ATTN_O_KPS", str(kps))
    p = str(tmp_path / "m.gguf")
    write_random_gguf(p, preset(name), ft, seed=7, quantize_from_float=True)
    g = Runner(p, device="cuda:0", max_batch=16, max_seqs=1, ctx=512)
    assert g.exe.exe.x8_on == 1
    c = Runner(p, device="cpu", max_batch=16, max_seqs=1, ctx=512, cpu_backend="torch")
    prompt = [1] + [(5 * i + 11) % 500 for i in range(1, plen)]
    sg, sc = g.new_sequence(), c.new_sequence()
    g.prefill(sg, prompt)
    c.prefill(sc, prompt)
    V = g.cfg.n_vocab
    C = native()
    for i, t in enumerate([8, 9, 10, 11]):
        g.set_tokens([t])
        eager = i == 3  # one eager step: the launch counters see this step's own enqueues
        g.use_graphs = not eager
        C.reset_launch_counts()
        g.decode_step(sg)
        torch.cuda.synchronize()
        if eager:
            n = C.launch_counts()
            assert n["attn_o"] == g.cfg.n_layer and n["attn_decode"] == 0, n
        g.kv.seqs[sg].tokens.append(t)
        c.prefill(sc, [t])
        assert rel(g.logits[0, :V].cpu(), c.logits[0, :V]) < 3e-2
    assert g.x8_error() == 0
    assert g.exe.exe.n_attn_o >= g.cfg.n_layer


def test_attn_o_off_matches(tmp_path, monkeypatch):
    """OMX_ATTN_O=0 (the default): the separate attention + O launches serve the same model"""
    monkeypatch.setenv("OMX_ATTN_O", "0")
    p = str(tmp_path / "m.gguf")
    write_random_gguf(p, preset("tiny-llama-d128"), FileType.MOSTLY_Q4_K_M, seed=7, quantize_from_float=True)
    g = Runner(p, device="cuda:0", max_batch=16, max_seqs=1, ctx=512)
    c = Runner(p, device="cpu", max_batch=16, max_seqs=1, ctx=512, cpu_backend="torch")
    prompt = [1] + [(5 * i + 11) % 500 for i in range(1, 150)]
    sg, sc = g.new_sequence(), c.new_sequence()
    g.prefill(sg, prompt)
    c.prefill(sc, prompt)
    g.set_tokens([8])
    g.decode_step(sg)
    torch.cuda.synchronize()
    c.prefill(sc, [8])
    assert g.exe.exe.n_attn_o == 0
    assert rel(g.logits[0, :g.cfg.n_vocab].cpu(), c.logits[0, :g.cfg.n_vocab]) < 3e-2
