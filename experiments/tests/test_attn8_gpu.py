"""The fused batch-1 decode layer halves (csrc/kernels/attn8.hip: QKV + attention + O in one launch;
gemv8.hip ffn8_kernel: gate_up + down in one launch) against the fp32 torch twin, teacher-forced through
the decode graph, with the fused paths asserted to have run and no hand-off timeout."""
import pytest
import torch

from ollama_operator_amd.engine.runner import Runner
from ollama_operator_amd.gguf.constants import FileType
from ollama_operator_amd.models.config import preset
from ollama_operator_amd.models.random_init import write_random_gguf

pytestmark = pytest.mark.gpu


def rel(a, b):
    return float((a - b).norm() / (b.norm() + 1e-12))


@pytest.mark.parametrize("name,ft", [("tiny-llama-d128", FileType.MOSTLY_Q4_K_M),
                                     ("tiny-llama-d128", FileType.MOSTLY_Q4_0),
                                     ("tiny-llama-d128-gqa", FileType.MOSTLY_Q4_K_M)])
def test_fused_halves_match_torch(tmp_path, monkeypatch, name, ft):
    # opt-in (off by default: measured slower than the separate launches, profiles/r4_decode)
    monkeypatch.setenv("OMX_ATTN_FUSE", "1")
    monkeypatch.setenv("OMX_X8_FUSE", "1")
    p = str(tmp_path / "m.gguf")
    write_random_gguf(p, preset(name), ft, seed=5, quantize_from_float=True)
    g = Runner(p, device="cuda:0", max_batch=16, max_seqs=1, ctx=512)
    assert g.exe.exe.x8_on == 1
    c = Runner(p, device="cpu", max_batch=16, max_seqs=1, ctx=512, cpu_backend="torch")
    prompt = [1] + [(7 * i + 3) % 500 for i in range(1, 40)]
    sg, sc = g.new_sequence(), c.new_sequence()
    g.prefill(sg, prompt)
    c.prefill(sc, prompt)
    V = g.cfg.n_vocab
    a0, f0 = g.exe.exe.n_attn8, g.exe.exe.n_ffn8
    for t in [8, 9, 10, 11, 12, 13]:
        g.set_tokens([t])
        g.decode_step(sg)
        torch.cuda.synchronize()
        g.kv.seqs[sg].tokens.append(t)
        c.prefill(sc, [t])
        assert rel(g.logits[0, :V].cpu(), c.logits[0, :V]) < 3e-2
    assert g.x8_error() == 0
    # the decode graph was captured with the fused launches (layers 1.. for attention: layer 0 reads
    # the embedding through the fp32 prologue)
    assert g.exe.exe.n_attn8 > a0 or g.exe.exe.n_attn8 >= g.cfg.n_layer - 1
    assert g.exe.exe.n_ffn8 > f0 or g.exe.exe.n_ffn8 >= g.cfg.n_layer
