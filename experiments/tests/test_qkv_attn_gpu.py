"""The fused batch-1 QKV + attention launch (csrc/kernels/qkv_attn.hip: int8-chain QKV tiles, the last
block of each KV group runs the group's attention and writes O's int8 image) against the fp32 torch
twin, teacher-forced through the decode graphs of the split buckets it covers (S = 1 / 2 / 4 x 128
keys) and past them (the split flash-decode fallback), with the fused launch asserted to have run."""
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
@pytest.mark.parametrize("plen,maxs", [(40, 4), (200, 4), (400, 4), (200, 1)])
def test_qkv_attn_matches_torch(tmp_path, monkeypatch, name, ft, plen, maxs):
    """maxs = 1: a 200-token context (2 splits) is past the fused bound -> the split flash-decode path"""
    monkeypatch.setenv("OMX_QKV_ATTN_MAXS", str(maxs))
    p = str(tmp_path / "m.gguf")
    write_random_gguf(p, preset(name), ft, seed=6, quantize_from_float=True)
    g = Runner(p, device="cuda:0", max_batch=16, max_seqs=1, ctx=512)
    assert g.exe.exe.x8_on == 1 and g.qkv_attn_maxs == maxs  # opt-in (OMX_QKV_ATTN_MAXS, default 0)
    c = Runner(p, device="cpu", max_batch=16, max_seqs=1, ctx=512, cpu_backend="torch")
    prompt = [1] + [(7 * i + 3) % 500 for i in range(1, plen)]
    sg, sc = g.new_sequence(), c.new_sequence()
    g.prefill(sg, prompt)
    c.prefill(sc, prompt)
    V = g.cfg.n_vocab
    C = native()
    for i, t in enumerate([8, 9, 10, 11]):
        g.set_tokens([t])
        eager = i == 3  # one eager step: the launch counter sees this step's own enqueues
        g.use_graphs = not eager
        C.reset_launch_counts()
        g.decode_step(sg)
        torch.cuda.synchronize()
        if eager:
            n = C.launch_counts()
            fused = g.decode_splits(plen + i + 1) <= maxs
            assert n["qkv_attn"] == (g.cfg.n_layer - 1 if fused else 0), n
            assert n["attn_decode"] == (1 if fused else g.cfg.n_layer), n
        g.kv.seqs[sg].tokens.append(t)
        c.prefill(sc, [t])
        assert rel(g.logits[0, :V].cpu(), c.logits[0, :V]) < 3e-2
    assert g.x8_error() == 0
    # the decode graph of this bucket was captured with the fused launch (layers 1..; layer 0 reads the
    # embedding rows through the fp32 prologue)
    if g.decode_splits(plen + 1) <= maxs:
        assert g.exe.exe.n_qkv_attn >= 2 * (g.cfg.n_layer - 1)
