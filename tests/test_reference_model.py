import numpy as np
import torch

from ollama_operator_amd.gguf import read_gguf
from ollama_operator_amd.models.config import ModelConfig
from ollama_operator_amd.models.reference import KVCacheRef, ReferenceModel


def test_config_from_gguf(tiny_models):
    g = read_gguf(tiny_models["tiny-llama"])
    cfg = ModelConfig.from_gguf_metadata(g.metadata)
    assert (cfg.n_embd, cfg.n_layer, cfg.n_head, cfg.n_head_kv) == (256, 2, 4, 2)
    assert cfg.head_dim == 64
    g2 = read_gguf(tiny_models["tiny-mixtral"])
    assert ModelConfig.from_gguf_metadata(g2.metadata).n_expert == 4
    g3 = read_gguf(tiny_models["tiny-phi2"])
    assert ModelConfig.from_gguf_metadata(g3.metadata).arch == "phi2"


def _check_incremental(path):
    g = read_gguf(path)
    m = ReferenceModel(g)
    toks = torch.tensor([1, 5, 9, 33, 2, 7, 100, 4])
    full = m.forward(toks, KVCacheRef(m.cfg, 64), start=0)
    c = KVCacheRef(m.cfg, 64)
    part = [m.forward(toks[:5], c)]
    for t in toks[5:]:
        part.append(m.forward(t[None], c))
    inc = torch.cat(part)
    assert torch.isfinite(full).all()
    np.testing.assert_allclose(inc.numpy(), full.numpy(), rtol=1e-4, atol=1e-4)
    return full


def test_reference_llama_incremental_matches_full(tiny_models):
    _check_incremental(tiny_models["tiny-llama"])


def test_reference_mixtral_incremental_matches_full(tiny_models):
    _check_incremental(tiny_models["tiny-mixtral"])


def test_reference_phi2_incremental_matches_full(tiny_models):
    _check_incremental(tiny_models["tiny-phi2"])


def test_unknown_architecture_fails_loudly(tmp_path):
    """An architecture the engine does not implement must raise at load, never run as llama."""
    import pytest as _pt

    from ollama_operator_amd.gguf.constants import FileType
    from ollama_operator_amd.gguf.reader import read_gguf
    from ollama_operator_amd.models.config import ModelConfig, UnsupportedArchitecture, preset
    from ollama_operator_amd.models.random_init import write_random_gguf
    path = str(tmp_path / "t.gguf")
    write_random_gguf(path, preset("tiny-llama"), FileType.MOSTLY_Q8_0, seed=0)
    md = dict(read_gguf(path).metadata)
    md2 = {k.replace("llama.", "starcoder2."): v for k, v in md.items()}
    md2["general.architecture"] = "starcoder2"
    with _pt.raises(UnsupportedArchitecture, match="starcoder2"):
        ModelConfig.from_gguf_metadata(md2)
    del md["general.architecture"]
    with _pt.raises(UnsupportedArchitecture):
        ModelConfig.from_gguf_metadata(md)


def test_gemma_config_and_tensors(tmp_path):
    """Gemma (reference README.md:58-59): head dim from attention.key_length (256 != E / H), NEOX
    RoPE, GeGLU, sqrt(E) embedding scale, tied output (no output.weight)."""
    import math

    from ollama_operator_amd.gguf.constants import FileType
    from ollama_operator_amd.gguf.reader import read_gguf
    from ollama_operator_amd.models.config import ROPE_NEOX, ModelConfig, preset
    from ollama_operator_amd.models.random_init import write_random_gguf
    path = str(tmp_path / "g.gguf")
    write_random_gguf(path, preset("tiny-gemma"), FileType.MOSTLY_Q4_K_M, seed=0)
    g = read_gguf(path)
    cfg = ModelConfig.from_gguf_metadata(g.metadata)
    assert cfg.arch == "gemma" and cfg.head_dim == 256 and cfg.n_embd_q == 512 and cfg.rope_mode == ROPE_NEOX
    assert cfg.gelu_glu and math.isclose(cfg.embed_scale, 16.0)
    assert "output.weight" not in g.tensors and "token_embd.weight" in g.tensors
    assert tuple(g.tensors["blk.0.attn_output.weight"].shape) == (512, 256)
    for name in ("gemma-2b", "gemma-7b"):
        c = preset(name)
        assert c.head_dim == 256 and c.n_vocab == 256000
