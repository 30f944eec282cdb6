"""LLaVA on the MI355X: CLIP encoder (fp16 on the GPU) against the fp64 oracle, and external embedding
rows through the native HIP engine (embed_rows_kernel ext path) -- exact-invariant check as on CPU."""
import numpy as np
import pytest
import torch

from test_llava import E_LLM, _png, tiny_clip  # noqa: F401  (fixture)

pytestmark = pytest.mark.gpu


def test_clip_encoder_gpu_matches_oracle(tiny_clip):  # noqa: F811
    from ollama_operator_amd.models.clip import ClipEncoder, preprocess, reference_encode
    enc = ClipEncoder(tiny_clip, "cuda")
    px = preprocess(_png(seed=4), enc.cfg)
    got = enc.encode_pixels(px).cpu().numpy()
    ref = reference_encode(tiny_clip, px)
    assert np.linalg.norm(got - ref) / np.linalg.norm(ref) < 2e-2


def test_ext_rows_native_gpu(tiny_models):
    from ollama_operator_amd.engine.runner import Runner
    from ollama_operator_amd.gguf import read_gguf
    from ollama_operator_amd.quant import dequantize
    r = Runner(tiny_models["tiny-llama"], device="cuda", max_batch=16, max_seqs=4, ctx=64, ext_rows=8)
    V = r.cfg.n_vocab
    prompt = [1, 17, 42, 99, 5, 230, 7, 11, 64, 3, 8, 21, 77, 300, 12, 14, 400, 2]  # >= GEMM_MIN_B rows
    r.prefill(r.new_sequence(), prompt)
    want = r.logits[0, :V].clone()
    g = read_gguf(tiny_models["tiny-llama"])
    t = g.tensors["token_embd.weight"]
    emb = dequantize(g.raw("token_embd.weight"), t.ggml_type, t.n_elements).reshape(t.torch_shape)
    g.close()
    r.set_ext([-7, -8], emb[[42, 300]] * r.cfg.embed_scale)
    p2 = list(prompt)
    p2[2], p2[13] = -7, -8
    r.prefill(r.new_sequence(), p2)
    torch.cuda.synchronize()
    assert torch.allclose(r.logits[0, :V], want, rtol=1e-4, atol=1e-4)
    toks = list(r.generate(r.new_sequence(), p2[:6], max_tokens=4))
    assert len(toks) == 4 and all(0 <= x < V for x in toks)


@pytest.mark.parametrize("gelu", [False, True])
def test_native_clip_tower_matches_oracle(tmp_path, gelu):
    """The CLIP tower on the engine's kernels (F16 MFMA GEMMs with fused LayerNorm / bias / GELU epilogues,
    RoPE-less QKV scatter, bidirectional flash attention) against the fp64 numpy oracle."""
    from ollama_operator_amd.models.clip import ClipEncoder, preprocess, reference_encode, write_random_clip_gguf
    p = str(tmp_path / "mmproj.gguf")
    write_random_clip_gguf(p, out_dim=E_LLM, image_size=168, patch_size=14, E=256, F_=512, n_layer=2, n_head=4,
                           seed=3, use_gelu=gelu)
    enc = ClipEncoder(p, "cuda")
    assert enc.native is not None and enc.cfg.n_patches == 144
    px = preprocess(_png(seed=5), enc.cfg)
    got = enc.encode_pixels(px).cpu().numpy()
    ref = reference_encode(p, px)
    assert got.shape == ref.shape
    assert np.linalg.norm(got - ref) / np.linalg.norm(ref) < 2e-2
    torch_path = enc.encode_pixels_torch(px).cpu().numpy()
    assert np.linalg.norm(got - torch_path) / np.linalg.norm(torch_path) < 2e-2


@pytest.mark.gpu
def test_native_anyres_matches_cpu(tmp_path):
    """LLaVA-1.6 any-resolution views through the native tower on the GPU vs the fp32 CPU encoder."""
    from ollama_operator_amd.models.clip import ClipEncoder, write_random_clip_gguf
    p = str(tmp_path / "mmproj16.gguf")
    write_random_clip_gguf(p, out_dim=E_LLM, image_size=168, patch_size=14, E=256, F_=512, n_layer=2, n_head=4,
                           seed=6, grid_pinpoints=[(168, 336), (336, 168), (336, 336)])
    gpu, cpu = ClipEncoder(p, "cuda"), ClipEncoder(p, "cpu")
    assert gpu.native is not None
    img = (np.random.default_rng(2).random((90, 160, 3)) * 255).astype(np.uint8)
    a, b = gpu.encode(img).cpu().numpy(), cpu.encode(img).numpy()
    assert a.shape == b.shape and a.shape[0] > 144
    assert np.linalg.norm(a - b) / np.linalg.norm(b) < 2e-2
