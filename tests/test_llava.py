"""LLaVA multimodal path (models/clip.py + external embedding rows in the engine + server `images`).

Parity unpinned: no real LLaVA mmproj GGUF exists here. The CLIP encoder is pinned to an independent
float64 numpy oracle of the same file, and the engine's external-row path is pinned by an exact
invariant: a row equal to token t's (dequantised, scaled) embedding must give the logits token t gives.
"""
import base64
import io

import numpy as np
import pytest
import torch

from ollama_operator_amd.models.clip import (ClipEncoder, VisionError, ImageIds, preprocess, preprocess_anyres,
                                             select_best_resolution,
                                             reference_encode, write_random_clip_gguf)

E_LLM = 256  # tiny-llama n_embd


def _png(w=40, h=24, seed=0) -> bytes:
    from PIL import Image
    a = (np.random.default_rng(seed).random((h, w, 3)) * 255).astype(np.uint8)
    buf = io.BytesIO()
    Image.fromarray(a).save(buf, format="PNG")
    return buf.getvalue()


@pytest.fixture(scope="module")
def tiny_clip(tmp_path_factory):
    p = str(tmp_path_factory.mktemp("clip") / "mmproj.gguf")
    write_random_clip_gguf(p, out_dim=E_LLM, image_size=28, patch_size=14, E=64, F_=128, n_layer=2, n_head=4, seed=1)
    return p


def test_clip_encoder_matches_fp64_oracle(tiny_clip):
    enc = ClipEncoder(tiny_clip, "cpu")
    assert enc.cfg.n_patches == 4 and enc.out_dim == E_LLM
    px = preprocess(_png(), enc.cfg)
    got = enc.encode_pixels(px).numpy()
    ref = reference_encode(tiny_clip, px)
    assert got.shape == (4, E_LLM)
    assert np.linalg.norm(got - ref) / np.linalg.norm(ref) < 1e-4


def test_clip_gelu_variant(tmp_path):
    p = str(tmp_path / "g.gguf")
    write_random_clip_gguf(p, out_dim=32, image_size=28, patch_size=14, E=32, F_=64, n_layer=1, n_head=2, use_gelu=True)
    enc = ClipEncoder(p, "cpu")
    px = preprocess(_png(seed=3), enc.cfg)
    ref = reference_encode(p, px)
    assert np.linalg.norm(enc.encode_pixels(px).numpy() - ref) / np.linalg.norm(ref) < 1e-4


def test_preprocess_pads_to_square_with_mean(tiny_clip):
    enc = ClipEncoder(tiny_clip, "cpu")
    im = np.zeros((10, 28, 3), np.uint8)  # wide black strip: padded above and below with the mean colour
    a = preprocess(im, enc.cfg)
    assert a.shape == (3, 28, 28)
    top = a[:, 0, 0]
    assert np.allclose(top, 0.0, atol=0.02)  # mean colour normalises to ~0
    mid = a[:, 14, 14]
    assert (mid < -1.0).all()  # black, normalised
    with pytest.raises(VisionError):
        preprocess(b"not an image", enc.cfg)


def test_image_token_ids_stable_and_negative():
    reg = ImageIds()
    a = reg.ids_for(b"img-a", 576)
    assert a == reg.ids_for(b"img-a", 576) and len(set(a)) == 576
    assert all(-(2 ** 31) < t < 0 for t in a)
    assert not set(a) & set(reg.ids_for(b"img-b", 576))
    assert reg.issued(a[0]) and reg.issued(a[-1]) and not reg.issued(a[-1] - 1) and not reg.issued(5)


def test_image_ids_never_shared_by_colliding_digests():
    """A truncated-hash collision must not give two images the same ids (advisor r3): with ONE bucket
    pair, the second image is probed into the other bucket; the space, once full, refuses."""
    reg = ImageIds(n_buckets=2)
    a, b = reg.ids_for(b"first", 4), reg.ids_for(b"second", 4)
    assert not set(a) & set(b) and reg.ids_for(b"first", 4) == a
    with pytest.raises(VisionError):
        reg.ids_for(b"third", 4)


def test_preprocess_rejects_huge_or_thin_canvas(tiny_clip):
    """A tiny PNG declaring a 1 x 200000 canvas is refused from its header (no 200000^2 padding); a
    large-but-legal image is downscaled before padding (bounded memory)."""
    import io as _io
    from PIL import Image
    cfg = ClipEncoder(tiny_clip).cfg
    buf = _io.BytesIO()
    Image.new("RGB", (1, 20000), (0, 0, 0)).save(buf, format="PNG")
    data = bytearray(buf.getvalue())
    # patch the IHDR height field (bytes 20..24) to 200000: the header alone declares the canvas
    data[20:24] = (200000).to_bytes(4, "big")
    with pytest.raises(VisionError):
        preprocess(bytes(data), cfg)
    buf = _io.BytesIO()
    Image.new("RGB", (4000, 30), (255, 0, 0)).save(buf, format="PNG")
    a = preprocess(buf.getvalue(), cfg)
    assert a.shape == (3, cfg.image_size, cfg.image_size) and np.isfinite(a).all()


@pytest.mark.parametrize("backend", ["torch", "native"])
def test_ext_row_equal_to_token_embedding_gives_token_logits(tiny_models, backend):
    from ollama_operator_amd.engine.runner import Runner
    from ollama_operator_amd.ops.reference import TorchExecutor  # noqa: F401  (twin import check)
    if backend == "native":
        from ollama_operator_amd.ops import cpu
        if cpu.cpu_module() is None:
            pytest.skip("CPU backend module not built")
    r = Runner(tiny_models["tiny-llama"], device="cpu", max_batch=8, max_seqs=6, ctx=64, cpu_backend=backend,
               ext_rows=16)
    V = r.cfg.n_vocab
    prompt = [1, 17, 42, 99, 5, 230, 7, 11, 64]
    s0 = r.new_sequence()
    r.prefill(s0, prompt)
    want = r.logits[0, :V].clone()
    # rows 42 and 230 replaced by external rows holding exactly their embeddings
    from ollama_operator_amd.quant import dequantize
    from ollama_operator_amd.gguf import read_gguf
    g = read_gguf(tiny_models["tiny-llama"])
    t = g.tensors["token_embd.weight"]
    emb = dequantize(g.raw("token_embd.weight"), t.ggml_type, t.n_elements).reshape(t.torch_shape)
    g.close()
    ids = [-1000, -1001]
    r.set_ext(ids, emb[[42, 230]] * r.cfg.embed_scale)
    s1 = r.new_sequence()
    r.prefill(s1, [1, 17, -1000, 99, 5, -1001, 7, 11, 64])
    got = r.logits[0, :V]
    assert torch.allclose(got, want, rtol=1e-5, atol=1e-5)
    # different rows change the result
    r.set_ext([-2000], np.random.default_rng(0).standard_normal((1, E_LLM)).astype(np.float32))
    s2 = r.new_sequence()
    r.prefill(s2, [1, 17, -2000, 99, 5, 230, 7, 11, 64])
    assert not torch.allclose(r.logits[0, :V], want, atol=1e-3)
    with pytest.raises(ValueError):
        r.prefill(r.new_sequence(), [1, -31337])  # unregistered id
    # sampling penalties ignore external rows
    toks = list(r.generate(r.new_sequence(), [1, 17, -1000, 99], max_tokens=3))
    assert len(toks) == 3 and all(0 <= x < V for x in toks)


def test_set_ext_ring_keeps_known_ids(tiny_models):
    from ollama_operator_amd.engine.runner import Runner
    r = Runner(tiny_models["tiny-llama"], device="cpu", max_batch=8, max_seqs=2, ctx=64, ext_rows=4)
    rows = np.arange(3 * E_LLM, dtype=np.float32).reshape(3, E_LLM)
    r.set_ext([-1, -2, -3], rows)
    r.set_ext([-1, -2, -3], rows + 1)  # already registered: unchanged
    assert torch.equal(r.ext[:3], torch.from_numpy(rows))
    r.set_ext([-4, -5], rows[:2])  # wraps: rows 0, 1 reused, ids -1 / -2 dropped
    assert set(r._ext_map) == {-3, -4, -5}
    with pytest.raises(ValueError):
        r.set_ext([-9] * 5, np.zeros((5, E_LLM), np.float32))
    with pytest.raises(ValueError):
        r.set_ext([3], rows[:1])


# ------------------------------------------------------------------------------------- server
@pytest.fixture(scope="module")
def llava_client(tmp_path_factory, tiny_models, tiny_clip):
    from fastapi.testclient import TestClient
    from ollama_operator_amd.server.app import create_app
    from ollama_operator_amd.server.manager import ModelManager
    from ollama_operator_amd.server.store import MT_PROJECTOR, ModelStore
    root = str(tmp_path_factory.mktemp("llava_store"))
    st = ModelStore(root)
    app = create_app(st, ModelManager(st, device="cpu"))
    c = TestClient(app)
    mf = f"FROM {tiny_models['tiny-llama']}\nFROM {tiny_clip}\nTEMPLATE \"USER: {{{{ .Prompt }}}} ASSISTANT:\"\n" \
         "PARAMETER temperature 0\nPARAMETER num_ctx 128\n"
    r = c.post("/api/create", json={"model": "tiny-llava", "modelfile": mf, "stream": False})
    assert r.status_code == 200, r.text
    m = st.read_manifest("tiny-llava")
    assert m.layer(MT_PROJECTOR) is not None
    st.create("tiny-text", gguf_path=tiny_models["tiny-llama"], params={"temperature": 0.0, "num_ctx": 128})
    return c


def test_generate_with_image(llava_client):
    img = base64.b64encode(_png()).decode()
    body = {"model": "tiny-llava", "prompt": "what is in this picture?", "images": [img], "stream": False,
            "options": {"num_predict": 6, "seed": 1}}
    r = llava_client.post("/api/generate", json=body)
    assert r.status_code == 200, r.text
    d = r.json()
    assert d["done"] and d["eval_count"] >= 1
    ctx = d["context"]
    assert sum(1 for t in ctx if t < 0) == 4  # 4 patches of the tiny encoder
    # deterministic and image-dependent
    assert llava_client.post("/api/generate", json=body).json()["response"] == d["response"]
    other = dict(body, images=[base64.b64encode(_png(seed=9)).decode()])
    d2 = llava_client.post("/api/generate", json=other).json()
    assert [t for t in d2["context"] if t < 0] != [t for t in ctx if t < 0]
    # explicit marker position
    body3 = dict(body, prompt="before [img-0] after")
    d3 = llava_client.post("/api/generate", json=body3).json()
    assert d3["done"]
    # multi-turn: the returned context (with its image ids) is accepted back...
    d4 = llava_client.post("/api/generate", json={"model": "tiny-llava", "prompt": " more", "context": ctx,
                                                  "stream": False, "options": {"num_predict": 2}})
    assert d4.status_code == 200, d4.text
    # ...but a negative id this server never issued (another row of the shared ring) is refused
    bad = llava_client.post("/api/generate", json={"model": "tiny-llava", "prompt": "x", "context": [1, -7],
                                                   "stream": False, "options": {"num_predict": 2}})
    assert bad.status_code == 400 and "context" in bad.json()["error"]


def test_chat_and_openai_with_image(llava_client):
    img = base64.b64encode(_png(seed=2)).decode()
    r = llava_client.post("/api/chat", json={"model": "tiny-llava", "stream": False, "options": {"num_predict": 4},
                                             "messages": [{"role": "user", "content": "describe", "images": [img]}]})
    assert r.status_code == 200, r.text
    assert r.json()["done"]
    r = llava_client.post("/v1/chat/completions", json={
        "model": "tiny-llava", "max_tokens": 4,
        "messages": [{"role": "user", "content": [{"type": "text", "text": "describe"},
                                                  {"type": "image_url", "image_url": {"url": "data:image/png;base64," + img}}]}]})
    assert r.status_code == 200, r.text
    assert r.json()["choices"][0]["message"]["role"] == "assistant"


def test_images_rejected_without_projector(llava_client):
    img = base64.b64encode(_png()).decode()
    r = llava_client.post("/api/generate", json={"model": "tiny-text", "prompt": "hi", "images": [img], "stream": False})
    assert r.status_code == 400 and "image" in r.json()["error"]
    r = llava_client.post("/api/generate", json={"model": "tiny-llava", "prompt": "hi", "images": ["%%%"],
                                                 "stream": False})
    assert r.status_code == 400


def test_show_lists_clip_family(llava_client):
    d = llava_client.post("/api/show", json={"model": "tiny-llava"}).json()
    assert "clip" in (d.get("details", {}).get("families") or [])


# ------------------------------------------------------------------ LLaVA-1.6 any-resolution
PINS = [(28, 56), (56, 28), (56, 56)]


@pytest.fixture(scope="module")
def anyres_clip(tmp_path_factory):
    p = str(tmp_path_factory.mktemp("clip16") / "mmproj.gguf")
    write_random_clip_gguf(p, out_dim=E_LLM, image_size=28, patch_size=7, E=64, F_=128, n_layer=2, n_head=4, seed=4,
                           grid_pinpoints=PINS)
    return p


def test_select_best_resolution_llava16_grid():
    grid = [(336, 672), (672, 336), (672, 672), (1008, 336), (336, 1008)]
    assert select_best_resolution((400, 200), grid) == (672, 336)  # keeps every pixel with the least waste
    assert select_best_resolution((200, 400), grid) == (336, 672)
    assert select_best_resolution((1000, 1000), grid) == (672, 672)  # most pixels kept
    assert select_best_resolution((2000, 500), grid) == (1008, 336)
    assert select_best_resolution((20, 30), PINS) == (28, 56)


def test_anyres_preprocess_views_and_padding(anyres_clip):
    enc = ClipEncoder(anyres_clip, "cpu")
    c = enc.cfg
    assert c.grid_pinpoints == tuple(PINS) and c.merge == "spatial_unpad"
    assert c.max_rows == 16 + 8 * 9  # base 4x4 + the 56x56 grid (8 x 8 patches + a newline per row)
    img = np.full((30, 20, 3), 200, np.uint8)  # 20 wide, 30 tall -> grid 28 x 56 (two tiles stacked)
    views, size, grid = preprocess_anyres(img, c)
    assert views.shape == (3, 3, 28, 28) and size == (20, 30) and grid == (28, 56)
    black = (0.0 - np.asarray(c.mean)) / np.asarray(c.std)
    # fitted 28 x 42, centred: rows 0..6 of the top tile and 49..55 (tile 2 rows 21..27) are black bands
    assert np.allclose(views[1][:, :7].transpose(1, 2, 0), black, atol=1e-5)
    assert np.allclose(views[2][:, 21:].transpose(1, 2, 0), black, atol=1e-5)
    assert not np.allclose(views[1][:, 8], black[:, None], atol=0.1)


def _oracle_anyres(path, img, c):
    """Stitch per-view fp64 oracle features the LLaVA-NeXT way, written independently of ClipEncoder."""
    from ollama_operator_amd.gguf import read_gguf
    views, (w, h), (W, H) = preprocess_anyres(img, c)
    f = [reference_encode(path, v) for v in views]
    g, S = c.image_size // c.patch_size, c.image_size
    gw, gh = W // S, H // S
    rows, cols = gh * g, gw * g
    full = np.zeros((rows, cols, f[0].shape[1]))
    for R in range(rows):
        for C in range(cols):
            full[R, C] = f[1 + (R // g) * gw + C // g][(R % g) * g + C % g]
    if w * rows > h * cols:  # wider than the grid: trim rows
        keep = int(h * cols / w)
        p = (rows - keep) // 2
        full = full[p:rows - p]
    else:
        keep = int(w * rows / h)
        p = (cols - keep) // 2
        full = full[:, p:cols - p]
    gg = read_gguf(path)
    nl = np.asarray(gg.array("model.image_newline"), np.float64).reshape(-1)
    gg.close()
    out = [f[0]]
    for r in full:
        out += [r, nl[None]]
    return np.concatenate(out)


@pytest.mark.parametrize("shape", [(30, 20), (24, 40), (50, 50)])
def test_anyres_encode_matches_oracle(anyres_clip, shape):
    enc = ClipEncoder(anyres_clip, "cpu")
    img = (np.random.default_rng(sum(shape)).random(shape + (3,)) * 255).astype(np.uint8)
    got = enc.encode(img).numpy()
    ref = _oracle_anyres(anyres_clip, img, enc.cfg)
    assert got.shape == ref.shape and got.shape[0] <= enc.cfg.max_rows
    assert np.linalg.norm(got - ref) / np.linalg.norm(ref) < 1e-4


def test_anyres_flat_merge_and_bad_metadata(tmp_path):
    p = str(tmp_path / "flat.gguf")
    write_random_clip_gguf(p, out_dim=32, image_size=28, patch_size=14, E=32, F_=64, n_layer=1, n_head=2,
                           grid_pinpoints=[(56, 28)], merge="flat")
    enc = ClipEncoder(p, "cpu")
    assert enc.encode(np.zeros((10, 30, 3), np.uint8)).shape == (12, 32)  # base + 2 tiles, 4 patches each
    bad = str(tmp_path / "bad.gguf")
    write_random_clip_gguf(bad, out_dim=32, image_size=28, patch_size=14, E=32, F_=64, n_layer=1, n_head=2,
                           grid_pinpoints=[(50, 28)])
    with pytest.raises(VisionError):
        ClipEncoder(bad, "cpu")
