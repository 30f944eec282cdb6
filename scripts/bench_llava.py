"""LLaVA-1.5-7B-shaped multimodal benchmark on one GPU: random-init Llama-2-7B Q4_K_M language model +
random-init CLIP ViT-L/14-336 projector (23 blocks, 4096-wide MLP projector, F16), as an Ollama llava
model is laid out. Measures the image encode (576 patch rows), the time to first token of an
image + 64-token prompt (encode + 640-row prefill), and decode tok/s after it.

    python scripts/bench_llava.py [--steps 128] [--dir /tmp/omx_bench]
"""
import argparse
import io
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from bench import ensure_model  # noqa: E402
from ollama_operator_amd.engine.runner import Runner  # noqa: E402
from ollama_operator_amd.engine.sampling import SamplingOptions  # noqa: E402
from ollama_operator_amd.models.clip import ClipEncoder, ImageIds, write_random_clip_gguf  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=128)
    ap.add_argument("--dir", default=os.environ.get("OMX_BENCH_DIR", "/tmp/omx_bench"))
    a = ap.parse_args()
    lm = ensure_model(os.path.join(a.dir, "llama2-7b-Q4_K_M.gguf"), "llama2-7b", "Q4_K_M")
    mmproj = os.path.join(a.dir, "clip-vit-l-336-mmproj-f16.gguf")
    if not os.path.exists(mmproj):
        write_random_clip_gguf(mmproj + ".tmp", out_dim=4096)
        os.replace(mmproj + ".tmp", mmproj)
    enc = ClipEncoder(mmproj, "cuda")
    r = Runner(lm, device="cuda", max_batch=2048, max_seqs=2, ctx=2048, ext_rows=2 * enc.cfg.n_patches)
    r.warmup()
    from PIL import Image

    def png(seed):
        buf = io.BytesIO()
        Image.fromarray((np.random.default_rng(seed).random((480, 640, 3)) * 255).astype(np.uint8)).save(buf, "PNG")
        return buf.getvalue()
    img = png(0)
    for _ in range(3):
        enc.encode(img)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(10):
        rows = enc.encode(img)
    torch.cuda.synchronize()
    enc_ms = (time.perf_counter() - t0) * 1e3 / 10
    rng = np.random.default_rng(1)
    text = [int(t) for t in rng.integers(100, 30000, 64)]

    def ttft(prompt_img: bytes):
        torch.cuda.synchronize()
        t = time.perf_counter()
        rows = enc.encode(prompt_img)
        ids = ImageIds().ids_for(prompt_img, rows.shape[0])
        r.set_ext(ids, rows)
        sid = r.new_sequence()
        g = r.generate(sid, [1] + ids + text, SamplingOptions(temperature=0), max_tokens=a.steps)
        next(g)
        dt = (time.perf_counter() - t) * 1e3
        return sid, g, dt

    sid, g, _ = ttft(img)  # warm: plans, graphs
    for _ in g:
        pass
    r.free_sequence(sid)
    img2 = png(1)  # a different image: no KV prefix reuse
    sid, g, t_ms = ttft(img2)
    t1 = time.perf_counter()
    n = 1 + sum(1 for _ in g)
    dec = (n - 1) / (time.perf_counter() - t1)
    out = {"model": "LLaVA-1.5-7B shaped (Llama-2-7B Q4_K_M + CLIP ViT-L/14-336 F16 projector), random init",
           "image_patches": int(rows.shape[0]), "image_encode_ms": round(enc_ms, 2),
           "ttft_image_plus_64_tokens_ms": round(t_ms, 2), "decode_tok_s": round(dec, 1), "steps": n}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
