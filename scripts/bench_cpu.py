"""CPU serving benchmark (BASELINE config 1: `image: phi`, CPU-only server, replicas=1).

Measures, in a fresh process, what the reference's demo recordings show for Phi-2 on a CPU node
(docs/public/demo.cast:528-579 load 5.2-6.6 s; demo-full.cast:868-1191 decode 8.4-10.7 tok/s):
  * first request -> first token: model load (GGUF mmap + repack) + prefill of a chat-sized prompt
  * decode tokens/s over N tokens (Ollama-default sampling)
  * peak RSS of the serving process
Weights: random-init Phi-2 Q4_0 GGUF (no network); backend: the native CPU engine (csrc/cpu).

    python scripts/bench_cpu.py [--model phi2] [--ftype Q4_0] [--tokens 64] [--out profiles/r3_cpu/phi2_q4_0.json]
"""
import argparse
import json
import os
import platform
import resource
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="phi2")
    ap.add_argument("--ftype", default="Q4_0")
    ap.add_argument("--tokens", type=int, default=64)
    ap.add_argument("--prompt", type=int, default=32)
    ap.add_argument("--dir", default=os.environ.get("OMX_BENCH_DIR", "/tmp/omx_bench"))
    ap.add_argument("--backend", default="native", choices=["native", "torch"])
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    from bench import ensure_model  # noqa: E402  (bench.py at the repo root)
    path = ensure_model(os.path.join(a.dir, f"{a.model}-{a.ftype.lower()}.gguf"), a.model, a.ftype)
    t_req = time.perf_counter()  # "first request": the server loads lazily, as Ollama does
    from ollama_operator_amd.engine.runner import Runner
    from ollama_operator_amd.engine.sampling import SamplingOptions
    r = Runner(path, device="cpu", max_batch=64, max_seqs=1, ctx=2048, cpu_backend=a.backend)
    t_loaded = time.perf_counter()
    prompt = [r.cfg.bos_id] + [(37 * i + 11) % (r.cfg.n_vocab - 3) + 3 for i in range(a.prompt - 1)]
    gen = r.generate(r.new_sequence(), prompt, SamplingOptions(seed=1), max_tokens=a.tokens + 1)
    next(gen)
    t_first = time.perf_counter()
    n = 0
    for _ in gen:
        n += 1
    t_end = time.perf_counter()
    from ollama_operator_amd.ops.cpu import cpu_module
    C = cpu_module()
    out = {
        "config": f"BASELINE config 1: {a.model} {a.ftype} CPU-only serving (random-init weights)",
        "backend": a.backend, "isa": C.isa() if C else None, "threads": C.threads() if C else None,
        "cpu": platform.processor() or platform.machine(), "cores": os.cpu_count(),
        "load_s": round(t_loaded - t_req, 3),
        "first_token_s": round(t_first - t_req, 3),
        "prefill_tokens": len(prompt), "prefill_s": round(t_first - t_loaded, 3),
        "decode_tokens": n, "decode_tok_s": round(n / (t_end - t_first), 2),
        "peak_rss_gb": round(resource.getrusage(resource.RUSAGE_SELF).ru_maxrss / 1e6, 3),
        "weights_gb": round(r.w.nbytes / 1e9, 3),
        "reference": {"load_s": [5.2, 6.6], "decode_tok_s": [8.4, 10.7], "ram_note": ">= 8 GB for a 7B model",
                      "sources": ["docs/public/demo.cast:528-579", "docs/public/demo-full.cast:868-1191",
                                  "README.md:64"]},
    }
    print(json.dumps(out))
    if a.out:
        os.makedirs(os.path.dirname(a.out), exist_ok=True)
        with open(a.out, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
