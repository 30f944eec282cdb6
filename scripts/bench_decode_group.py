"""A/B of decode steps per graph replay (Runner.decode_group) in ONE process, alternating, with the
bench's exact-step timing (steps enqueued in the window, syncs on both sides). On the GPU box:
    python scripts/bench_decode_group.py [--steps 128] [--groups 1,4,2,8] [--rounds 2]"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=128)
    ap.add_argument("--groups", default="1,4")
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--prompt", type=int, default=128)
    a = ap.parse_args()
    import torch
    from bench import ensure_model
    from ollama_operator_amd.engine.runner import Runner
    from ollama_operator_amd.engine.sampling import SamplingOptions
    path = ensure_model("/tmp/omx_bench/llama2-7b-q4_k_m.gguf", "llama2-7b", "Q4_K_M")
    groups = [int(x) for x in a.groups.split(",")]
    os.environ["OMX_DECODE_GROUP"] = str(max(groups))
    r = Runner(path, device="cuda", max_batch=2048, max_seqs=2, ctx=a.prompt + 2 * a.steps + 256)
    for G in groups:  # capture every group size's graphs up front
        r.decode_group = G
        r.warmup()
    g = torch.Generator().manual_seed(1)
    prompt = [1] + torch.randint(3, r.cfg.n_vocab, (a.prompt - 1,), generator=g).tolist()
    for rnd in range(a.rounds):
        for G in groups:
            r.decode_group = G
            sid = r.new_sequence()
            gen = r.generate(sid, prompt, SamplingOptions(seed=42), max_tokens=16 + a.steps + 4 * G + 4)
            for _ in range(16):
                next(gen)
            torch.cuda.synchronize()
            s0 = r.steps_issued
            t0 = time.perf_counter()
            while r.steps_issued - s0 < a.steps:
                next(gen)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            n = r.steps_issued - s0
            gen.close()
            r.free_sequence(sid)
            print(f"round {rnd} group {G}: {n} steps, {dt / n * 1e3:.4f} ms/step, {n / dt:.1f} tok/s", flush=True)


if __name__ == "__main__":
    main()
