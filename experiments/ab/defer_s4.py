"""A/B inside one process: batch-1 decode after a 2048-token prompt with 4 vs 8 deferred attention splits
(Runner.defer_s4_max 3072 vs 0), alternating blocks of 96 steps so clocks and KV placement are shared.
Run on the GPU box: python experiments/ab/defer_s4.py"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

import bench  # noqa: E402
from ollama_operator_amd.engine.runner import Runner  # noqa: E402
from ollama_operator_amd.engine.sampling import SamplingOptions  # noqa: E402


def main():
    d = os.environ.get("OMX_BENCH_DIR", "/tmp/omx_bench_models")
    os.makedirs(d, exist_ok=True)
    path = bench.ensure_model(os.path.join(d, "llama2-7b-q4_k_m.gguf"), "llama2-7b", "Q4_K_M")
    r = Runner(path, device="cuda:0", max_batch=2048, max_seqs=1, ctx=4096)
    r.warmup()
    g = torch.Generator().manual_seed(0)
    p = [1] + torch.randint(3, r.cfg.n_vocab, (2047,), generator=g).tolist()
    sid = r.new_sequence()
    gen = r.generate(sid, p, SamplingOptions(temperature=0.8, top_k=40, top_p=0.9), max_tokens=1000)
    for _ in range(8):
        next(gen)
    res = {0: [], 3072: []}
    for rnd in range(4):
        for v in (0, 3072):
            r.defer_s4_max = v
            for _ in range(4):  # drain the steps issued under the other setting
                next(gen)
            torch.cuda.synchronize()
            s0, t0 = r.steps_issued, time.perf_counter()
            while r.steps_issued - s0 < 96:
                next(gen)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            res[v].append((r.steps_issued - s0) / dt)
            print(f"round {rnd} s4max {v}: {res[v][-1]:.1f} tok/s (keys ~{r.kv.seqs[sid].length})", flush=True)
    for v, xs in res.items():
        print(f"s4max {v}: mean {sum(xs) / len(xs):.1f} tok/s over {len(xs)} blocks", flush=True)
    gen.close()


if __name__ == "__main__":
    main()
