"""A/B inside one process: batch-1 decode with the attention's consecutive-page arithmetic (page0) vs the
block-table load, alternating blocks of 96 steps, after a 128- and a 2048-token prompt.
Run on the GPU box: python experiments/ab/page0.py"""
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
    for L in (128, 2048):
        p = [1] + torch.randint(3, r.cfg.n_vocab, (L - 1,), generator=g).tolist()
        sid = r.new_sequence()
        gen = r.generate(sid, p, SamplingOptions(temperature=0.8, top_k=40, top_p=0.9), max_tokens=1000)
        for _ in range(8):
            next(gen)
        res = {True: [], False: []}
        for rnd in range(4):
            for on in (False, True):
                r.attn_page0 = on
                r._adv_next = None  # the next step re-uploads its inputs (page0 or -1)
                for _ in range(4):
                    next(gen)
                torch.cuda.synchronize()
                s0, t0 = r.steps_issued, time.perf_counter()
                while r.steps_issued - s0 < 96:
                    next(gen)
                torch.cuda.synchronize()
                res[on].append((r.steps_issued - s0) / (time.perf_counter() - t0))
        for on, xs in res.items():
            print(f"prompt {L}: page0 {int(on)}: mean {sum(xs) / len(xs):.1f} tok/s  {[round(x, 1) for x in xs]}",
                  flush=True)
        gen.close()
        r.free_sequence(sid)


if __name__ == "__main__":
    main()
