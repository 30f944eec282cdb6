"""Probe: time Runner.admit_many (3 prompts x 129 rows) vs sequential admits on Llama-2-7B Q4_K_M."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from bench import ensure_model  # noqa: E402
from ollama_operator_amd.engine.runner import Runner  # noqa: E402
from ollama_operator_amd.engine.sampling import SamplingOptions  # noqa: E402

path = ensure_model("/tmp/omx_bench/llama2-7b-Q4_K_M.gguf", "llama2-7b", "Q4_K_M")
r = Runner(path, device="cuda", max_batch=2048, max_seqs=9, ctx=2048)
r.warmup()
o = SamplingOptions()
rng = np.random.default_rng(0)
for trial in range(3):
    prompts = [[1] + [int(x) for x in rng.integers(3, 30000, 128 + 7 * trial)] for _ in range(3)]
    sids = [r.new_sequence() for _ in prompts]
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    r.admit_many([(sid, 0, p, o, p, 0) for sid, p in zip(sids, prompts)])
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    for sid in sids:
        r.free_sequence(sid)
    sids = [r.new_sequence() for _ in prompts]
    t2 = time.perf_counter()
    for sid, p in zip(sids, prompts):
        r.admit(sid, 0, p, o, p, 0)
    torch.cuda.synchronize()
    t3 = time.perf_counter()
    for sid in sids:
        r.free_sequence(sid)
    print(f"trial {trial}: admit_many {1e3 * (t1 - t0):.1f} ms, 3 x admit {1e3 * (t3 - t2):.1f} ms", flush=True)
