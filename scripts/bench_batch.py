"""Continuous-batching decode step cost on one GPU: B sequences per step (engine/scheduler.py shape),
ms per step and aggregate tok/s for each B, with the B = 1 step as the reference. Run under
`rocprofv3 --kernel-trace --stats` for the per-kernel split of the batched step.

    python scripts/bench_batch.py [--model llama2-7b] [--ftype Q4_K_M] [--batches 1,2,4,8] [--steps 64]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama2-7b")
    ap.add_argument("--ftype", default="Q4_K_M", type=str.upper)
    ap.add_argument("--dir", default=os.environ.get("OMX_BENCH_DIR", "/tmp/omx_bench_models"))
    ap.add_argument("--batches", default="1,4")
    ap.add_argument("--steps", type=int, default=64)
    ap.add_argument("--warmup", type=int, default=8)
    ap.add_argument("--prompt", type=int, default=128)
    a = ap.parse_args()
    import torch

    import bench
    from ollama_operator_amd.engine.runner import Runner
    from ollama_operator_amd.engine.sampling import SamplingOptions
    path = os.path.join(a.dir, f"{a.model}-{a.ftype.lower()}.gguf")
    os.makedirs(a.dir, exist_ok=True)
    bench.ensure_model(path, a.model, a.ftype)
    Bs = [int(b) for b in a.batches.split(",")]
    runner = Runner(path, device="cuda", max_batch=256, max_seqs=max(2, max(Bs)),
                    ctx=a.prompt + a.warmup + a.steps + 64)
    out = {}
    for B in Bs:
        runner.capture_batch_graphs(B) if B > 1 else None
        g = torch.Generator().manual_seed(4321)
        sids, poss, firsts, prompts = [], [], [], []
        for b in range(B):
            p = [1] + torch.randint(3, runner.cfg.n_vocab, (a.prompt - 1,), generator=g).tolist()
            sid = runner.new_sequence()
            runner.prefill(sid, p)
            runner._set_sampler(0, SamplingOptions(seed=7 + b), p, 7 + b, 0)
            runner._sample(1)
            firsts.append(int(runner.s_out[0].item()))
            sids.append(sid)
            poss.append(len(p))
            prompts.append(p)
        for b in range(B):
            runner._set_sampler(b, SamplingOptions(seed=7 + b), prompts[b] + [firsts[b]], 7 + b, 1)
        runner.set_tokens(firsts)
        evs = []

        def step():
            runner.decode_batch(sids, poss)
            for b in range(B):
                poss[b] += 1
            e = torch.cuda.Event()
            e.record()
            evs.append(e)
            if len(evs) > 2:
                evs.pop(0).synchronize()

        for _ in range(a.warmup):
            step()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            step()
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / a.steps * 1e3
        out[B] = {"ms_per_step": round(ms, 4), "tok_s": round(B * 1e3 / ms, 1)}
        for sid in sids:
            runner.free_sequence(sid)
        print(f"B={B}: {ms:.4f} ms/step, {B * 1e3 / ms:.1f} tok/s", flush=True)
    if 1 in out:
        for B in out:
            out[B]["vs_b1_cost"] = round(out[B]["ms_per_step"] / out[1]["ms_per_step"], 3)
    print(json.dumps({"model": a.model, "ftype": a.ftype, "steps": a.steps, "batches": out}))


if __name__ == "__main__":
    main()
