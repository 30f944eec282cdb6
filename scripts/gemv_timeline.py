"""Intra-kernel timeline of the decode GEMV (flight kernel) per Llama-2-7B shape: every block stamps
s_memrealtime (100 MHz) at entry, prologue done (x normalised/quantised in LDS), first tile computed
(its weights had landed) and exit. Shows where a launch's fixed cost goes: dispatch ramp, activation
round trip, weight first-byte latency, tail. The launch runs right behind another GEMV on the same
stream (as in the decode graph) on MALL-cold weights.
Run on the GPU box:  python scripts/gemv_timeline.py"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench_gemv import SHAPES, make  # noqa: E402
from ollama_operator_amd.ops import native  # noqa: E402


def pct(a, q):
    return float(np.percentile(a, q)) * 10.0 / 1e3  # ticks (10 ns) -> us


def main():
    C = native()
    s = torch.cuda.current_stream().cuda_stream
    big = torch.empty(256 << 20, dtype=torch.uint8, device="cuda")
    for _ in range(50):
        big.add_(1)
    del big
    if os.environ.get("OMX_BENCH_KNOBS"):  # blocks/CU, rows, debug variant, ks
        C.set_gemv_tuning(*[int(v) for v in os.environ["OMX_BENCH_KNOBS"].split(",")])
    keep = os.environ.get("OMX_BENCH_SHAPES", "").split(",") if os.environ.get("OMX_BENCH_SHAPES") else None
    for name, qt, N, K, epi in SHAPES:
        if keep and name not in keep:
            continue
        tups, ts, nbytes = make(qt, N, K)
        x = torch.randn(1, K, device="cuda")
        nw = torch.ones(K, device="cuda")
        y = torch.zeros(1, N // 2 if epi == 2 else N, device="cuda")
        norm = 1 if name in ("qkv", "gate_up") else 0
        stamps = torch.zeros(4 * 4096 + 64, dtype=torch.int64, device="cuda")  # + grid counter (DBG 16)
        res = []
        for rep in range(6):
            stamps.zero_()
            a = tups[(2 * rep) % len(tups)]
            b = tups[(2 * rep + 1) % len(tups)]
            C.gemv(a, 1, x.data_ptr(), K, norm, nw.data_ptr(), 0, 1e-5, epi, y.data_ptr(), y.shape[1], 0, 0, {}, s)
            C.gemv(b, 1, x.data_ptr(), K, norm, nw.data_ptr(), 0, 1e-5, epi, y.data_ptr(), y.shape[1], 0, 0,
                   {"dbg_ts": stamps.data_ptr()}, s)
            torch.cuda.synchronize()
            t = stamps[:4 * 4096].view(-1, 4).cpu().numpy()
            t = t[t[:, 0] > 0].astype(np.float64)
            t0 = t[:, 0].min()
            t = t - t0
            res.append(t)
        t = np.concatenate(res[1:])
        nb = len(res[-1])
        span = np.mean([r[:, 3].max() for r in res[1:]]) * 10 / 1e3
        print(f"{name:9s} blocks={nb:4d} span={span:6.2f}us | entry p50/p90/max {pct(t[:,0],50):5.2f} {pct(t[:,0],90):5.2f} "
              f"{pct(t[:,0],100):5.2f} | prologue p50/p90 {pct(t[:,1]-t[:,0],50):5.2f} {pct(t[:,1]-t[:,0],90):5.2f} "
              f"| weights-after-prologue p50/p90 {pct(t[:,2]-t[:,1],50):5.2f} {pct(t[:,2]-t[:,1],90):5.2f} "
              f"| first-tile p50 {pct(t[:,2],50):5.2f} | rest p50 {pct(t[:,3]-t[:,2],50):5.2f} "
              f"| exit p10/p50/p90/max {pct(t[:,3],10):5.2f} {pct(t[:,3],50):5.2f} {pct(t[:,3],90):5.2f} {pct(t[:,3],100):5.2f}",
              flush=True)


if __name__ == "__main__":
    main()
