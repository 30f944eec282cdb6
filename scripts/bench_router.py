"""Fused MoE router microbenchmark (csrc/kernels/moe.hip moe_router) on the Mixtral-8x7B shape
(8 experts x 4096, Q8_0 as the loader requantises the F32 router): per-launch time in a hipGraph over
rotating copies of the router rows (cold, as in a decode step where 32 layers' routers are touched
once each), and the in-kernel phase timeline from s_memrealtime stamps (100 MHz).

    python scripts/bench_router.py [--B 1]
"""
import argparse
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ollama_operator_amd.gguf import GGMLType  # noqa: E402
from ollama_operator_amd.ops import native  # noqa: E402
from ollama_operator_amd.quant import REPACK_STREAMS, random_blocks, repack  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=1)
    ap.add_argument("--copies", type=int, default=256)
    a = ap.parse_args()
    C = native()
    X, K, B, k = 8, 4096, a.B, 2
    qt = GGMLType.Q8_0
    st = repack(random_blocks(qt, X, K, np.random.default_rng(0)), qt, X, K)
    base = [torch.from_numpy(np.ascontiguousarray(st[n])).cuda() for n in REPACK_STREAMS[qt]]
    tups = []
    keep = []
    for c in range(a.copies):
        ts = [t.clone() for t in base]
        keep.append(ts)
        p = [t.data_ptr() for t in ts] + [0] * (4 - len(ts))
        tups.append((p[0], p[1], p[2], p[3], X, K, int(qt)))
    xs = [torch.randn(B, K, device="cuda") for _ in range(a.copies)]
    nw = torch.rand(K, device="cuda") + 0.5
    ids = torch.zeros(B, k, dtype=torch.int32, device="cuda")
    w = torch.zeros(B, k, device="cuda")
    ts = torch.zeros(a.copies, B, 8, dtype=torch.int64, device="cuda")

    def launch(i, stamps=False):
        C.moe_router(tups[i], B, xs[i].data_ptr(), K, nw.data_ptr(), 1e-5, k, ids.data_ptr(), w.data_ptr(),
                     torch.cuda.current_stream().cuda_stream, ts[i].data_ptr() if stamps else 0)

    for i in range(4):
        launch(i)
    torch.cuda.synchronize()
    for stamps in (False, True):
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for i in range(a.copies):
                launch(i, stamps)
        g.replay()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(5):
            g.replay()
        e1.record()
        torch.cuda.synchronize()
        print(f"B={B} stamps={int(stamps)}: {e0.elapsed_time(e1) * 1e3 / (5 * a.copies):6.2f} us/launch", flush=True)
    t = ts[:, 0, :5].cpu().numpy().astype(np.float64) * 0.01  # 100 MHz ticks -> us
    d = np.diff(t, axis=1)
    med = np.median(d, axis=0)
    gap = np.median(t[1:, 0] - t[:-1, 4])
    print("phase medians (us): stats %.2f  stage %.2f  dots %.2f  top-k %.2f  | entry-to-exit %.2f  "
          "exit->next entry %.2f" % (*med, med.sum(), gap), flush=True)


if __name__ == "__main__":
    main()
