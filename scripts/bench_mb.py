"""Microbenchmark of the batched matrix-core decode GEMV (csrc/kernels/gemv_mfma.hip) on the
Llama-2-7B Q4_K_M shapes, as the decode chain launches them (fp16 activations from global memory,
RMS partials, residual emission, fp16 GLU output). Each configuration is captured into a hipGraph of
launches over rotating copies of the layout M weights (so they stream from HBM, not the 256 MiB
Infinity Cache) and timed per launch.

    python scripts/bench_mb.py [--batches 4,16] [--dbg 0,1,2,3,7] [--bpc 1,2] [--shapes qk,v,...]
"""
import argparse
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ollama_operator_amd.gguf import GGMLType  # noqa: E402
from ollama_operator_amd.ops import native  # noqa: E402
from ollama_operator_amd.quant import random_blocks, repack  # noqa: E402

STREAMS = {GGMLType.Q4_K: ["qs", "meta"], GGMLType.Q6_K: ["ql", "qh", "sc", "d"],
           GGMLType.Q4_0: ["qs", "d"], GGMLType.Q8_0: ["qs", "d"]}
SHAPES = {  # name: (qtype, N, K, kind)
    "qk": (GGMLType.Q4_K, 8192, 4096, "norm_store"),
    "v": (GGMLType.Q6_K, 4096, 4096, "norm_store"),
    "o": (GGMLType.Q4_K, 4096, 4096, "add_emit"),
    "gate_up": (GGMLType.Q4_K, 22016, 4096, "norm_glu16"),
    "down_q6k": (GGMLType.Q6_K, 4096, 11008, "add_emit"),
    "down_q4k": (GGMLType.Q4_K, 4096, 11008, "add_emit"),
    "lm_head": (GGMLType.Q6_K, 32000, 4096, "norm_store"),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batches", default="4,16")
    ap.add_argument("--dbg", default="0,1,2,3,7")
    ap.add_argument("--bpc", default="1")
    ap.add_argument("--shapes", default=",".join(SHAPES))
    ap.add_argument("--launches", type=int, default=24)
    a = ap.parse_args()
    C = native()
    s = torch.cuda.current_stream().cuda_stream
    for name in a.shapes.split(","):
        qt, N, K, kind = SHAPES[name]
        rng = np.random.default_rng(0)
        raw = random_blocks(qt, N, K, rng)
        st = repack(raw, qt, N, K)
        streams = [torch.from_numpy(np.ascontiguousarray(st[n])).cuda() for n in STREAMS[qt]]
        p = [t.data_ptr() for t in streams] + [0] * (4 - len(streams))
        base = (p[0], p[1], p[2], p[3], N, K, int(qt))
        nb = C.mfma_layout_bytes(int(qt), N, K)
        m0 = torch.empty(nb, dtype=torch.uint8, device="cuda")
        C.repack_m(base, m0.data_ptr(), s)
        copies = max(2, (768 << 20) // nb)
        mts = [m0] + [m0.clone() for _ in range(copies - 1)]
        ld = (K + 255) // 256 * 256
        for B in [int(b) for b in a.batches.split(",")]:
            x = torch.randn(B, K, device="cuda")
            x16 = torch.zeros(17, ld, device="cuda", dtype=torch.float16)
            x16[:B, :K] = x.half()
            parts = torch.rand((K + 15) // 16, 16, device="cuda")
            nw = torch.rand(max(N, K), device="cuda") + 0.5
            y = torch.zeros(B, N, device="cuda")
            y16 = torch.zeros(17, N, device="cuda", dtype=torch.float16)
            e16 = torch.zeros(17, N, device="cuda", dtype=torch.float16)
            est = torch.zeros((N + 15) // 16 * 16, device="cuda")
            extra = dict(x16=x16.data_ptr(), ld16=ld, zrow16=16)
            norm, epi = 0, 0
            if kind.startswith("norm"):
                norm = 1
                extra.update(xstat=parts.data_ptr(), xstat_n=(K + 15) // 16)
            if kind == "norm_glu16":
                epi = 2
                extra.update(y16=y16.data_ptr(), ld16y=N)
            if kind == "add_emit":
                epi = 1
                extra.update(emit16=e16.data_ptr(), ld_emit=N, emit_nw=nw.data_ptr(), emit_stat=est.data_ptr())

            def launch(i):
                C.gemv(base + (0, mts[i % len(mts)].data_ptr()), B, x.data_ptr(), K, norm, nw.data_ptr(), 0, 1e-5,
                       epi, y.data_ptr(), N if epi != 2 else N // 2, 0, 0, extra,
                       torch.cuda.current_stream().cuda_stream)  # the capture stream inside graph()

            for bpc in [int(v) for v in a.bpc.split(",")]:
                for dbg in [int(v) for v in a.dbg.split(",")]:
                    C.set_mb_tuning(dbg, bpc)
                    for i in range(3):
                        launch(i)
                    torch.cuda.synchronize()
                    g = torch.cuda.CUDAGraph()
                    with torch.cuda.graph(g):
                        for i in range(a.launches):
                            launch(i)
                    g.replay()
                    torch.cuda.synchronize()
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    reps = 10
                    e0.record()
                    for _ in range(reps):
                        g.replay()
                    e1.record()
                    torch.cuda.synchronize()
                    us = e0.elapsed_time(e1) * 1e3 / (reps * a.launches)
                    print(f"{name:9s} B={B:2d} bpc={bpc} dbg={dbg}: {us:7.2f} us/launch  "
                          f"{raw.nbytes / us / 1e6:6.2f} TB/s", flush=True)
        C.set_mb_tuning(0, 1)


if __name__ == "__main__":
    main()
