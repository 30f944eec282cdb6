"""dq GEMM tile / split-K sweep (csrc/kernels/gemm_dq.hip) on Llama-2-7B Q4_K_M shapes: for every shape and
M, each forced (tile config, split-K) pair next to the automatic choice, time per call (prep + GEMM +
finalize) and TFLOP/s. Feeds the chooser in run_dq. On the GPU box: python scripts/bench_dq_sweep.py"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ollama_operator_amd.ops import native  # noqa: E402
from ollama_operator_amd.quant import REPACK_STREAMS, random_blocks, repack  # noqa: E402
from bench_gemm import SHAPES  # noqa: E402

CFGS = {0: "256x256", 1: "256x128", 2: "128x256", 3: "128x128"}


def main():
    C = native()
    s = torch.cuda.current_stream().cuda_stream
    ms = [int(v) for v in os.environ.get("OMX_BENCH_M", "512,1024,2048").split(",")]
    sks = [int(v) for v in os.environ.get("OMX_SWEEP_SK", "1,2,3,4").split(",")]
    gws = torch.empty(3 << 27, device="cuda")  # 1.5 GiB of split-K slabs
    for name, qt, N, K in SHAPES:
        st = repack(random_blocks(qt, N, K, np.random.default_rng(0)), qt, N, K)
        ts = [torch.from_numpy(np.ascontiguousarray(st[n])).cuda() for n in REPACK_STREAMS[qt]]
        p = [t.data_ptr() for t in ts] + [0] * (4 - len(ts))
        tup = (p[0], p[1], p[2], p[3], N, K, int(qt))
        for M in ms:
            x = torch.randn(M, K, device="cuda")
            y = torch.zeros(M, N, device="cuda")
            xws = torch.empty(M * ((K + 255) // 256 * 256), device="cuda", dtype=torch.float16)
            ws = {"xws": xws.data_ptr(), "xws_elems": xws.numel(), "gws": gws.data_ptr(), "gws_elems": gws.numel()}
            fn = lambda: C.gemv(tup, M, x.data_ptr(), K, 0, 0, 0, 1e-5, 0, y.data_ptr(), N, 0, 0, ws, s)  # noqa: E731
            C.set_gemm_lib_min_m(0)
            C.set_dq_gemm(1)
            res = []
            for cfg, sk in [(-1, 0)] + [(c, k) for c in CFGS for k in sks]:
                C.set_dq_tuning(cfg, sk)
                for _ in range(3):
                    fn()
                torch.cuda.synchronize()
                n = 20
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(n):
                    fn()
                e1.record()
                torch.cuda.synchronize()
                us = e0.elapsed_time(e1) * 1e3 / n
                res.append((us, "auto" if cfg < 0 else f"{CFGS[cfg]} sk={sk}"))
            C.set_dq_tuning(-1, 0)
            auto = res[0][0]
            best = min(res[1:])
            print(f"{name:9s} N={N:6d} K={K:6d} M={M:5d} auto {auto:8.1f} us {2 * M * N * K / auto / 1e6:6.1f} TF | best "
                  f"{best[1]:16s} {best[0]:8.1f} us {2 * M * N * K / best[0] / 1e6:6.1f} TF | "
                  + " ".join(f"{lbl}:{us:.0f}" for us, lbl in res[1:]), flush=True)


if __name__ == "__main__":
    main()
