"""Prefill GEMM microbenchmark on Llama-2-7B Q4_K_M shapes: the stream-order dequant GEMM
(csrc/kernels/gemm_dq.hip, "dq", the default), the 128 x 128 natural-order tile (gemm.hip, "tile") and
the hipBLASLt path (prep + dequant to fp16 + library GEMM + epilogue pass; csrc/runtime/blas.cpp; opt-in
since round 6) and the register-ring edition of the dq kernel ("ring", the default since round 6; "dq" is
the glds edition): time per call (everything the path launches) and TFLOP/s vs M (prompt tokens). On the
GPU box:
  python scripts/bench_gemm.py   (OMX_BENCH_SHAPES / OMX_BENCH_M / OMX_BENCH_PATHS filter, e.g. for PMC runs)"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ollama_operator_amd.gguf import GGMLType  # noqa: E402
from ollama_operator_amd.ops import native  # noqa: E402
from ollama_operator_amd.quant import REPACK_STREAMS, random_blocks, repack  # noqa: E402

SHAPES = [("qkv", GGMLType.Q4_K, 12288, 4096), ("o", GGMLType.Q4_K, 4096, 4096),
          ("gate_up", GGMLType.Q4_K, 22016, 4096), ("down_q4k", GGMLType.Q4_K, 4096, 11008),
          ("down_q6k", GGMLType.Q6_K, 4096, 11008), ("q8_0", GGMLType.Q8_0, 4096, 4096)]


def main():
    C = native()
    s = torch.cuda.current_stream().cuda_stream
    keep = os.environ.get("OMX_BENCH_SHAPES")
    ms = [int(v) for v in os.environ.get("OMX_BENCH_M", "128,256,512,2048").split(",")]
    for name, qt, N, K in SHAPES:
        if keep and name not in keep.split(","):
            continue
        st = repack(random_blocks(qt, N, K, np.random.default_rng(0)), qt, N, K)
        ts = [torch.from_numpy(np.ascontiguousarray(st[n])).cuda() for n in REPACK_STREAMS[qt]]
        p = [t.data_ptr() for t in ts] + [0] * (4 - len(ts))
        tup = (p[0], p[1], p[2], p[3], N, K, int(qt))
        for M in ms:
            x = torch.randn(M, K, device="cuda")
            y = torch.zeros(M, N, device="cuda")
            xws = torch.empty(M * ((K + 255) // 256 * 256), device="cuda", dtype=torch.float16)
            gws = torch.empty(32 << 20, device="cuda")  # the runner's split-K workspace (GEMM_SPLIT_WS_FLOATS)
            w16 = torch.empty(N * K, device="cuda", dtype=torch.float16)
            yws = torch.empty(M * N, device="cuda")
            ws = {"xws": xws.data_ptr(), "xws_elems": xws.numel(), "gws": gws.data_ptr(), "gws_elems": gws.numel(), "w16ws": w16.data_ptr(),
                  "w16_elems": w16.numel(), "yws": yws.data_ptr(), "yws_elems": yws.numel()}
            paths = os.environ.get("OMX_BENCH_PATHS", "ring,dq,tile,hipblaslt").split(",")
            for path, min_m, dq in (("ring", 0, 1), ("dq", 0, 1), ("tile", 0, 0), ("hipblaslt", 1, 0)):
                if path not in paths:
                    continue
                fn = lambda: C.gemv(tup, M, x.data_ptr(), K, 0, 0, 0, 1e-5, 0, y.data_ptr(), N, 0, 0, ws, s)  # noqa: E731
                C.set_gemm_lib_min_m(min_m)
                C.set_dq_gemm(dq)
                C.set_dq_ring(1 if path == "ring" else 0)
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
                print(f"{name:9s} {qt.name:5s} N={N:6d} K={K:6d} M={M:5d} {path:9s}: {us:9.1f} us  "
                      f"{2 * M * N * K / us / 1e6:7.1f} TFLOP/s", flush=True)


if __name__ == "__main__":
    main()
