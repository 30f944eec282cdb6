"""Decode-GEMV microbenchmark on the Llama-2-7B Q4_K_M shapes: achieved HBM GB/s per launch shape.
Run on the GPU box:  python scripts/bench_gemv.py  (prints one line per shape x tuning)."""
import itertools
import time
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
SHAPES = [  # (name, qtype, N, K, epi)
    ("qkv", GGMLType.Q4_K, 12288, 4096, 0),
    ("o", GGMLType.Q4_K, 4096, 4096, 1),
    ("gate_up", GGMLType.Q4_K, 22016, 4096, 2),
    ("down_q4k", GGMLType.Q4_K, 4096, 11008, 1),
    ("down_q6k", GGMLType.Q6_K, 4096, 11008, 1),
    ("v_q6k", GGMLType.Q6_K, 4096, 4096, 0),
    ("lm_head", GGMLType.Q6_K, 32000, 4096, 0),
]


def make(qt, N, K):
    """Enough copies of the matrix that rotating through them misses the 256 MiB Infinity Cache
    (decode streams 4 GB of distinct weights per token; a re-read matrix would be MALL-served)."""
    rng = np.random.default_rng(0)
    raw = random_blocks(qt, N, K, rng)
    st = repack(raw, qt, N, K)
    copies = max(2, (768 << 20) // raw.nbytes)
    if os.environ.get("OMX_BENCH_HOT"):  # one copy re-read: MALL/L2-served (prefetch upper bound)
        copies = 1
    tups, keep = [], []
    for _ in range(copies):
        ts = [torch.from_numpy(np.ascontiguousarray(st[n])).cuda() for n in STREAMS[qt]]
        p = [t.data_ptr() for t in ts] + [0] * (4 - len(ts))
        tups.append((p[0], p[1], p[2], p[3], N, K, int(qt)))
        keep.append(ts)
    return tups, keep, raw.nbytes


def main():
    C = native()
    s = torch.cuda.current_stream().cuda_stream
    res = []
    keep = os.environ.get("OMX_BENCH_SHAPES", "").split(",") if os.environ.get("OMX_BENCH_SHAPES") else None
    mats = {name: make(qt, N, K) for name, qt, N, K, _ in SHAPES if keep is None or name in keep}
    knobs = [(b, r, 0, 0) for b in (1, 2, 4) for r in (1, 2)]
    if os.environ.get("OMX_BENCH_DEBUG"):  # memory-path experiments on the Q4_K K=4096 kernel
        knobs = [(b, 1, d, 1) for b in (2, 4) for d in (0, 1, 2, 3)]
    if os.environ.get("OMX_BENCH_KS"):  # in-block K split of the flight kernel (1 = off), full and memory-only
        knobs = [(4, 1, d, k) for k in (1, 2, 3, 4) for d in (0, 3)]
        if os.environ["OMX_BENCH_KS"] != "1":  # e.g. OMX_BENCH_KS=3: all debug variants at that split
            knobs = [(4, 1, d, int(os.environ["OMX_BENCH_KS"])) for d in (0, 1, 2, 3)]
    if os.environ.get("OMX_BENCH_KNOBS"):  # e.g. "3,2,1" (profiling one configuration)
        knobs = [tuple(int(v) for v in os.environ["OMX_BENCH_KNOBS"].split(","))]
    shapes = SHAPES
    if os.environ.get("OMX_BENCH_SHAPES"):
        keep = os.environ["OMX_BENCH_SHAPES"].split(",")
        shapes = [s for s in SHAPES if s[0] in keep]
    # knob tuple: (blocks/CU, rows, debug, ks, xfirst, xbar, stream, stream_bpc, ws); missing -> defaults
    knobs = [tuple(k) + (0, 0, 0, 0, 0, 0, 0, 1, 0)[len(k):] for k in knobs]
    if os.environ.get("OMX_BENCH_XBAR_AB"):  # A/B of the x-barrier launch on every knob
        knobs = [k[:5] + (xb,) + k[6:] for k in knobs for xb in (0, 1)]
    if os.environ.get("OMX_BENCH_STREAM_AB"):  # flight vs streaming kernel (1 and 2 blocks per CU)
        knobs = [k[:6] + (0, 1) + k[8:] for k in knobs] + [k[:6] + (1, b) + k[8:] for k in knobs for b in (1, 2)]
    if os.environ.get("OMX_BENCH_WS_AB"):  # flight vs the wave-specialised LDS-DMA kernel (gemv_ws.hip)
        knobs = [k[:8] + (w,) for k in knobs for w in (0, 1)]
    # clock warm-up: the first shape measured on an idle GPU otherwise reads up to 2x slow
    big = torch.empty(256 << 20, dtype=torch.uint8, device="cuda")
    t0 = time.time()
    while time.time() - t0 < 1.5:
        big.add_(1)
    torch.cuda.synchronize()
    del big
    for (name, qt, N, K, epi), (bpc, rpw, r1, ks, xf, xb, st, sbpc, ws) in itertools.product(shapes, knobs):
        C.set_gemv_tuning(bpc, rpw, r1, ks, xf, xb, st, sbpc, ws=ws)
        tups, ts, nbytes = mats[name]
        x = torch.randn(1, K, device="cuda")
        nw = torch.ones(K, device="cuda")
        y = torch.zeros(1, N // 2 if epi == 2 else N, device="cuda")
        norm = 1 if name in ("qkv", "gate_up") else 0
        argl = [(tup, 1, x.data_ptr(), K, norm, nw.data_ptr(), 0, 1e-5, epi, y.data_ptr(), y.shape[1], 0, 0, {}, s)
                for tup in tups]
        for i in range(10):
            C.gemv(*argl[i % len(argl)])
        torch.cuda.synchronize()
        n = 200
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for i in range(n):
            C.gemv(*argl[i % len(argl)])
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / n
        res.append((name, f"blocks/CU={bpc} rows={rpw} dbg={r1} ks={ks} xfirst={xf} xbar={xb} stream={st}x{sbpc} ws={ws}",
                    us, nbytes / us / 1e3))
        print(f"{name:10s} {res[-1][1]} {us:8.2f} us  {nbytes/us/1e3:7.1f} GB/s", flush=True)
    C.set_gemv_tuning(4, 1, 0, 0, 0, 0, 0, 1, ws=0)
    print("best per shape:")
    for name in mats:
        b = min((r for r in res if r[0] == name), key=lambda r: ("dbg=0" not in r[1], r[2]))
        print(f"  {name:10s} {b[1]} {b[2]:.2f} us {b[3]:.0f} GB/s")


if __name__ == "__main__":
    main()
