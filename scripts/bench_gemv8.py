"""Batch-1 decode GEMVs on the int8 activation chain (gemv8.hip), Llama-2-7B Q4_K_M shapes, each with its
production input (int8 image + RMS partials, or the plain image) and emission: time per launch inside a
replayed hipGraph of back-to-back launches, weights rotated over enough copies to miss the 256 MiB
Infinity Cache (decode streams 4 GB of distinct weights per token). OMX_BENCH_HOT=1: one copy re-read
(MALL-served: what a perfect weight prefetch would give). OMX_BENCH_DBG8=1: the memory path alone (no
dot products: what the launch + weight stream cost without the compute).
Run on the GPU box:  python scripts/bench_gemv8.py"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ollama_operator_amd.gguf import GGMLType  # noqa: E402
from ollama_operator_amd.ops import native  # noqa: E402
from ollama_operator_amd.quant import random_blocks, repack  # noqa: E402

STREAMS = {GGMLType.Q4_K: ["qs", "meta"], GGMLType.Q6_K: ["ql", "qh", "sc", "d"],
           GGMLType.Q4_0: ["qs", "d"], GGMLType.Q8_0: ["qs", "d"]}
EPI_STORE, EPI_ADD, EPI_GLU = 0, 1, 2
# (name, qtype, N, K, epi, rms input, emits)
SHAPES = [
    ("qkv", GGMLType.Q4_K, 12288, 4096, EPI_STORE, True, False),
    ("o", GGMLType.Q4_K, 4096, 4096, EPI_ADD, False, True),
    ("gate_up", GGMLType.Q4_K, 22016, 4096, EPI_GLU, True, True),
    ("down_q4k", GGMLType.Q4_K, 4096, 11008, EPI_ADD, False, True),
    ("down_q6k", GGMLType.Q6_K, 4096, 11008, EPI_ADD, False, True),
    ("lm_head", GGMLType.Q6_K, 32000, 4096, EPI_STORE, True, False),
]
# OMX_BENCH_BIG=1: the K-split down projections of Llama-2-13B (54 super-blocks) and 70B (112), and 7B's
# padded K (44); OMX_BENCH_GEO=nsb,ks forces the launch geometry of those (gemv8.hip set_gemv8_geo)
BIG = [
    ("down7_q4k", GGMLType.Q4_K, 4096, 11264, EPI_ADD, False, True),
    ("down7_q6k", GGMLType.Q6_K, 4096, 11264, EPI_ADD, False, True),
    ("down13_q4k", GGMLType.Q4_K, 5120, 13824, EPI_ADD, False, True),
    ("down13_q6k", GGMLType.Q6_K, 5120, 13824, EPI_ADD, False, True),
    ("down70_q40", GGMLType.Q4_0, 8192, 28672, EPI_ADD, False, True),
    ("downphi2_q40", GGMLType.Q4_0, 2560, 10240, EPI_ADD, False, True),
]
# OMX_BENCH_ALIGN=1: down-shaped probes at K = 12288 (48 super-blocks: each K group of the 3-way split
# gets exactly 16, piece segments 128-B aligned) vs the real K = 11008 (43: 15 + 15 + 13, 688-B strides)
ALIGN = [
    ("down_q4k_k12288", GGMLType.Q4_K, 4096, 12288, EPI_ADD, False, True),
    ("down_q6k_k12288", GGMLType.Q6_K, 4096, 12288, EPI_ADD, False, True),
    # K = 10240: 40 super-blocks (piece runs 128-B aligned, the last K group 8 of 16 lanes): alignment
    # alone; K = 11264: 44 (64-B aligned runs)
    ("down_q4k_k10240", GGMLType.Q4_K, 4096, 10240, EPI_ADD, False, True),
    ("down_q6k_k10240", GGMLType.Q6_K, 4096, 10240, EPI_ADD, False, True),
    ("down_q6k_k11264", GGMLType.Q6_K, 4096, 11264, EPI_ADD, False, True),
]


def make(qt, N, K, hot):
    rng = np.random.default_rng(0)
    raw = random_blocks(qt, N, K, rng)
    st = repack(raw, qt, N, K)
    copies = 1 if hot else max(2, (768 << 20) // raw.nbytes)
    tups, keep = [], []
    planes = [np.ascontiguousarray(st[n]).view(np.uint8).reshape(-1) for n in STREAMS[qt]]
    offs, tot = [], 0
    for a in planes:
        offs.append(tot)
        tot += (a.size + 255) // 256 * 256
    for _ in range(copies):
        # one buffer per copy, planes at 256-B aligned offsets (the prefetch probe streams the whole copy)
        flat = torch.zeros(tot, dtype=torch.uint8, device="cuda")
        for a, o in zip(planes, offs):
            flat[o: o + a.size].copy_(torch.from_numpy(a))
        p = [flat.data_ptr() + o for o in offs] + [0] * (4 - len(offs))
        tups.append((p[0], p[1], p[2], p[3], N, K, int(qt)))
        keep.append(flat)
    return tups, keep, raw.nbytes


def main():
    C = native()
    hot = bool(os.environ.get("OMX_BENCH_HOT"))
    only = os.environ.get("OMX_BENCH_SHAPES", "").split(",") if os.environ.get("OMX_BENCH_SHAPES") else None
    big = torch.empty(256 << 20, dtype=torch.uint8, device="cuda")
    t0 = time.time()
    while time.time() - t0 < 1.5:  # clock warm-up
        big.add_(1)
    torch.cuda.synchronize()
    del big
    if os.environ.get("OMX_BENCH_BPC"):  # persistent-grid cap per CU: the J (tiles per block) rule of gemv8
        C.set_gemv_tuning(int(os.environ["OMX_BENCH_BPC"]), 1, 0)
    if os.environ.get("OMX_BENCH_GEO"):
        C.set_gemv8_geo(*[int(v) for v in os.environ["OMX_BENCH_GEO"].split(",")])
    shapes = SHAPES + (ALIGN if os.environ.get("OMX_BENCH_ALIGN") else []) + \
        (BIG if os.environ.get("OMX_BENCH_BIG") else [])
    for name, qt, N, K, epi, rms, emits in shapes:
        if only and name not in only:
            continue
        tups, keep, nbytes = make(qt, N, K, hot)
        img = torch.zeros(C.x8_bytes(K), dtype=torch.uint8, device="cuda")
        img[: C.x8_slots(K) * 16] = torch.randint(-100, 100, (C.x8_slots(K) * 16,), dtype=torch.int8,
                                                  device="cuda").view(torch.uint8)
        fl = img[C.x8_slots(K) * 16:].view(torch.float32).view(-1, 2)
        fl[:, 0] = 0.01
        fl[:, 1] = 0.1
        st = torch.rand(K // 16 + 4, device="cuda")
        Ny = N // 2 if epi == EPI_GLU else N
        y = torch.zeros(1, Ny, device="cuda")
        nw = torch.rand(max(N, K), device="cuda") + 0.5
        out = torch.zeros(C.x8_bytes(Ny), dtype=torch.uint8, device="cuda")
        ost = torch.zeros(Ny // 16 + 4, device="cuda")
        # K split across blocks (OMX_GEMV8_KB in the kernel library: 0 auto, 1 off, 2 on): its row partials
        # and self re-arming tile tickets
        kb_ws = torch.zeros(2 * N + 64, device="cuda")
        kb_cnt = torch.zeros((N + 15) // 16, dtype=torch.int32, device="cuda")
        ops = {"x8": img.data_ptr(), "dbg8": int(os.environ.get("OMX_BENCH_DBG8", "0")),
               "kb_ws": kb_ws.data_ptr(), "kb_cnt": kb_cnt.data_ptr()}
        if rms:
            ops["x8_stat"] = st.data_ptr()
        if emits and not os.environ.get("OMX_BENCH_NOEMIT"):  # NOEMIT: the producer without its int8 emission
            ops.update(emit8=out.data_ptr(), emit8_nw=nw.data_ptr())
            if epi == EPI_ADD:
                ops["emit8_stat"] = ost.data_ptr()
        s = torch.cuda.Stream()
        n_launch = 64
        with torch.cuda.stream(s):
            sh = s.cuda_stream
            for i in range(3):  # warm (instantiation, lds attributes)
                C.gemv(tups[i % len(tups)], 1, 0, K, 0, 0, 0, 1e-5, epi, y.data_ptr(), Ny, 0, 0, ops, sh)
            torch.cuda.synchronize()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=s):
                for i in range(n_launch):
                    C.gemv(tups[i % len(tups)], 1, 0, K, 0, 0, 0, 1e-5, epi, y.data_ptr(), Ny, 0, 0, ops, sh)
        for _ in range(3):
            g.replay()
        torch.cuda.synchronize()
        ts = []
        for _ in range(10):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            g.replay()
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1) * 1e3 / n_launch)
        t = float(np.median(ts))
        geo = os.environ.get("OMX_BENCH_GEO")
        kbm = os.environ.get("OMX_GEMV8_KB")
        bpc = os.environ.get("OMX_BENCH_BPC")
        tag = ("hot " if hot else "cold") + (f" geo {geo}" if geo else "") + (f" kb {kbm}" if kbm else "")
        tag += f" bpc {bpc}" if bpc else ""
        tag += (" mem-only" if ops["dbg8"] else "") + (" no-emit" if emits and os.environ.get("OMX_BENCH_NOEMIT") else "")
        print(f"{name:9s} {tag} {t:7.2f} us/launch  {nbytes / t / 1e3:7.1f} GB/s  "
              f"({len(tups)} copies, {nbytes / 1e6:.1f} MB)", flush=True)
        del g, tups, keep


if __name__ == "__main__":
    main()
