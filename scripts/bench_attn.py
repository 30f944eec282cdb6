"""Decode-attention microbenchmark: paged fp16 KV, one query per sequence, per-call latency vs context
length and flash-decode split count. Also times the GEMV fixed cost (tiny N) with / without the fused
RMSNorm prologue and an empty-ish launch, to split per-kernel overhead from bandwidth.
Run on the GPU box:  python scripts/bench_attn.py"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ollama_operator_amd.gguf import GGMLType  # noqa: E402
from ollama_operator_amd.ops import native  # noqa: E402
from ollama_operator_amd.quant import random_blocks, repack  # noqa: E402


def timeit(fn, n=200):
    for _ in range(10):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / n


def timeit_graph(fn, n=50, reps=20):
    """Device time per call: n calls captured in one hipGraph, replayed (no host launch cost)."""
    st = torch.cuda.Stream()
    st.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(st):
        for _ in range(3):
            fn(st.cuda_stream)
    torch.cuda.current_stream().wait_stream(st)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        s = torch.cuda.current_stream().cuda_stream
        for _ in range(n):
            fn(s)
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / (n * reps)


def attn_kps_sweep(C):
    """Graph-timed decode attention vs keys-per-split (the on-device split rule) at serving lengths."""
    bs = 16
    for H, Hkv, D in ((32, 32, 128), (32, 8, 128)):
        for L in (128, 464, 1024, 2048, 4096):
            nblk = (L + bs - 1) // bs
            kc = torch.randn(nblk, Hkv, bs, D, device="cuda").half()
            vc = torch.randn(nblk, Hkv, bs, D, device="cuda").half()
            bt = torch.arange(nblk, device="cuda", dtype=torch.int32)
            qlen = torch.tensor([L], device="cuda", dtype=torch.int32)
            q = torch.randn(1, H * D, device="cuda")
            out = torch.empty(1, H * D, device="cuda")
            S = max(1, min(32, 512 // Hkv))
            ws = torch.empty(max(1, C.attention_ws_floats(1, H, D, S)), device="cuda")
            cnt = torch.zeros(H, device="cuda", dtype=torch.int32)
            row = []
            for kps in (32, 64, 128, 256):
                C.set_attn_tuning(kps)
                fn = lambda st: C.attention(q.data_ptr(), H * D, kc.data_ptr(), vc.data_ptr(), bt.data_ptr(), nblk,  # noqa
                                            0, qlen.data_ptr(), 1, H, Hkv, D, bs, D ** -0.5, 0, out.data_ptr(), H * D,
                                            ws.data_ptr(), S, cnt.data_ptr(), st)
                row.append(f"kps={kps}:{timeit_graph(fn):6.2f}")
            print(f"attn(graph) H={H} Hkv={Hkv} L={L:5d} S<={S}  " + "  ".join(row) + "  (us)", flush=True)
    C.set_attn_tuning(256)


def attn_cold_sweep(C):
    """Graph-timed decode attention with the KV cache rotated over enough copies to miss the 256 MiB
    Infinity Cache (a decode step streams every layer's cache once): keys-per-split x split cap, with the
    in-launch merge (the on-device split rule the runner uses past 1024 keys)."""
    bs = 16
    for H, Hkv, D in ((32, 32, 128), (32, 8, 128)):
        for L in (512, 1024, 2048, 4096, 8192):
            nblk = (L + bs - 1) // bs
            per = nblk * Hkv * bs * D * 2 * 2  # K + V bytes
            copies = max(2, (640 << 20) // per + 1)
            kcs = [torch.randn(nblk, Hkv, bs, D, device="cuda").half() for _ in range(copies)]
            vcs = [torch.randn(nblk, Hkv, bs, D, device="cuda").half() for _ in range(copies)]
            bt = torch.arange(nblk, device="cuda", dtype=torch.int32)
            qlen = torch.tensor([L], device="cuda", dtype=torch.int32)
            q = torch.randn(1, H * D, device="cuda")
            out = torch.empty(1, H * D, device="cuda")
            row = []
            for smax in (16, 32):
                S = max(1, min(smax, 512 // Hkv if smax == 16 else 1024 // Hkv))
                ws = torch.empty(max(1, C.attention_ws_floats(1, H, D, S)), device="cuda")
                cnt = torch.zeros(H, device="cuda", dtype=torch.int32)
                for kps in (64, 128, 256, 512):
                    C.set_attn_tuning(kps)
                    it = [0]

                    def fn(st):
                        i = it[0] % copies
                        it[0] += 1
                        C.attention(q.data_ptr(), H * D, kcs[i].data_ptr(), vcs[i].data_ptr(), bt.data_ptr(), nblk, 0,
                                    qlen.data_ptr(), 1, H, Hkv, D, bs, D ** -0.5, 0, out.data_ptr(), H * D,
                                    ws.data_ptr(), S, cnt.data_ptr(), st)
                    t = timeit_graph(fn, n=2 * copies, reps=10)
                    row.append(f"S<={S},kps={kps}:{t:6.2f}")
            gbs = per / 1e3
            print(f"attn(cold) H={H} Hkv={Hkv} L={L:5d} ({per / 1e6:.1f} MB/layer)  " + "  ".join(row) + "  (us)",
                  flush=True)
            del kcs, vcs
    C.set_attn_tuning(256)


def attn_hpb_sweep(C):
    """Graph-timed decode attention vs query heads per block (GQA group split) and keys per split."""
    bs = 16
    for H, Hkv, D in ((64, 8, 128), (32, 8, 128), (32, 32, 128)):
        for L in (128, 560, 2048):
            nblk = (L + bs - 1) // bs
            kc = torch.randn(nblk, Hkv, bs, D, device="cuda").half()
            vc = torch.randn(nblk, Hkv, bs, D, device="cuda").half()
            bt = torch.arange(nblk, device="cuda", dtype=torch.int32)
            qlen = torch.tensor([L], device="cuda", dtype=torch.int32)
            q = torch.randn(1, H * D, device="cuda")
            out = torch.empty(1, H * D, device="cuda")
            S = max(1, min(32, 512 // Hkv))
            ws = torch.empty(max(1, C.attention_ws_floats(1, H, D, S)), device="cuda")
            cnt = torch.zeros(H, device="cuda", dtype=torch.int32)
            ref = None
            for hpb in sorted({1, 2, 4, 8, H // Hkv}):
                if hpb > H // Hkv:
                    continue
                row = []
                for kps in (64, 128, 256):
                    C.set_attn_tuning(kps, hpb)
                    fn = lambda st: C.attention(q.data_ptr(), H * D, kc.data_ptr(), vc.data_ptr(), bt.data_ptr(), nblk,  # noqa
                                                0, qlen.data_ptr(), 1, H, Hkv, D, bs, D ** -0.5, 0, out.data_ptr(), H * D,
                                                ws.data_ptr(), S, cnt.data_ptr(), st)
                    row.append(f"kps={kps}:{timeit_graph(fn):6.2f}")
                    torch.cuda.synchronize()
                    if ref is None:
                        ref = out.clone()
                    err = float((out - ref).abs().max())
                    assert err < 1e-3, (H, Hkv, L, hpb, kps, err)
                print(f"attn(graph) H={H} Hkv={Hkv} L={L:5d} hpb={hpb}  " + "  ".join(row) + "  (us)", flush=True)
    C.set_attn_tuning(256, 0)


def attn_sweep(C, s):
    bs = 16
    for H, Hkv, D in ((32, 32, 128), (32, 8, 128)):
        for L in (64, 200, 512, 1024, 4096):
            nblk = (L + bs - 1) // bs
            kc = torch.randn(nblk, Hkv, bs, D, device="cuda").half()
            vc = torch.randn(nblk, Hkv, bs, D, device="cuda").half()
            bt = torch.arange(nblk, device="cuda", dtype=torch.int32)
            qlen = torch.tensor([L], device="cuda", dtype=torch.int32)
            q = torch.randn(1, H * D, device="cuda")
            out = torch.empty(1, H * D, device="cuda")
            row = []
            for S in (1, 2, 4, 8, 16, 32):
                ws = torch.empty(max(1, C.attention_ws_floats(1, H, D, S)), device="cuda")
                cnt = torch.zeros(H, device="cuda", dtype=torch.int32)
                fn = lambda: C.attention(q.data_ptr(), H * D, kc.data_ptr(), vc.data_ptr(), bt.data_ptr(), nblk,  # noqa
                                         0, qlen.data_ptr(), 1, H, Hkv, D, bs, D ** -0.5, 0, out.data_ptr(), H * D,
                                         ws.data_ptr(), S, cnt.data_ptr(), s)
                row.append(f"S={S}:{timeit(fn):6.2f}")
            print(f"attn H={H} Hkv={Hkv} D={D} L={L:5d}  " + "  ".join(row) + "  (us)", flush=True)


def gemv_fixed(C, s):
    rng = np.random.default_rng(0)
    K = 4096
    for N in (64, 1024, 4096):
        raw = random_blocks(GGMLType.Q4_K, N, K, rng)
        st = repack(raw, GGMLType.Q4_K, N, K)
        ts = [torch.from_numpy(np.ascontiguousarray(st[n])).cuda() for n in ("qs", "meta")]
        tup = (ts[0].data_ptr(), ts[1].data_ptr(), 0, 0, N, K, int(GGMLType.Q4_K))
        x = torch.randn(1, K, device="cuda")
        nw = torch.ones(K, device="cuda")
        y = torch.zeros(1, N, device="cuda")
        for norm in (0, 1):
            fn = lambda: C.gemv(tup, 1, x.data_ptr(), K, norm, nw.data_ptr(), 0, 1e-5, 0, y.data_ptr(), N, 0, 0, {}, s)  # noqa
            print(f"gemv Q4_K N={N:5d} K={K} norm={norm}: {timeit(fn):6.2f} us (MALL-resident weights)", flush=True)
    a = torch.zeros(256, device="cuda")
    b = torch.zeros(256, device="cuda")
    print(f"add_inplace 256 floats (launch floor): {timeit(lambda: C.add_inplace(a.data_ptr(), b.data_ptr(), 256, s)):6.2f} us")


def main():
    C = native()
    s = torch.cuda.current_stream().cuda_stream
    if os.environ.get("OMX_BENCH_HPB"):
        attn_hpb_sweep(C)
        return
    if os.environ.get("OMX_BENCH_KPS"):
        attn_kps_sweep(C)
        return
    if os.environ.get("OMX_BENCH_COLD"):
        attn_cold_sweep(C)
        return
    gemv_fixed(C, s)
    attn_sweep(C, s)


if __name__ == "__main__":
    main()
