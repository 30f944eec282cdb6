"""Model runner: weights + paged KV cache + step buffers + executor + sampler + hipGraph decode.

One `Runner` serves one model on one device (one TP rank). The executor is the native gfx950 one
(`_C.Executor`, csrc/runtime/executor.cpp) on a GPU and the torch twin (`ops.reference`) on CPU;
both read the same buffers, so prefill/decode/batching logic is shared and tested on CPU.

Decode is captured once per batch size into a hipGraph (torch.cuda.CUDAGraph): forward over all
layers + on-device sampling + feeding the sampled token back as the next input. The host only
uploads (pos, slot, q_len) for the next step from a pinned ring and reads the sampled token one
step behind, so the GPU never waits on Python.
"""
from __future__ import annotations

import ctypes
import gc
import os
import time
import weakref
from dataclasses import dataclass
from typing import Callable, Iterator

import numpy as np
import torch

from ..models.config import cache_head_dim
from ..ops import native, stream_handle
from ..ops.reference import TorchExecutor
from ..utils.trace import trace_range
from .kv_cache import PagedKV
from .sampling import SamplingOptions, sample_host
from .weights import DeviceWeights, DevQMat

HIST_CAP = 256
GEMM_SPLIT_WS_FLOATS = 32 << 20  # 128 MiB of fp32 split-K slabs (2-way split of a 2048 x 8192 output)


class NativeExec:
    """Adapter: runner buffers -> a native executor: `_C.Executor` (gfx950 kernels, GPU runner) or
    `_cpu.Executor` (the CPU serving backend, csrc/cpu; same call surface)."""

    def __init__(self, runner: "Runner", module=None):
        C = module if module is not None else native()
        self.on_gpu = module is None
        r = runner
        w, loc, cfg = r.w, r.w.local, r.w.cfg
        self.r = r
        self.exe = e = C.Executor()
        e.configure(dict(arch=1 if cfg.arch == "phi2" else 0, E=loc["E"], H=loc["H"], Hkv=loc["Hkv"], D=loc["D"], Dc=r.Dc,
                         n_rot=cfg.n_rot, F=loc["F"], n_layer=cfg.n_layer, V=loc["V"], eps=float(cfg.norm_eps),
                         n_expert=cfg.n_expert, n_expert_used=cfg.n_expert_used, window=cfg.sliding_window,
                         tp=r.tp_size, embed_scale=float(cfg.embed_scale), glu_act=int(cfg.gelu_glu),
                         kv8=int(getattr(r, "kv8", False)), F_valid=loc["F"] - getattr(w, "ffn_pad", 0)))
        p = lambda t: t.data_ptr() if t is not None else 0  # noqa: E731
        e.set_globals(w.tok_embd.tup, p(w.out_norm), p(w.out_norm_b), w.lm_head.tup, p(w.lm_bias), p(w.inv_freq))
        if getattr(w, "lm_c1", None) is not None and self.on_gpu:  # phi2 int8 chain (executor.cpp ln8)
            e.set_head_ln(p(w.lm_c1), p(w.lm_c2))
        for i, L in enumerate(w.layers):
            d = {}
            for k, v in L.items():
                if v is None:
                    continue
                d[k] = v.tup if hasattr(v, "tup") else v.data_ptr()
            d["kc"] = r.kc[i].data_ptr()
            d["vc"] = r.vc[i].data_ptr()
            e.set_layer(i, d)
        e.set_workspace(dict(resid=p(r.resid), qbuf=p(r.qbuf), abuf=p(r.abuf), hbuf=p(r.hbuf), ypart=p(r.ypart),
                             lbuf=p(r.lbuf), rlogits=p(r.rlogits), eids=p(r.eids), ew=p(r.ew),
                             attn_ws=p(r.attn_ws), attn_cnt=p(r.attn_cnt), x16=p(r.x16), x16_elems=r.x16.numel(),
                             gws=p(r.gws),
                             moe_rows=p(r.moe_rows) if cfg.n_expert else 0, moe_tiles=p(r.moe_tiles),
                             moe_ntiles=p(r.moe_ntiles),
                             gws_elems=r.gws.numel(), max_B=r.max_batch, ld_logits=r.logits.shape[1],
                             ext=p(r.ext), w16=p(r.w16), w16_elems=r.w16.numel() if r.w16 is not None else 0,
                             yws=p(r.yws), yws_elems=r.yws.numel() if r.yws is not None else 0,
                             n_splits=1, **self._chain_ws(r), **self._x8_ws(r)))
        # step buffers bound once: every stage call below passes integers only
        e.set_inputs(dict(tokens=p(r.d_tokens), pos=p(r.d_pos), slot=p(r.d_slot), q_len=p(r.d_qlen),
                          q_seq=p(r.d_qseq), block_table=p(r.d_block_table), max_blocks=r.max_blocks,
                          bs=r.block_size, logits=p(r.logits), logit_idx=p(r.d_logit_idx),
                          full_logits=p(r.full_logits), ld_full=r.full_logits.shape[1]))
        if r.ar is not None:
            e.set_ar(r.ar.params)
        self.stages = dict(forward=C.ST_FORWARD, embed=C.ST_EMBED, attn=C.ST_ATTN, ffn=C.ST_FFN, head=C.ST_HEAD,
                           forward_tp=C.ST_FORWARD_TP)

    @staticmethod
    def _chain_ws(r) -> dict:
        """The fp16 matrix-core decode chain buffers (the executor enables the chain only when every
        projection takes the matrix-core kernel: Executor::chain_capable)."""
        mb = getattr(r, "mb_bufs", None)
        if not mb:
            return {}
        d = {k: v.data_ptr() for k, v in mb.items()}
        d.update(mb_ok=1, ld_e=mb["xa16"].shape[1], ld_f=mb["h16"].shape[1], ld_q=mb["a16"].shape[1])
        return d

    @staticmethod
    def _x8_ws(r) -> dict:
        """The batch-1 int8 activation chain buffers (gemv8.hip; the executor turns the chain on only
        when every emitter is covered: Executor::x8_capable)."""
        b = getattr(r, "x8_bufs", None)
        if not b:
            return {}
        return dict(x8e=b["x8e"].data_ptr(), x8f=b["x8f"].data_ptr(), x8st=b["x8st"].data_ptr(), x8_ok=1,
                    x8sum=b["x8sum"].data_ptr(), x8kb=b["x8kb"].data_ptr(), x8cnt=b["x8cnt"].data_ptr(),
                    # batch rows on the chain: B = 2 measured 1.73 vs 2.08 ms per step on the int8 rows, B = 3
                    # 2.15 vs 2.19 ms; at 4 rows layout M's MFMA GEMVs win (profiles/r4_batch), so 3 by default
                    x8_bmax=int(os.environ.get("OMX_X8_BATCH", "3")))

    def ar_fits(self, B: int) -> bool:
        return self.exe.ar_fits(B)

    def run(self, stage: str, layer: int, B: int, n_logits: int = 0, use_idx: bool = False,
            prefill: bool = False):
        S, defer = self.r.split_plan(B)
        self.exe.set_splits(S, defer)
        self.exe.step(self.stages[stage], layer, B, n_logits, use_idx, prefill, stream_handle() if self.on_gpu else 0)


def kv_cache_type() -> str:
    """GPU KV cache element type from OMX_KV_CACHE_TYPE / OLLAMA_KV_CACHE_TYPE: "fp8" (e4m3; also for
    Ollama's "q8_0", the 8-bit setting) or "f16" (default; "q4_0" falls back to it)."""
    v = (os.environ.get("OMX_KV_CACHE_TYPE") or os.environ.get("OLLAMA_KV_CACHE_TYPE") or "f16").strip().lower()
    return "fp8" if v in ("fp8", "e4m3", "q8_0") else "f16"


@dataclass
class StepTimes:
    prompt_tokens: int = 0
    prompt_s: float = 0.0
    gen_tokens: int = 0
    gen_s: float = 0.0
    load_s: float = 0.0


class Runner:
    def __init__(self, model_path: str, device: str | None = None, max_batch: int = 64, max_seqs: int = 4,
                 ctx: int | None = None, block_size: int = 16, tp_rank: int = 0, tp_size: int = 1,
                 tp_group=None, use_graphs: bool | None = None, weights: DeviceWeights | None = None,
                 tp_ctrl=None, cpu_backend: str | None = None, ext_rows: int = 0):
        """cpu_backend (device "cpu" only): "native" = the quantised C++ backend (csrc/cpu, the serving
        default), "torch" = the fp32 torch twin (test oracle). Default: $OMX_CPU_BACKEND, else native
        when its module is built. ext_rows: capacity of the external embedding rows (image patches of
        multimodal prompts, `set_ext`); 0 = text only."""
        t0 = time.perf_counter()
        if device is None:
            device = f"cuda:{torch.cuda.current_device()}" if torch.cuda.is_available() else "cpu"
        self.device = torch.device(device)
        self.is_gpu = self.device.type == "cuda"
        if self.is_gpu:
            native()  # fail loudly: no silent torch fallback on a GPU box
            if os.environ.get("OMX_GEMV_XFIRST") in ("0", "1"):  # decode GEMV x-first knob (gemv.hip)
                native().set_gemv_tuning(xfirst=int(os.environ["OMX_GEMV_XFIRST"]))
            if os.environ.get("OMX_GEMV_XBAR") in ("0", "1"):  # x-barrier one-block-per-CU decode GEMVs
                native().set_gemv_tuning(xbar=int(os.environ["OMX_GEMV_XBAR"]))
        self.tp_rank, self.tp_size, self.tp_group = tp_rank, tp_size, tp_group
        self._closed = False
        # TP serving (parallel/tp.py): rank 0 signals each decode step, followers mirror it
        self.tp_ctrl = tp_ctrl
        self.w = weights or DeviceWeights(model_path, self.device, tp_rank, tp_size)
        # continuous batching on the matrix cores (gemv_mfma.hip): layout M weight copies, built on the
        # device, whenever this runner can batch sequences (OMX_MFMA_BATCH=0 keeps the int8 GEMV only).
        # Reading the resident v2 streams directly instead measured 2x slower at B = 4 (16-B row runs per
        # load instruction: experiments/kernels/gemv_mfma_v2_piece_per_wave.hip, profiles/r4_batch)
        self.mfma_bytes = 0
        if self.is_gpu and max_seqs > 1 and os.environ.get("OMX_MFMA_BATCH", "1") != "0":
            self.mfma_bytes = self.w.build_mfma_layouts()
        # rows from which prefill chunks take hipBLASLt (gemm.hip gemm_lib_min_m; default 0 = never: every
        # prefill GEMM runs the hand-written dequant kernel over the resident quantised weights, and no fp16
        # weight copy exists -- OMX_GEMM_LIB_MIN_M=<rows> is the A/B knob)
        self.lib_min = native().gemm_lib_min_m() if self.is_gpu else 0
        # MoE prefill: (token, expert) pairs from which each expert's GEMM runs on hipBLASLt over its
        # per-call dequantised weights (gemm.hip moe_gemm_lib; default 256, OMX_MOE_LIB_MIN_M)
        self.moe_lib = native().moe_lib_min_m() if self.is_gpu and self.w.cfg.n_expert else 0
        cfg = self.cfg = self.w.cfg
        loc = self.w.local
        self.max_batch = max_batch
        self.max_seqs = max_seqs
        self.block_size = block_size
        self.ctx = min(ctx or cfg.ctx_len, cfg.ctx_len)
        self.max_blocks = (self.ctx + block_size - 1) // block_size
        n_blocks = max_seqs * self.max_blocks
        dev = self.device
        f32 = dict(device=dev, dtype=torch.float32)
        i32 = dict(device=dev, dtype=torch.int32)
        E, Eq, Fl, Vl = loc["E"], loc["H"] * loc["D"], loc["F"], loc["V"]
        ksel = max(1, cfg.n_expert_used)
        # CPU: the cache stays untouched (and out of RSS) until blocks are written -- every slot is
        # written by its QKV step before any attention reads it
        kv_alloc = torch.zeros if self.is_gpu else torch.empty
        # GPU cache rows are as wide as an attention kernel's head dim (Orca Mini's 100 -> 112, zero pad);
        # the CPU backends keep the model's head dim
        self.Dc = cache_head_dim(loc["D"]) if self.is_gpu else loc["D"]
        # KV cache element type: fp16 (Ollama's default f16) or, on the GPU, fp8 e4m3 (OCP e4m3fn, half the
        # bytes every decode step streams: OMX_KV_CACHE_TYPE=fp8, or Ollama's OLLAMA_KV_CACHE_TYPE=q8_0,
        # served by this 8-bit format instead of q8_0 blocks)
        self.kv_type = kv_cache_type() if self.is_gpu else "f16"
        self.kv8 = self.kv_type == "fp8"
        kv_dt = torch.uint8 if self.kv8 else torch.float16
        self.kc = [kv_alloc(n_blocks, loc["Hkv"], block_size, self.Dc, device=dev, dtype=kv_dt)
                   for _ in range(cfg.n_layer)]
        self.vc = [kv_alloc(n_blocks, loc["Hkv"], block_size, self.Dc, device=dev, dtype=kv_dt)
                   for _ in range(cfg.n_layer)]
        self.resid = torch.zeros(max_batch, E, **f32)
        self.qbuf = torch.zeros(max_batch, Eq, **f32)
        self.abuf = torch.zeros(max_batch, Eq, **f32)
        self.hbuf = torch.zeros(max_batch, ksel * Fl, **f32)
        self.ypart = torch.zeros(max_batch, E, **f32)
        self.lbuf = torch.zeros(max_batch, E, **f32)
        self.rlogits = torch.zeros(max_batch, max(1, cfg.n_expert), **f32)
        self.eids = torch.zeros(max_batch, ksel, **i32)
        self.ew = torch.zeros(max_batch, ksel, **f32)
        # fp16 activations for the prefill MFMA GEMM (any GEMM input: E, H*D, F, k*F wide)
        self.x16 = torch.zeros(max_batch * max(E, Eq, ksel * Fl, ksel * E), device=dev, dtype=torch.float16)
        # batched decode chain on the matrix cores (executor.cpp chain(): 2 <= B <= 16): fp16 activation
        # rows [17][ld] (row 16 stays zero) + RMS sum-of-squares partial slabs
        self.mb_bufs = None
        if self.mfma_bytes:
            r256 = lambda n: (n + 255) // 256 * 256  # noqa: E731
            h16 = dict(device=dev, dtype=torch.float16)
            self.mb_bufs = dict(xa16=torch.zeros(17, r256(E), **h16), h16=torch.zeros(17, r256(Fl), **h16),
                                a16=torch.zeros(17, r256(Eq), **h16), st0=torch.zeros((E + 15) // 16 * 16 + 32, **f32),
                                st1=torch.zeros((E + 15) // 16 * 16 + 32, **f32))
        # batch-1 int8 activation chain (csrc/kernels/gemv8.hip): zeroed images (pad slots stay zero)
        self.x8_bufs = None
        if self.is_gpu and os.environ.get("OMX_X8", "1") != "0":
            C = native()
            u8 = dict(device=dev, dtype=torch.uint8)
            nb = 4  # batch rows of the chain (gemv8.hip X8_MAX_B): row b's image at b * x8_bytes
            self.x8_bufs = dict(x8e=torch.zeros(nb * C.x8_bytes(E), **u8), x8f=torch.zeros(nb * C.x8_bytes(Fl), **u8),
                                x8st=torch.zeros(nb * C.x8_stat_ld(E) + 4, **f32),
                                x8sum=torch.zeros(nb * C.x8_stat_ld(E) + 4, **f32),  # phi2: LayerNorm means
                                # gemv8 K split across blocks: row partials [N][2], tile tickets (self re-arming)
                                x8kb=torch.zeros(2 * 65536, **f32), x8cnt=torch.zeros(8192, **i32))
        # MoE prefill grouping (csrc/kernels/moe.hip moe_sort -> grouped MFMA GEMM)
        n_pairs = max_batch * ksel
        self.moe_rows = torch.zeros(n_pairs, **i32)
        self.moe_tiles = torch.zeros(3 * (n_pairs // 128 + max(1, cfg.n_expert) + 1), **i32)
        self.moe_ntiles = torch.zeros(1, **i32)
        # external embedding rows (multimodal prompts): token id t < 0 maps through _ext_map to a row of
        # self.ext, which the embed stage copies instead of a token embedding (models/clip.py)
        self.ext = torch.zeros(ext_rows, E, **f32) if ext_rows > 0 else None
        self._ext_map: dict[int, int] = {}
        self._ext_next = 0
        # split-K partial slabs of small-M prefill GEMMs (the kernel picks splits that fit)
        self.gws = torch.zeros(GEMM_SPLIT_WS_FLOATS if str(dev).startswith("cuda") else 1, **f32)
        # hipBLASLt prefill (gemm.hip gemm_lib) for chunks of >= gemm_lib_min_m() rows (default 2048;
        # OMX_GEMM_LIB_MIN_M, 0 = never): fp16 dequantised-weight scratch sized for the largest dense
        # layer matrix and its fp32 output slab at max_batch rows
        self.w16 = self.yws = None
        dense_lib = self.lib_min > 0 and max_batch >= max(16, self.lib_min)
        moe_lib = self.moe_lib > 0 and max_batch * ksel >= self.moe_lib
        if self.is_gpu and (dense_lib or moe_lib):
            # expert stacks count per expert (DevQMat.N = rows of one expert): moe_gemm_lib
            mats = [v for L in self.w.layers for k, v in L.items() if isinstance(v, DevQMat) and k != "router"
                    and (dense_lib or k in ("gu_exps", "down_exps"))]
            if mats:
                self.w16 = torch.empty(max(m.N * m.K for m in mats), device=dev, dtype=torch.float16)
                self.yws = torch.empty(max_batch * (ksel if moe_lib else 1) * max(m.N for m in mats), **f32)
        ws = max(self._ws_floats(B) for B in range(1, max_batch + 1))
        self.attn_ws = torch.zeros(max(ws, 1), **f32)
        self.attn_cnt = torch.zeros(max_batch * loc["H"], **i32)  # self re-arming tickets
        self.logits = torch.zeros(max_batch, Vl, **f32)
        self.full_logits = torch.zeros(max_batch, cfg.n_vocab, **f32) if tp_size > 1 else self.logits
        # step inputs, packed so one H2D copy refreshes (pos, slot, q_len, q_seq, logit_idx)
        self.d_step = torch.zeros(6, max_batch, **i32)
        self.d_pos, self.d_slot, self.d_qlen, self.d_qseq, self.d_logit_idx, self.d_tokens = self.d_step.unbind(0)
        self.d_block_table = torch.zeros(max_seqs, self.max_blocks, **i32)
        # sampler state (indexed by batch row)
        self.s_temp = torch.zeros(max_batch, **f32)
        self.s_topk = torch.zeros(max_batch, **i32)
        self.s_topp = torch.ones(max_batch, **f32)
        self.s_minp = torch.zeros(max_batch, **f32)
        self.s_rpen = torch.ones(max_batch, **f32)
        self.s_ppen = torch.zeros(max_batch, **f32)
        self.s_fpen = torch.zeros(max_batch, **f32)
        self.s_lastn = torch.zeros(max_batch, **i32)
        self.s_seed = torch.zeros(max_batch, device=dev, dtype=torch.int64)
        self.s_step = torch.zeros(max_batch, **i32)
        self.s_hist = torch.zeros(max_batch, HIST_CAP, **i32)
        self.s_hcount = torch.zeros(max_batch, **i32)
        self.s_out = torch.zeros(max_batch, **i32)
        # multi-block sampler: per-row candidate lists (ceil(V/1024) blocks x 64 x {value, index})
        # and hand-off tickets (zeroed once; the kernel re-arms them)
        self.s_ws = torch.zeros(max_batch, -(-cfg.n_vocab // 1024) * 128, **f32)
        self.s_tickets = torch.zeros(max_batch, **i32)
        # sampler error word: a row whose logits were non-finite (its id is clamped to 0 on device)
        self.s_err = torch.zeros(1, **i32)
        self.kv = PagedKV(n_blocks, block_size, max_seqs, self.max_blocks)
        # deferred flash-decode merge (B == 1): attention leaves S <= 8 partial slabs, the O GEMV
        # merges them in its activation prologue (no in-launch ticket + re-read)
        self.defer_kps = int(os.environ.get("OMX_DEFER_KPS", "128"))
        # batch-1 generation: decode steps per graph replay (1 = one token per replay)
        # (default 1: with the sampler's host-ring fence in every step, 4-step graphs measured 1.3 % slower;
        # without it 0.5 % faster (profiles/r6_decode/group_ab_nofence.log) -- not worth streaming tokens
        # in bursts and computing up to k - 1 steps past a stop)
        self.decode_group = max(1, int(os.environ.get("OMX_DECODE_GROUP", "1")))
        # OMX_GRAPH_PAIR=1 (A/B knob): batch-1 decode alternates between two captured instances of each
        # step graph, so a replay never re-launches the executable the previous replay is still running
        self.graph_pair = os.environ.get("OMX_GRAPH_PAIR", "0") == "1"
        # system-scope fence after the sampler's host-ring store: off by default (OMX_RING_FENCE=1 restores
        # it). The host reads a ring slot only after that step's event, whose completion is itself a
        # system-scope release of every earlier write; the fence inside the graph cost 707 -> 724 tok/s on
        # the 256-step headline (profiles/r6_decode/ring_fence)
        self.ring_fence = 1 if os.environ.get("OMX_RING_FENCE", "0") == "1" else 0
        self.steps_issued = 0  # decode steps enqueued so far (batched steps count once): bench timing
        # past 8 x defer_kps keys, up to 8 x 512: 8 deferred splits of ceil(len / 8) keys (OMX_DEFER_LONG=1,
        # default: attention 14.4 -> 11.6 us at 2k keys, the O prologue's 8-slab merge 4.9 -> 7.1 us, net
        # decode_ctx2048 593 -> 602 tok/s, profiles/r5_decode) or the on-device split rule with the
        # in-launch ticket merge (0; always past 4096 keys)
        self.defer_long = os.environ.get("OMX_DEFER_LONG", "1") != "0"
        self.defer_max_s = int(os.environ.get("OMX_DEFER_MAX_S", "8"))  # 2, 4 or 8 deferred splits at most
        # past 8 x defer_kps keys and up to this length: 4 deferred splits instead of 8 (default 0 = never).
        # The chain probe (profiles/r6_attn/attn_probe*.log) timed S = 4 1.1 us per layer ahead at 2048
        # keys, but in the model it measured equal at 2.2k keys and 3 % behind at 2.6-2.9k
        # (experiments/ab/defer_s4.py, profiles/r6_attn/defer_s4_ab.log)
        self.defer_s4_max = int(os.environ.get("OMX_DEFER_S4_MAX", "0"))
        # the O GEMV merges the slabs: gemv.hip for K <= 4096; the int8-chain GEMV up to K = 8192 (13B / 70B)
        # only with OMX_DEFER_KSPLIT=1 -- measured 343 vs 341 tok/s for 13B at short context but 273 vs 297
        # at 2k keys, and no gain for 70B (profiles/r6_models/defer_ksplit); checked again once the executor
        # reports the chain on, below
        ksplit = os.environ.get("OMX_DEFER_KSPLIT", "0") == "1"
        self._defer_ok = (self.is_gpu and os.environ.get("OMX_DEFER_MERGE", "1") != "0" and self.n_splits(1) >= 8 and
                          (native().gemv_merge_supported(1, Eq, loc["D"], 8) or
                           (ksplit and tp_size == 1 and native().gemv8_merge_supported(Eq, loc["D"], 8))))
        self._decode_S = 0
        self._adv_next = None  # (sid, pos) the device step inputs were advanced to by the last decode
        # TP decode collectives: one-shot all-reduce over peer-mapped slabs (parallel/custom_ar.py),
        # decode-size messages only (<= ~1 MB); prefill chunks keep RCCL
        self.ar = None
        if self.is_gpu and tp_size > 1 and os.environ.get("OMX_CUSTOM_AR", "1") != "0":
            from ..parallel.custom_ar import CustomAllReduce
            rows = max(1, min(max_batch, max(max_seqs, 16), (1 << 18) // max(E, Vl)))
            self.ar = CustomAllReduce(tp_group, tp_rank, tp_size, rows * max(E, Vl))
        if self.is_gpu:
            self.exe = NativeExec(self)
            if self._defer_ok and not native().gemv_merge_supported(1, Eq, loc["D"], 8) and not self.exe.exe.x8_on:
                self._defer_ok = False  # K > 4096 merges only on the int8 chain
        else:
            from ..ops.cpu import cpu_module
            choice = cpu_backend or os.environ.get("OMX_CPU_BACKEND") or ("native" if cpu_module() else "torch")
            if choice == "native":
                mod = cpu_module()
                if mod is None:
                    raise RuntimeError("CPU backend ollama_operator_amd._cpu is not built (python build_native.py)")
                self.exe = NativeExec(self, mod)
            else:
                self.exe = TorchExecutor(self)
        self.cpu_backend = None if self.is_gpu else ("native" if isinstance(self.exe, NativeExec) else "torch")
        if use_graphs is None:  # TP: graph-captured only through the custom all-reduce
            use_graphs = (self.is_gpu and (tp_size == 1 or self.ar is not None) and
                          os.environ.get("OMX_NO_GRAPH", "0") != "1")
        self.use_graphs = use_graphs
        self.graphs: dict[int, torch.cuda.CUDAGraph] = {}
        self._host_sampler: dict[int, tuple] = {}
        self._pinned = None
        if self.is_gpu:
            self._pinned = [torch.zeros(5, max_batch, dtype=torch.int32).pin_memory() for _ in range(4)]
            self._pin_i = 0
            self._tok_host = torch.zeros(max_batch, dtype=torch.int32).pin_memory()
            # sampled tokens of the B == 1 steps, written by the feedback kernel straight into host-mapped
            # pinned memory (slot = input position % ring): no D2H copy command per step
            self._ring_n = 32  # > the steps in flight: two groups of decode_group steps (generate)
            h, d = native().host_alloc_mapped(4 * self._ring_n)
            self._host_ring_dev = d
            self._host_ring = np.ctypeslib.as_array((ctypes.c_int32 * self._ring_n).from_address(h))
            weakref.finalize(self, native().host_free_mapped, h)
        self.load_s = time.perf_counter() - t0

    def close(self) -> None:
        """Release the TP collective workspace (all ranks call this together). The executor forgets
        the slabs and the captured graphs (which point at them) go first, so no later step can write
        into freed memory; a closed runner refuses further steps.

        Then everything else goes with it: the graphs, the Runner <-> NativeExec reference cycle and the
        device tensors. warmup() froze the objects alive after load (gc.freeze), and a frozen cycle is
        never collected, so without this every unload (keep-alive expiry, eviction, reload) would keep
        the model's weights, KV cache and graphs resident on the GPU."""
        if self._closed:
            return
        if self.ar is not None:
            if isinstance(self.exe, NativeExec):
                self.exe.exe.clear_ar()
            self.graphs.clear()
            self.ar.close()
            self.ar = None
        self._closed = True
        self.graphs.clear()
        ex, self.exe = self.exe, None
        if isinstance(ex, NativeExec):
            ex.r = None
            ex.exe = None
        for k, v in list(vars(self).items()):  # device buffers and weights: dropped now, not at collection
            if isinstance(v, (torch.Tensor, list, dict, DeviceWeights)) and k not in ("graphs",):
                setattr(self, k, None)
        if self.is_gpu:
            torch.cuda.synchronize(self.device)
        refreeze = gc.get_freeze_count() > 0
        gc.unfreeze()
        gc.collect()
        if refreeze:  # the other loaded models stay out of the collector's way
            gc.freeze()
        if self.is_gpu:
            torch.cuda.empty_cache()

    # ------------------------------------------------------------------ sizing helpers
    def n_splits(self, B: int) -> int:
        hkv = self.w.local["Hkv"]
        return max(1, min(32, 512 // max(1, B * hkv)))

    def split_plan(self, B: int) -> tuple[int, int]:
        """(splits, deferred) for the next launch sequence. B == 1 decode uses the length bucket set
        by `decode_step` (`_decode_S`): S partial slabs merged in the O GEMV prologue; everything
        else keeps the on-device split rule with the in-launch merge."""
        S = self._decode_S if B == 1 else 0
        if S:
            return S, int(S > 1)
        return self.n_splits(B), 0

    def decode_splits(self, length: int) -> int:
        """Flash-decode split bucket for a B == 1 step over `length` visible keys: 1 / 2 / 4 / 8
        deferred splits of >= DEFER_KPS keys, 0 (= on-device rule, in-launch merge) beyond."""
        if not self._defer_ok:
            return 0
        S = 1
        while S < self.defer_max_s and length > S * self.defer_kps:
            S *= 2
        if S == 8 and self.defer_long and 8 * self.defer_kps < length <= self.defer_s4_max:
            S = 4
        return S if length <= S * self.defer_kps or (self.defer_long and length <= 8 * 512) else 0

    def _ws_floats(self, B: int) -> int:
        loc = self.w.local
        S = self.n_splits(B)
        return B * loc["H"] * S * (self.Dc + 2) if S > 1 else 0

    # ------------------------------------------------------------------ forward
    def _all_reduce_add(self, B: int):
        import torch.distributed as dist
        with trace_range("tp all_reduce"):
            dist.all_reduce(self.ypart[:B], group=self.tp_group)
        self.resid[:B] += self.ypart[:B]

    def forward(self, B: int, n_logits: int, use_idx: bool = False, prefill: bool = False):
        """prefill=True: the B rows are one sequence's contiguous positions (MFMA flash attention)."""
        if self._closed:
            raise RuntimeError("runner is closed")
        if self.tp_size == 1:
            self.exe.run("forward", 0, B, n_logits, use_idx, prefill)
            return
        if self.ar is not None and self.exe.ar_fits(B):  # whole TP step in one native call
            self.exe.run("forward_tp", 0, B, n_logits, use_idx, prefill)
            return
        import torch.distributed as dist
        self.exe.run("embed", 0, B)
        for i in range(self.cfg.n_layer):
            self.exe.run("attn", i, B, prefill=prefill)
            self._all_reduce_add(B)
            self.exe.run("ffn", i, B)
            self._all_reduce_add(B)
        self.exe.run("head", 0, B, n_logits, use_idx)
        if n_logits:
            parts = [torch.empty_like(self.logits[:n_logits]) for _ in range(self.tp_size)]
            dist.all_gather(parts, self.logits[:n_logits].contiguous(), group=self.tp_group)
            self.full_logits[:n_logits] = torch.cat(parts, dim=1)

    # ------------------------------------------------------------------ inputs
    def _upload(self, arr: np.ndarray, tokens: np.ndarray | None):
        """arr: int32 [5, B] = (pos, slot, qlen, qseq, logit_idx)."""
        B = arr.shape[1]
        self._adv_next = None  # device step inputs no longer follow the last B == 1 decode
        if self.is_gpu:
            buf = self._pinned[self._pin_i]
            self._pin_i = (self._pin_i + 1) % len(self._pinned)
            buf[:, :B] = torch.from_numpy(arr)
            self.d_step[:5, :B].copy_(buf[:, :B], non_blocking=True)
            if tokens is not None:
                self.d_tokens[:len(tokens)].copy_(torch.from_numpy(tokens.astype(np.int32)), non_blocking=False)
        else:
            self.d_step[:5, :B] = torch.from_numpy(arr)
            if tokens is not None:
                self.d_tokens[:len(tokens)] = torch.from_numpy(tokens.astype(np.int32))

    def _sync_block_table(self, sid: int):
        self._adv_next = None
        s = self.kv.seqs[sid]
        row = torch.tensor(s.blocks, dtype=torch.int32)
        self.d_block_table[s.row, :len(s.blocks)].copy_(row.to(self.device))

    # ------------------------------------------------------------------ sequences
    def new_sequence(self) -> int:
        self._adv_next = None
        return self.kv.new_seq()

    def free_sequence(self, sid: int) -> None:
        self._adv_next = None
        self.kv.free_seq(sid)

    def set_ext(self, ids: list[int], rows) -> None:
        """Register external embedding rows (e.g. an image's projected patches) under negative token
        ids; prompts then carry those ids where the rows belong. Rows are kept in a ring of ext_rows
        (an id already registered keeps its row), so ids of requests still waiting for their prefill
        stay valid while the ring holds them."""
        if self.ext is None:
            raise ValueError("this runner has no external embedding rows (ext_rows=0)")
        rows = torch.as_tensor(np.asarray(rows, np.float32) if not isinstance(rows, torch.Tensor) else rows)
        if rows.dim() != 2 or rows.shape[1] != self.ext.shape[1] or rows.shape[0] != len(ids):
            raise ValueError(f"external rows must be [{len(ids)}, {self.ext.shape[1]}], got {tuple(rows.shape)}")
        cap = self.ext.shape[0]
        if len(ids) > cap:
            raise ValueError(f"{len(ids)} external rows exceed the capacity {cap}")
        if any(i >= 0 for i in ids):
            raise ValueError("external embedding ids must be negative")
        new = [j for j, i in enumerate(ids) if i not in self._ext_map]
        if not new:
            return
        if self._ext_next + len(new) > cap:
            self._ext_next = 0
        taken = set(range(self._ext_next, self._ext_next + len(new)))
        self._ext_map = {i: r for i, r in self._ext_map.items() if r not in taken}
        dst = torch.arange(self._ext_next, self._ext_next + len(new))
        self.ext[dst.to(self.ext.device)] = rows[new].to(self.ext.device, torch.float32)
        for k, j in enumerate(new):
            self._ext_map[ids[j]] = self._ext_next + k
        self._ext_next += len(new)
        if self.is_gpu:
            torch.cuda.synchronize(self.device)  # visible to a prefill issued from another thread

    def _device_tokens(self, tokens) -> np.ndarray:
        a = np.asarray(tokens, np.int64)
        if (a < 0).any():
            try:
                a = np.array([t if t >= 0 else -(self._ext_map[t] + 1) for t in a.tolist()], np.int64)
            except KeyError as e:
                raise ValueError(f"external embedding id {e.args[0]} is not registered (set_ext)") from None
        return a.astype(np.int32)

    def prefill(self, sid: int, tokens: list[int], want_logits: bool = True) -> None:
        """Append `tokens` to sequence `sid` (KV computed), leaving logits of the last one in row 0.
        Negative ids are external embedding rows registered with `set_ext`."""
        s = self.kv.seqs[sid]
        start = s.length
        n = len(tokens)
        if start + n > self.ctx:
            raise ValueError(f"context overflow: {start + n} > {self.ctx}")
        self.kv.reserve(sid, start + n)
        self._sync_block_table(sid)
        C = self.max_batch
        for c0 in range(0, n, C):
            chunk = tokens[c0:c0 + C]
            B = len(chunk)
            pos = np.arange(start + c0, start + c0 + B, dtype=np.int32)
            slots = np.array([self.kv.slot(sid, int(p)) for p in pos], np.int32)
            last = c0 + B >= n
            arr = np.stack([pos, slots, pos + 1, np.full(B, s.row, np.int32),
                            np.full(B, B - 1, np.int32)]).astype(np.int32)
            self._upload(arr, self._device_tokens(chunk))
            with trace_range(f"prefill B={B}"):
                self.forward(B, 1 if (last and want_logits) else 0, use_idx=True, prefill=True)
        s.tokens.extend(tokens)

    def embed(self, tokens: list[int]) -> np.ndarray:
        """Mean-pooled final hidden state (after the output norm) -- /api/embed, /v1/embeddings."""
        sid = self.new_sequence()
        try:
            acc, n = None, 0
            for c0 in range(0, len(tokens), self.max_batch):
                chunk = tokens[c0:c0 + self.max_batch]
                self.prefill(sid, chunk, want_logits=False)
                h = self.resid[:len(chunk)].float()
                if self.cfg.arch == "phi2":
                    h = torch.nn.functional.layer_norm(h, (h.shape[-1],), self.w.out_norm, self.w.out_norm_b,
                                                       self.cfg.norm_eps)
                else:
                    h = h * torch.rsqrt(h.pow(2).mean(-1, keepdim=True) + self.cfg.norm_eps) * self.w.out_norm
                s = h.sum(0)
                acc = s if acc is None else acc + s
                n += len(chunk)
            return (acc / max(n, 1)).cpu().numpy()
        finally:
            self.free_sequence(sid)

    # ------------------------------------------------------------------ sampling
    def _set_sampler(self, row: int, o: SamplingOptions, history: list[int], seed: int, step: int = 0):
        history = [t for t in history if t >= 0]  # external embedding rows (images) are not tokens
        self.s_temp[row] = o.temperature
        self.s_topk[row] = o.top_k
        self.s_topp[row] = o.top_p
        self.s_minp[row] = o.min_p
        self.s_rpen[row] = o.repeat_penalty
        self.s_ppen[row] = o.presence_penalty
        self.s_fpen[row] = o.frequency_penalty
        self.s_lastn[row] = o.repeat_last_n
        self.s_seed[row] = seed - (1 << 64) if seed >= (1 << 63) else seed
        self.s_step[row] = step  # RNG counter: draws already made for this request
        h = history[-HIST_CAP:]
        self.s_hist[row].zero_()
        if h:
            self.s_hist[row, :len(h)] = torch.tensor(h, dtype=torch.int32)
        self.s_hcount[row] = len(h)
        self._host_sampler[row] = (o, list(history), seed, step)

    def _sample(self, B: int, feedback: bool = False):
        """feedback (GPU): the sampler's finishing lane of each row also feeds the token back and
        advances the row (csrc/kernels/feedback.h; a separate launch per decode step before round 6)."""
        lg = self.full_logits
        if self.is_gpu:
            p = lambda t: t.data_ptr()  # noqa: E731
            d = dict(logits=p(lg), B=B, V=self.cfg.n_vocab, ld=lg.shape[1], temperature=p(self.s_temp),
                     top_k=p(self.s_topk), top_p=p(self.s_topp), min_p=p(self.s_minp),
                     repeat_penalty=p(self.s_rpen), presence_penalty=p(self.s_ppen),
                     frequency_penalty=p(self.s_fpen), history=p(self.s_hist),
                     hist_count=p(self.s_hcount), hist_cap=HIST_CAP, repeat_last_n=p(self.s_lastn),
                     seed=p(self.s_seed), step=p(self.s_step), out=p(self.s_out),
                     ws=p(self.s_ws), counters=p(self.s_tickets), err=p(self.s_err))
            if feedback:
                d.update(fb_step=p(self.d_step), fb_ld=self.d_step.shape[1], fb_block_table=p(self.d_block_table),
                         fb_max_blocks=self.max_blocks, fb_bs=self.block_size,
                         fb_host_ring=self._host_ring_dev if B == 1 else 0, fb_ring=self._ring_n,
                         fb_sysfence=self.ring_fence)
            native().sample(d, stream_handle())
        else:
            for b in range(B):
                o, hist, seed, step = self._host_sampler[b]
                t = sample_host(lg[b, :self.cfg.n_vocab].numpy(), hist, o, seed, step)
                hist.append(t)
                self._host_sampler[b] = (o, hist, seed, step + 1)
                self.s_out[b] = t

    # ------------------------------------------------------------------ decode
    def _decode_body(self, B: int):
        self.forward(B, B, use_idx=False)
        # GPU: the sampler also feeds each token back and advances its row on device (feedback.h)
        self._sample(B, feedback=True)
        if not self.is_gpu:
            self.d_tokens[:B].copy_(self.s_out[:B])

    def _graph(self, B: int, steps: int = 1, inst: int = 0):
        """The decode graph of `steps` consecutive steps for B rows (one replay = `steps` tokens per row:
        the feedback kernel advances every row on device between them, so no host work sits in between).
        inst: which of the two instances (graph_pair)."""
        key = (B, self._decode_S, steps, inst)
        g = self.graphs.get(key)
        if g is None:
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                # warm-up on the capture stream (first launches load code objects)
                self.forward(B, B, use_idx=False)
            torch.cuda.current_stream().wait_stream(s)
            g = torch.cuda.CUDAGraph()
            # No cyclic GC while capturing: a collection that frees another Runner's graph or
            # events issues HIP destroy calls mid-capture, which invalidates the capture (abort).
            # thread_local: other threads (scheduler, server) may keep issuing HIP calls meanwhile.
            gc.collect()
            gc_was = gc.isenabled()
            gc.disable()
            try:
                with torch.cuda.graph(g, capture_error_mode="thread_local"):
                    for _ in range(steps):
                        self._decode_body(B)
            finally:
                if gc_was:
                    gc.enable()
            self.graphs[key] = g
        return g

    def warmup(self) -> None:
        """Load-time warm-up (as Ollama does at model load): capture the batch-1 decode graph so the
        first request's time-to-first-token does not pay for it. Scratch KV writes land in slot 0,
        which any sequence overwrites at prefill before reading."""
        if not self.is_gpu:
            return
        if self.w16 is not None:  # hipBLASLt plans for the long-prefill path (gemm.hip gemm_lib)
            C = native()
            lm = self.lib_min
            if (lm > 0 and self.max_batch >= lm) or self.moe_lib > 0:
                shapes = {(v.N, v.K) for L in self.w.layers for k, v in L.items()
                          if isinstance(v, DevQMat) and k != "router" and (lm > 0 or k in ("gu_exps", "down_exps"))}
                for N, K in sorted(shapes):
                    if N * K <= self.w16.numel():  # from 128: MoE experts see any row count
                        C.gemm_lib_prepare(N, K, 128, self.max_batch, self.gws.numel() * 4)
        # short prompts through the prefill path (GEMM + prep/finalize kernels resolved once); one per
        # hipBLASLt M bucket too -- a bucket's first GEMM also loads its kernel's code object (~0.1 s),
        # which must not land in a request's TTFT
        lens = [min(self.max_batch, 32), min(self.max_batch, 128)]  # the tile and the dq GEMM paths
        if self.w16 is not None and self.lib_min > 0:
            m = self.lib_min
            while m <= min(self.max_batch, self.ctx - 1):  # every hipBLASLt M bucket (blas.cpp bucket_of)
                lens.append(m)
                m = m * 2 if m < 256 else m + 256
        V = self.cfg.n_vocab
        toks = lambda n, k=0: [self.cfg.bos_id] + [3 + (i * 7919 + k) % max(1, V - 3) for i in range(n - 1)]  # noqa: E731
        for n in lens:  # varied tokens: MoE routing spreads over the experts (per-expert row buckets)
            sid = self.new_sequence()
            try:
                self.prefill(sid, toks(n))
            finally:
                self.free_sequence(sid)
        # batched admission once with a row count off the power-of-two buckets (admit_many rows,
        # hipBLASLt's algorithm check for an exact M): the first call of that check costs ~0.3 s,
        # which the first burst of concurrent requests would otherwise pay
        lm = self.lib_min
        n_each = max(67, lm // 2 + 3) if self.w16 is not None and lm > 0 else 67
        if len(self.kv.rows_free) >= 2 and self.max_batch >= 2 * n_each and self.ctx > n_each:
            sids = [self.new_sequence(), self.new_sequence()]
            try:
                o = SamplingOptions()
                self.admit_many([(sid, 0, toks(n_each, j), o, [], 0) for j, sid in enumerate(sids)])
            finally:
                for sid in sids:
                    self.free_sequence(sid)
        if self.use_graphs:
            buckets = sorted({self.decode_splits(n) for n in range(1, self.ctx + 1)})
            for S in buckets:  # one decode graph per split bucket reachable at this context size
                self._decode_S = S
                self._graph(1)
                if self.decode_group > 1 and self.tp_ctrl is None:
                    self._graph(1, self.decode_group)
            self._decode_S = 0
        torch.cuda.synchronize()
        # the objects alive after load (torch, the model, graphs) move to the permanent generation: a
        # full collection no longer walks them, so one cannot land as a multi-ms pause inside a decode
        # stream (the 256-step engine bench varied 666-698 tok/s while the served stream of the same
        # run held 700-713)
        if os.environ.get("OMX_GC_FREEZE", "1") != "0":
            gc.collect()
            gc.freeze()

    def decode_steps(self, sid: int, pos: int, k: int) -> None:
        """k consecutive batch-1 decode steps of sequence `sid` from input position `pos`, as ONE graph
        replay when graphs are on (generate's pipelined loop): the boundary between two replayed graphs
        costs ~13 us of idle GPU (profiles/r5_decode step traces, the gap after the step's last kernel), paid once
        per k tokens instead of once per token. Every step of the group uses the split bucket of the
        group's last length (any bucket is exact; only its speed depends on the length)."""
        if k <= 1 or not (self.is_gpu and self.use_graphs):
            for j in range(k):
                self.decode_batch([sid], [pos + j])
            return
        if self._closed:
            raise RuntimeError("runner is closed")
        s = self.kv.seqs[sid]
        reserved = False
        if pos + k > len(s.blocks) * self.block_size:
            self.kv.reserve(sid, min(self.ctx, pos + k + 4 * self.block_size))
            self._sync_block_table(sid)
            reserved = True
        if not (not reserved and self._adv_next == (sid, pos)):
            self._upload(np.array([[pos], [self.kv.slot(sid, pos)], [pos + 1], [s.row], [0]], np.int32), None)
        self._decode_S = self.decode_splits(pos + k)
        try:
            with trace_range(f"decode x{k}"):
                self._graph(1, k, self.steps_issued & 1 if self.graph_pair else 0).replay()
            self._adv_next = (sid, pos + k)
            self.steps_issued += k
        finally:
            self._decode_S = 0

    def decode_step(self, sid: int, pos: int | None = None) -> None:
        """One token for sequence `sid` whose input token (not yet in `tokens`) is already in
        d_tokens[0] on device; it sits at position `pos` (default len(tokens))."""
        s = self.kv.seqs[sid]
        self.decode_batch([sid], [s.length if pos is None else pos])

    def decode_batch(self, sids: list[int], poss: list[int]) -> None:
        """One decode step for B = len(sids) sequences (continuous batching: engine/scheduler.py).
        Row b's input token is d_tokens[b] on device and sits at position poss[b]; the step samples
        row b with sampler row b and feeds the sampled tokens back into d_tokens[:B]."""
        if self._closed:
            raise RuntimeError("runner is closed")
        B = len(sids)
        arr = np.empty((5, B), np.int32)
        reserved = False
        for b, (sid, pos) in enumerate(zip(sids, poss)):
            s = self.kv.seqs[sid]
            if pos + 1 > len(s.blocks) * self.block_size:
                self.kv.reserve(sid, min(self.ctx, pos + 4 * self.block_size))
                self._sync_block_table(sid)
                reserved = True
            arr[:, b] = (pos, self.kv.slot(sid, pos), pos + 1, s.row, b)
        # the previous step's feedback kernel already advanced the device inputs to exactly these
        # (sequence, position) rows -- replay without any host upload (continuous batching too)
        nxt = (sids[0], poss[0]) if B == 1 else (tuple(sids), tuple(poss))
        if not (self.is_gpu and not reserved and self._adv_next == nxt):
            self._upload(arr, None)
        self._decode_S = self.decode_splits(poss[0] + 1) if B == 1 else 0
        try:
            with trace_range(f"decode B={B}"):
                if self.use_graphs:
                    self._graph(B, 1, self.steps_issued & 1 if self.graph_pair and B == 1 else 0).replay()
                else:
                    self._decode_body(B)
            if self.is_gpu:
                self._adv_next = (sids[0], poss[0] + 1) if B == 1 else (tuple(sids), tuple(p + 1 for p in poss))
            self.steps_issued += 1
        finally:
            self._decode_S = 0

    def sampler_error(self) -> bool:
        """True (and the word re-armed) when a sample since the last check met non-finite logits: the
        tokens of that request are not valid output. One small device read (a sync)."""
        if self._closed or not self.is_gpu:
            return False
        if int(self.s_err.item()):
            self.s_err.zero_()
            return True
        return False

    def check_sampler(self) -> None:
        if self.sampler_error():
            raise RuntimeError("sampling met non-finite logits (numerical fault upstream); the generated tokens "
                               "are invalid")

    def set_tokens(self, tokens: list[int]) -> None:
        """Host -> d_tokens[:len(tokens)] (batch recomposition: rows' next inputs)."""
        self._upload(np.zeros((5, 0), np.int32), np.asarray(tokens, np.int32))

    # -- continuous-batching operations (engine/scheduler.py); TPRunnerProxy mirrors each one to the
    # -- follower ranks, so every KV / sampler decision of the leader is replayed, never re-derived
    def _keep_prefix(self, sid: int, keep: int, history: list[int]) -> None:
        """Truncate `sid` to its first `keep` tokens, which the caller took from `history[:keep]` (the
        scheduler's prefix match). Under tensor parallelism only the leader's scheduler appends the
        tokens its batched steps decode (scheduler.py `_run_stable`); a follower ran the same steps, so
        its KV holds those positions, but its token list may stop at the prompt. The leader's decision
        is authoritative: restore the follower's bookkeeping from `history` before truncating, so every
        rank keeps and prefills from the same position (a shorter follower list would otherwise free
        KV blocks and prefill at a different start than the leader)."""
        s = self.kv.seqs[sid]
        if s.length < keep:
            if keep > len(history) or keep > len(s.blocks) * self.block_size:
                raise RuntimeError(f"sequence {sid}: cannot keep {keep} tokens (have {s.length}, "
                                   f"{len(s.blocks) * self.block_size} KV slots)")
            s.tokens[s.length:] = list(history[s.length:keep])
        self.kv.truncate(sid, keep)

    def admit(self, sid: int, keep: int, tokens: list[int], opts: SamplingOptions, history: list[int],
              seed: int, n_sampled: int = 0) -> None:
        """Start row 0 of a new request: keep `keep` cached tokens of `sid`, prefill `tokens`, seed the
        sampler (n_sampled draws already made) and sample the first token into s_out[0]."""
        self._keep_prefix(sid, keep, history)
        self.prefill(sid, tokens)
        self._set_sampler(0, opts, history, seed, n_sampled)
        self._sample(1)

    def check_admit(self, sid: int, keep: int, tokens: list[int]) -> None:
        """Read-only validation of one admission (ValueError): every external id registered, the
        prompt within the context window. Lets the scheduler fail one bad request of a burst without
        touching the others' shared forward."""
        s = self.kv.seqs[sid]
        start = min(keep, max(s.length, keep))
        if start + len(tokens) > self.ctx:
            raise ValueError(f"context overflow: {start + len(tokens)} > {self.ctx}")
        self._device_tokens(tokens)

    def admit_many(self, items: list[tuple]) -> list[int]:
        """Start several requests with ONE forward: items[i] = (sid, keep, tokens, opts, history, seed
        [, n_sampled]). Their prompt rows go through the step as independent rows (own position / KV
        slot / block-table row; the multi-sequence paged attention, as a batched decode step), so queued
        requests prefill together instead of stalling the running batch once each. Returns the sampled
        tokens (row i = items[i]). An item may also be a running request's decode row (tokens = its next
        input, keep = its length, n_sampled = its sampler's draws so far) or one chunk of a prompt (its
        sample is the caller's to ignore): the scheduler's interleaved admission mixes both into one
        forward. Falls back to one `admit` per item when the rows exceed max_batch."""
        items = [tuple(it) + (0,) * (7 - len(it)) for it in items]
        total = sum(len(it[2]) for it in items)
        if len(items) == 1 or total > self.max_batch or len(items) > self.max_batch:
            out = []
            for sid, keep, tokens, opts, history, seed, n_s in items:
                self.admit(sid, keep, tokens, opts, history, seed, n_s)
                out.append(int(self.s_out[0].item()))
            return out
        pos_l, slot_l, row_l, toks, last = [], [], [], [], []
        for sid, keep, tokens, _o, history, _sd, _n in items:
            self._keep_prefix(sid, keep, history)
            s = self.kv.seqs[sid]
            start = s.length
            if start + len(tokens) > self.ctx:
                raise ValueError(f"context overflow: {start + len(tokens)} > {self.ctx}")
            self.kv.reserve(sid, start + len(tokens))
            self._sync_block_table(sid)
            for i in range(len(tokens)):
                pos_l.append(start + i)
                slot_l.append(self.kv.slot(sid, start + i))
                row_l.append(s.row)
            toks += list(tokens)
            last.append(len(toks) - 1)
        B, n = len(toks), len(items)
        pos = np.asarray(pos_l, np.int32)
        lidx = np.zeros(B, np.int32)
        lidx[:n] = last
        arr = np.stack([pos, np.asarray(slot_l, np.int32), pos + 1, np.asarray(row_l, np.int32), lidx])
        self._upload(arr.astype(np.int32), self._device_tokens(toks))
        # each admitted prompt is one sequence's contiguous positions: flash (MFMA) attention per segment
        segs, at = [], 0
        for _sid, _k, tokens, _o, _h, _sd, _n in items:
            segs.append((at, len(tokens)))
            at += len(tokens)
        seg_exe = getattr(getattr(self.exe, "exe", None), "set_segments", None) if self.is_gpu else None
        with trace_range(f"admit_many rows={B} seqs={n}"):
            if seg_exe is not None:
                seg_exe(segs)
                try:
                    self.forward(B, n, use_idx=True, prefill=True)
                finally:
                    seg_exe([])
            else:  # torch twin / CPU backend: their attention serves any row -> sequence mapping
                self.forward(B, n, use_idx=True, prefill=False)
        for i, (sid, _k, tokens, opts, history, seed, n_s) in enumerate(items):
            self.kv.seqs[sid].tokens.extend(tokens)
            self._set_sampler(i, opts, history, seed, n_s)
        self._sample(n)
        return [int(t) for t in self.s_out[:n].tolist()]

    def recompose(self, rows: list[tuple], tokens: list[int]) -> None:
        """New batch composition: rows[b] = (opts, history, seed, n_sampled) and the rows' next inputs."""
        for b, (o, hist, seed, n) in enumerate(rows):
            self._set_sampler(b, o, hist, seed, n)
        self.set_tokens(tokens)

    def evict(self, sid: int) -> None:
        """Drop a cached (idle) sequence's KV row."""
        self.kv.free_seq(sid)

    def capture_batch_graphs(self, max_B: int) -> None:
        """Load-time capture of the B = 2..max_B decode graphs (continuous batching)."""
        if self.use_graphs:
            for B in range(2, max_B + 1):
                self._graph(B)
            torch.cuda.synchronize()

    def _generate_pipelined(self, sid: int, st, first: int, max_tokens: int, stop, times, t1,
                            ctrl=None) -> Iterator[int]:
        """Two decode steps in flight: step i consumes token i+1 straight from device memory (written
        by step i-1's sampler), so the host never has to see a token before issuing the step after
        it. When token n is handed out, steps producing tokens n+1 and n+2 are already queued; the
        host's detokenise / stop checks / Python overhead hide behind ~2 steps of GPU work instead of
        leaving the GPU idle between steps (was ~130 us per step, profiles/r1_attn). A step issued
        past a stop is wasted work whose KV position is never recorded in `tokens`.

        Tensor parallel (`ctrl`): every rank runs this same loop. The leader decides each handed-out
        token (its server applies stop strings on text) and broadcasts go / stop on the gloo control
        group; followers take that decision instead of their own, so all ranks issue exactly the same
        steps, two in flight, and read their own (identical) sampled tokens from their host rings."""
        base = st.length  # position of `first`
        ring = self._host_ring  # host-mapped: step at input position p stores its token at p % R
        R = self._ring_n
        evs: list = [None] * R
        issued = 0
        # steps per graph replay (decode_steps): groups of G when this rank decides alone; TP ranks step
        # one token at a time, as the leader's go / stop signal does
        G = self.decode_group if ctrl is None else 1

        def issue(cap: int):
            nonlocal issued
            k = max(1, min(G, cap - issued))
            if k == 1:
                self.decode_step(sid, base + issued)
            else:
                self.decode_steps(sid, base + issued, k)
            e = torch.cuda.Event()
            e.record()
            for j in range(k):
                evs[(base + issued + j) % R] = e
            issued += k

        n = 0
        tok = first
        leader = ctrl is not None and ctrl.leader
        follower = ctrl is not None and not ctrl.leader
        try:
            while True:
                n += 1  # handing out token n (1-based; token 1 came from the prompt)
                if follower:
                    done = not ctrl.wait()
                else:
                    done = n >= max_tokens or (stop is not None and stop(tok))
                if not done:
                    if leader:
                        ctrl.signal(True)
                    # steps 0..n (tokens up to n+2) at least; a group keeps up to G - 1 more queued
                    target = min(n + (G if G > 1 else 1), max_tokens - 1)
                    while issued < min(n + 1, max_tokens - 1) or (G > 1 and issued < target):
                        issue(max_tokens - 1)
                    st.tokens.append(tok)  # step n-1 (issued) writes its KV
                yield tok
                if done:
                    break
                slot = (base + n - 1) % R  # step n-1 produced token n+1
                evs[slot].synchronize()
                tok = int(ring[slot])
        finally:
            if leader:
                ctrl.signal(False)  # generation over (also when the consumer closed us early)
            if ctrl is not None and self.ar is not None:
                self.ar.check()  # a peer that missed a barrier timed the step out: fail loudly
            self.check_sampler()
            if times is not None:
                times.gen_tokens = n
                times.gen_s = time.perf_counter() - t1

    def generate(self, sid: int, prompt: list[int], options: SamplingOptions | None = None,
                 max_tokens: int = 128, stop: Callable[[int], bool] | None = None,
                 times: StepTimes | None = None) -> Iterator[int]:
        """Stream sampled tokens. Reuses the KV prefix shared with what `sid` already holds."""
        o = options or SamplingOptions()
        seed = o.resolved_seed()
        st = self.kv.seqs[sid]
        keep = self.kv.common_prefix(st.tokens, prompt)
        keep = min(keep, len(prompt) - 1)
        self.kv.truncate(sid, keep)
        t0 = time.perf_counter()
        self.prefill(sid, prompt[keep:])
        self._set_sampler(0, o, prompt, seed)
        self._sample(1)
        if self.is_gpu:
            self.d_tokens[:1].copy_(self.s_out[:1])
            self._tok_host[:1].copy_(self.s_out[:1], non_blocking=True)
            torch.cuda.synchronize()
            first = int(self._tok_host[0])
        else:
            first = int(self.s_out[0])
            self.d_tokens[0] = first
        if times is not None:
            times.prompt_tokens = len(prompt) - keep
            times.prompt_s = time.perf_counter() - t0
        t1 = time.perf_counter()
        max_tokens = min(max_tokens, self.ctx - st.length)
        if self.is_gpu:
            yield from self._generate_pipelined(sid, st, first, max_tokens, stop, times, t1, ctrl=self.tp_ctrl)
            return
        n = 0
        tok = first
        ctrl = self.tp_ctrl
        follower = ctrl is not None and not ctrl.leader
        try:
            while True:
                n += 1
                if follower:  # the leader decides (its server applies stop strings on text)
                    done = not ctrl.wait()
                else:
                    done = n >= max_tokens or (stop is not None and stop(tok))
                if not done:
                    if ctrl is not None and ctrl.leader:
                        ctrl.signal(True)
                    # enqueue the next step before handing this token out: the GPU runs one step
                    # ahead of the host (detokenize / stream / stop checks overlap the forward)
                    self.decode_step(sid)
                    if self.is_gpu:
                        self._tok_host[:1].copy_(self.s_out[:1], non_blocking=True)
                        ev = torch.cuda.Event()
                        ev.record()
                    st.tokens.append(tok)  # its KV is being written by the step just issued
                yield tok
                if done:
                    break
                if self.is_gpu:
                    ev.synchronize()
                    tok = int(self._tok_host[0])
                else:
                    tok = int(self.s_out[0])
        finally:
            if ctrl is not None and ctrl.leader:
                ctrl.signal(False)  # generation over (also when the consumer closed us early)
            if self.ar is not None:
                self.ar.check()  # a peer that missed a barrier timed the step out: fail loudly
            if times is not None:
                times.gen_tokens = n
                times.gen_s = time.perf_counter() - t1
