"""Torch twin of the native step executor (csrc/runtime/executor.cpp).

Same weights (`DeviceWeights`, repacked streams), same buffers, same paged KV cache and the same
stage API (`embed`, `attn`, `ffn`, `head`), implemented with fp32 torch ops on dequantized
matrices. It is (a) the CPU serving backend (BASELINE config "phi on kind, CPU-only server"),
(b) the oracle the GPU tests compare the HIP executor against, and (c) the engine used by the
multi-process tensor-parallel tests on CPU (gloo).
"""
from __future__ import annotations

import math

import numpy as np
import torch
import torch.nn.functional as F

from ..gguf import GGMLType
from ..quant import REPACK_STREAMS, dequantize, repack_row_bytes, unrepack


def dequant_qmat(m) -> torch.Tensor:
    """DevQMat -> float32 [rows_total, K] on the matrix's device."""
    names = REPACK_STREAMS[GGMLType(m.qtype)]
    rows = m.streams[0].numel() // repack_row_bytes(m.qtype, m.K)[0]
    st = {n: s.detach().cpu().numpy() for n, s in zip(names, m.streams)}
    raw = unrepack(st, m.qtype, rows, m.K)
    w = dequantize(raw, m.qtype, rows * m.K).reshape(rows, m.K)
    return torch.from_numpy(w).to(m.streams[0].device)


class TorchExecutor:
    def __init__(self, runner):
        self.r = runner
        self.w = runner.w
        self._dq: dict[int, torch.Tensor] = {}

    def W(self, m) -> torch.Tensor:
        k = id(m)
        if k not in self._dq:
            self._dq[k] = dequant_qmat(m)
        return self._dq[k]

    # ------------------------------------------------------------------ helpers
    def _norm(self, x, w, b=None):
        cfg = self.w.cfg
        if cfg.arch == "phi2":
            return F.layer_norm(x, (x.shape[-1],), w, b, cfg.norm_eps)
        return x * torch.rsqrt(x.pow(2).mean(-1, keepdim=True) + cfg.norm_eps) * w

    def _rope_pairs(self, x: torch.Tensor, pos: torch.Tensor, D: int) -> torch.Tensor:
        """Rotate adjacent pairs (2i, 2i+1) for in-head dims < n_rot; x: [B, nh*D]."""
        n_rot = self.w.cfg.n_rot
        B = x.shape[0]
        x = x.view(B, -1, D).clone()
        inv = self.w.inv_freq.to(x.device)
        ang = pos.to(torch.float32)[:, None] * inv[None, :]  # [B, n_rot/2]
        cos, sin = torch.cos(ang)[:, None, :], torch.sin(ang)[:, None, :]
        x0, x1 = x[..., 0:n_rot:2].clone(), x[..., 1:n_rot:2].clone()
        x[..., 0:n_rot:2] = x0 * cos - x1 * sin
        x[..., 1:n_rot:2] = x0 * sin + x1 * cos
        return x.view(B, -1)

    # ------------------------------------------------------------------ stages
    def embed(self, B: int):
        r = self.r
        toks = r.d_tokens[:B].long()
        r.resid[:B] = self.W(self.w.tok_embd)[toks.clamp(min=0)] * self.w.cfg.embed_scale
        ext = toks < 0  # external embedding rows -(id + 1) (image patches), unscaled
        if bool(ext.any()):
            r.resid[:B][ext] = r.ext[(-toks[ext] - 1)].to(r.resid.dtype)

    def attn(self, i: int, B: int):
        r, w = self.r, self.w
        L = w.layers[i]
        loc = w.local
        D, H, Hkv = loc["D"], loc["H"], loc["Hkv"]
        Eq, Ekv = H * D, Hkv * D
        x = r.resid[:B]
        xn = self._norm(x, L["attn_norm"], L.get("attn_norm_b"))
        qkv = xn @ self.W(L["wqk"]).T
        if "wv" in L:
            qkv = torch.cat([qkv, xn @ self.W(L["wv"]).T], dim=1)
        if L.get("qkv_bias") is not None:
            qkv = qkv + L["qkv_bias"]
        pos = r.d_pos[:B].long()
        q = self._rope_pairs(qkv[:, :Eq], pos, D)
        k = self._rope_pairs(qkv[:, Eq:Eq + Ekv], pos, D)
        v = qkv[:, Eq + Ekv:Eq + 2 * Ekv]
        slot = r.d_slot[:B].long()
        bs = r.block_size
        kc, vc = r.kc[i], r.vc[i]
        blk, off = slot // bs, slot % bs
        kc[blk, :, off] = k.view(B, Hkv, D).to(kc.dtype)
        vc[blk, :, off] = v.view(B, Hkv, D).to(vc.dtype)
        if w.cfg.arch == "phi2":
            r.hbuf[:B, :loc["F"]] = self._gelu(xn @ self.W(L["wgu"]).T + L["bup"])
        out = torch.empty(B, Eq, device=x.device)
        G = H // Hkv
        scale = 1.0 / math.sqrt(D)
        window = w.cfg.sliding_window
        for b in range(B):
            n = int(r.d_qlen[b])
            row = int(r.d_qseq[b])
            start = max(0, n - window) if window else 0
            bt = r.d_block_table[row].long()
            t = torch.arange(start, n, device=x.device)
            kk = kc[bt[t // bs], :, t % bs].float()  # [n, Hkv, D]
            vv = vc[bt[t // bs], :, t % bs].float()
            qq = q[b].view(H, D)
            kk = kk.repeat_interleave(G, dim=1)
            vv = vv.repeat_interleave(G, dim=1)
            s = torch.einsum("hd,thd->ht", qq, kk) * scale
            p = torch.softmax(s, dim=-1)
            out[b] = torch.einsum("ht,thd->hd", p, vv).reshape(-1)
        r.abuf[:B] = out
        o = out @ self.W(L["wo"]).T
        if L.get("bo") is not None:
            o = o + L["bo"]
        if r.tp_size > 1:
            r.ypart[:B] = o
        else:
            r.resid[:B] += o

    @staticmethod
    def _gelu(x):
        return 0.5 * x * (1.0 + torch.tanh(math.sqrt(2.0 / math.pi) * (x + 0.044715 * x.pow(3))))

    def ffn(self, i: int, B: int):
        r, w = self.r, self.w
        L = w.layers[i]
        loc = w.local
        Fl = loc["F"]
        cfg = w.cfg
        if cfg.arch == "phi2":
            y = r.hbuf[:B, :Fl] @ self.W(L["wdown"]).T
            if L.get("bdown") is not None:
                y = y + L["bdown"]
        else:
            xn = self._norm(r.resid[:B], L["ffn_norm"])
            if cfg.n_expert:
                X, k = cfg.n_expert, cfg.n_expert_used
                logits = xn @ self.W(L["router"]).T
                probs = torch.softmax(logits, dim=-1)
                tw, ti = probs.topk(k, dim=-1)
                tw = tw / tw.sum(-1, keepdim=True)
                GU = self.W(L["gu_exps"]).view(X, 2 * Fl, -1)
                DN = self.W(L["down_exps"]).view(X, w.local["E"], -1)
                y = torch.zeros_like(xn)
                for b in range(B):
                    for j in range(k):
                        e = int(ti[b, j])
                        gu = GU[e] @ xn[b]
                        h = F.silu(gu[0::2]) * gu[1::2]
                        y[b] += tw[b, j] * (DN[e] @ h)
            else:
                gu = xn @ self.W(L["wgu"]).T
                act = self._gelu if cfg.gelu_glu else F.silu
                h = act(gu[:, 0::2]) * gu[:, 1::2]
                y = h @ self.W(L["wdown"]).T
        if r.tp_size > 1:
            r.ypart[:B] = y
        else:
            r.resid[:B] += y

    def head(self, n_logits: int, use_idx: bool):
        r, w = self.r, self.w
        if n_logits <= 0:
            return
        x = r.resid[r.d_logit_idx[:n_logits].long()] if use_idx else r.resid[:n_logits]
        xn = self._norm(x, w.out_norm, w.out_norm_b)
        lg = xn @ self.W(w.lm_head).T
        if w.lm_bias is not None:
            lg = lg + w.lm_bias
        r.logits[:n_logits, :lg.shape[1]] = lg

    def run(self, stage: str, layer: int, B: int, n_logits: int = 0, use_idx: bool = False,
            prefill: bool = False):
        if stage == "embed":
            self.embed(B)
        elif stage == "attn":
            self.attn(layer, B)
        elif stage == "ffn":
            self.ffn(layer, B)
        elif stage == "head":
            self.head(n_logits, use_idx)
        elif stage == "forward":
            self.embed(B)
            for i in range(self.w.cfg.n_layer):
                self.attn(i, B)
                self.ffn(i, B)
            self.head(n_logits, use_idx)
        else:
            raise ValueError(stage)


def np_to_i32(a) -> np.ndarray:
    return np.ascontiguousarray(a, dtype=np.int32)
