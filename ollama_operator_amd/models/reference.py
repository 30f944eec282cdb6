"""fp32 PyTorch reference forward for every supported architecture (llama / mistral / mixtral /
phi2), reading dequantized weights straight from a GGUF file. It is the numerical oracle for the
HIP kernels and the engine; it is never on the serving hot path.
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F

from ..gguf.reader import GGUFFile
from .config import ROPE_NEOX, ModelConfig


def rms_norm(x: torch.Tensor, w: torch.Tensor, eps: float) -> torch.Tensor:
    return x * torch.rsqrt(x.pow(2).mean(-1, keepdim=True) + eps) * w


def layer_norm(x: torch.Tensor, w: torch.Tensor, b: torch.Tensor, eps: float) -> torch.Tensor:
    return F.layer_norm(x, (x.shape[-1],), w, b, eps)


def gelu_tanh(x: torch.Tensor) -> torch.Tensor:
    return 0.5 * x * (1.0 + torch.tanh(math.sqrt(2.0 / math.pi) * (x + 0.044715 * x.pow(3))))


def rope(x: torch.Tensor, pos: torch.Tensor, n_rot: int, base: float, mode: int) -> torch.Tensor:
    """x: [T, H, D]; pos: [T] int. Rotates the first n_rot dims of each head."""
    T, H, D = x.shape
    half = n_rot // 2
    inv = base ** (-torch.arange(0, half, dtype=torch.float64) * 2.0 / n_rot)
    ang = pos.to(torch.float64)[:, None] * inv[None, :]
    cos = torch.cos(ang).to(x.dtype)[:, None, :]
    sin = torch.sin(ang).to(x.dtype)[:, None, :]
    out = x.clone()
    if mode == ROPE_NEOX:
        x0, x1 = x[..., :half], x[..., half:n_rot]
        out[..., :half] = x0 * cos - x1 * sin
        out[..., half:n_rot] = x0 * sin + x1 * cos
    else:
        x0, x1 = x[..., 0:n_rot:2], x[..., 1:n_rot:2]
        out[..., 0:n_rot:2] = x0 * cos - x1 * sin
        out[..., 1:n_rot:2] = x0 * sin + x1 * cos
    return out


class KVCacheRef:
    def __init__(self, cfg: ModelConfig, max_len: int, device="cpu", dtype=torch.float32):
        self.k = [torch.zeros(max_len, cfg.n_head_kv, cfg.head_dim, device=device, dtype=dtype)
                  for _ in range(cfg.n_layer)]
        self.v = [torch.zeros_like(t) for t in self.k]
        self.len = 0


class ReferenceModel:
    def __init__(self, gguf: GGUFFile, cfg: ModelConfig | None = None, device: str = "cpu",
                 dtype: torch.dtype = torch.float32):
        self.cfg = cfg or ModelConfig.from_gguf_metadata(gguf.metadata)
        self.device = device
        self.dtype = dtype
        self.w: dict[str, torch.Tensor] = {}
        for name in gguf.tensors:
            self.w[name] = torch.from_numpy(gguf.array(name).copy()).to(device=device, dtype=dtype)

    def _attn(self, q, k, v, cache: KVCacheRef, layer: int, start: int):
        cfg = self.cfg
        T = q.shape[0]
        cache.k[layer][start:start + T] = k
        cache.v[layer][start:start + T] = v
        L = start + T
        K = cache.k[layer][:L]
        V = cache.v[layer][:L]
        g = cfg.gqa
        K = K.repeat_interleave(g, dim=1)
        V = V.repeat_interleave(g, dim=1)
        s = torch.einsum("thd,lhd->htl", q, K) / math.sqrt(cfg.head_dim)
        qpos = torch.arange(start, start + T, device=q.device)[:, None]
        kpos = torch.arange(L, device=q.device)[None, :]
        mask = kpos > qpos
        if cfg.sliding_window:
            mask = mask | (kpos <= qpos - cfg.sliding_window)
        s = s.masked_fill(mask[None], float("-inf"))
        p = torch.softmax(s, dim=-1)
        o = torch.einsum("htl,lhd->thd", p, V)
        return o.reshape(T, cfg.n_head * cfg.head_dim)

    def _moe(self, xn, b):
        cfg = self.cfg
        logits = xn @ self.w[b + "ffn_gate_inp.weight"].T  # [T, X]
        probs = torch.softmax(logits, dim=-1)
        topw, topi = probs.topk(cfg.n_expert_used, dim=-1)
        topw = topw / topw.sum(-1, keepdim=True)
        out = torch.zeros_like(xn)
        G, U, D = (self.w[b + "ffn_gate_exps.weight"], self.w[b + "ffn_up_exps.weight"],
                   self.w[b + "ffn_down_exps.weight"])
        for t in range(xn.shape[0]):
            for j in range(cfg.n_expert_used):
                e = int(topi[t, j])
                h = F.silu(G[e] @ xn[t]) * (U[e] @ xn[t])
                out[t] += topw[t, j] * (D[e] @ h)
        return out

    @torch.no_grad()
    def forward(self, tokens: torch.Tensor, cache: KVCacheRef, start: int | None = None) -> torch.Tensor:
        cfg = self.cfg
        w = self.w
        start = cache.len if start is None else start
        T = tokens.shape[0]
        pos = torch.arange(start, start + T, device=self.device)
        x = w["token_embd.weight"][tokens]
        H, Hk, D = cfg.n_head, cfg.n_head_kv, cfg.head_dim
        for i in range(cfg.n_layer):
            b = f"blk.{i}."
            if cfg.arch == "phi2":
                xn = layer_norm(x, w[b + "attn_norm.weight"], w[b + "attn_norm.bias"], cfg.norm_eps)
                qkv = xn @ w[b + "attn_qkv.weight"].T + w[b + "attn_qkv.bias"]
                q, k, v = qkv.split([H * D, Hk * D, Hk * D], dim=-1)
                q = rope(q.reshape(T, H, D), pos, cfg.n_rot, cfg.rope_base, cfg.rope_mode)
                k = rope(k.reshape(T, Hk, D), pos, cfg.n_rot, cfg.rope_base, cfg.rope_mode)
                a = self._attn(q, k, v.reshape(T, Hk, D), cache, i, start)
                a = a @ w[b + "attn_output.weight"].T + w[b + "attn_output.bias"]
                h = gelu_tanh(xn @ w[b + "ffn_up.weight"].T + w[b + "ffn_up.bias"])
                f = h @ w[b + "ffn_down.weight"].T + w[b + "ffn_down.bias"]
                x = x + a + f
                continue
            xn = rms_norm(x, w[b + "attn_norm.weight"], cfg.norm_eps)
            q = (xn @ w[b + "attn_q.weight"].T).reshape(T, H, D)
            k = (xn @ w[b + "attn_k.weight"].T).reshape(T, Hk, D)
            v = (xn @ w[b + "attn_v.weight"].T).reshape(T, Hk, D)
            q = rope(q, pos, cfg.n_rot, cfg.rope_base, cfg.rope_mode)
            k = rope(k, pos, cfg.n_rot, cfg.rope_base, cfg.rope_mode)
            a = self._attn(q, k, v, cache, i, start)
            x = x + a @ w[b + "attn_output.weight"].T
            xn = rms_norm(x, w[b + "ffn_norm.weight"], cfg.norm_eps)
            if cfg.n_expert:
                x = x + self._moe(xn, b)
            else:
                h = F.silu(xn @ w[b + "ffn_gate.weight"].T) * (xn @ w[b + "ffn_up.weight"].T)
                x = x + h @ w[b + "ffn_down.weight"].T
        cache.len = start + T
        if cfg.arch == "phi2":
            xn = layer_norm(x, w["output_norm.weight"], w["output_norm.bias"], cfg.norm_eps)
            return xn @ w["output.weight"].T + w["output.bias"]
        xn = rms_norm(x, w["output_norm.weight"], cfg.norm_eps)
        return xn @ w["output.weight"].T
