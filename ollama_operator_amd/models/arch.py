"""GGUF tensor naming and per-tensor quant-type policy for each supported architecture.

Names follow the public llama.cpp GGUF conventions (`blk.{i}.attn_q.weight`, ...). The K-quant
mix for `Q4_K_M` follows llama.cpp's public rule: output.weight Q6_K; attn_v / ffn_down Q6_K in
the "more bits" layers (first and last eighth, and every third in between), Q4_K elsewhere;
`Q5_K_M` / `Q5_K_S` the same with Q5_K as the base type.
"""
from __future__ import annotations

from ..gguf.constants import FileType, GGMLType
from .config import ModelConfig


def use_more_bits(i: int, n: int) -> bool:
    return i < n // 8 or i >= 7 * n // 8 or (i - n // 8) % 3 == 2


def _matrix_type(ftype: FileType, role: str, layer: int, n_layer: int) -> GGMLType:
    if ftype == FileType.ALL_F32:
        return GGMLType.F32
    if ftype == FileType.MOSTLY_F16:
        return GGMLType.F16
    if ftype == FileType.MOSTLY_BF16:
        return GGMLType.BF16
    if ftype == FileType.MOSTLY_Q8_0:
        return GGMLType.Q8_0
    if ftype == FileType.MOSTLY_Q6_K:
        return GGMLType.Q6_K
    if ftype == FileType.MOSTLY_Q4_0:
        return GGMLType.Q6_K if role == "output" else GGMLType.Q4_0
    if ftype in (FileType.MOSTLY_Q4_K_M, FileType.MOSTLY_Q4_K_S):
        if role == "output":
            return GGMLType.Q6_K
        if ftype == FileType.MOSTLY_Q4_K_M and role in ("attn_v", "ffn_down") and use_more_bits(layer, n_layer):
            return GGMLType.Q6_K
        return GGMLType.Q4_K
    if ftype in (FileType.MOSTLY_Q5_K_M, FileType.MOSTLY_Q5_K_S):
        if role == "output":
            return GGMLType.Q6_K
        if ftype == FileType.MOSTLY_Q5_K_M and role in ("attn_v", "ffn_down") and use_more_bits(layer, n_layer):
            return GGMLType.Q6_K
        return GGMLType.Q5_K
    raise NotImplementedError(f"file type {ftype!r}")


# llama.cpp cannot k-quantise a row whose length is not a multiple of the 256-weight super-block
# (llama_tensor_get_type): it falls back to a 32-block type. Q4_K's fallback there is Q5_0, which this
# framework does not implement; Q4_0 stands in (same 32-block family).
_KQ_FALLBACK = {GGMLType.Q4_K: GGMLType.Q4_0, GGMLType.Q5_K: GGMLType.Q8_0, GGMLType.Q6_K: GGMLType.Q8_0}


def tensor_specs(cfg: ModelConfig, ftype: FileType) -> list[tuple[str, tuple[int, ...], GGMLType]]:
    """[(name, ggml shape (ne0 first), type)] for every tensor of the model."""
    return [(n, sh, _KQ_FALLBACK.get(t, t) if sh[0] % 256 else t) for n, sh, t in _tensor_specs(cfg, ftype)]


def _tensor_specs(cfg: ModelConfig, ftype: FileType) -> list[tuple[str, tuple[int, ...], GGMLType]]:
    E, F, V, L = cfg.n_embd, cfg.n_ff, cfg.n_vocab, cfg.n_layer
    Ekv = cfg.n_embd_kv
    f32 = GGMLType.F32
    mt = lambda role, i=0: _matrix_type(ftype, role, i, L)  # noqa: E731
    # tied embeddings (Gemma) carry the output projection's type (llama.cpp quantises token_embd as
    # output.weight when the latter is absent)
    emb_role = "output" if cfg.arch == "gemma" else "token_embd"
    specs: list[tuple[str, tuple[int, ...], GGMLType]] = [("token_embd.weight", (E, V), mt(emb_role))]
    if cfg.arch == "phi2":
        for i in range(L):
            b = f"blk.{i}."
            specs += [
                (b + "attn_norm.weight", (E,), f32), (b + "attn_norm.bias", (E,), f32),
                (b + "attn_qkv.weight", (E, E + 2 * Ekv), mt("attn_qkv", i)),
                (b + "attn_qkv.bias", (E + 2 * Ekv,), f32),
                (b + "attn_output.weight", (E, E), mt("attn_output", i)), (b + "attn_output.bias", (E,), f32),
                (b + "ffn_up.weight", (E, F), mt("ffn_up", i)), (b + "ffn_up.bias", (F,), f32),
                (b + "ffn_down.weight", (F, E), mt("ffn_down", i)), (b + "ffn_down.bias", (E,), f32),
            ]
        specs += [("output_norm.weight", (E,), f32), ("output_norm.bias", (E,), f32),
                  ("output.weight", (E, V), mt("output")), ("output.bias", (V,), f32)]
        return specs
    Eq = cfg.n_embd_q
    for i in range(L):
        b = f"blk.{i}."
        specs += [
            (b + "attn_norm.weight", (E,), f32),
            (b + "attn_q.weight", (E, Eq), mt("attn_q", i)),
            (b + "attn_k.weight", (E, Ekv), mt("attn_k", i)),
            (b + "attn_v.weight", (E, Ekv), mt("attn_v", i)),
            (b + "attn_output.weight", (Eq, E), mt("attn_output", i)),
            (b + "ffn_norm.weight", (E,), f32),
        ]
        if cfg.n_expert:
            X = cfg.n_expert
            specs += [
                (b + "ffn_gate_inp.weight", (E, X), f32),
                (b + "ffn_gate_exps.weight", (E, F, X), mt("ffn_gate", i)),
                (b + "ffn_up_exps.weight", (E, F, X), mt("ffn_up", i)),
                (b + "ffn_down_exps.weight", (F, E, X), mt("ffn_down", i)),
            ]
        else:
            specs += [
                (b + "ffn_gate.weight", (E, F), mt("ffn_gate", i)),
                (b + "ffn_up.weight", (E, F), mt("ffn_up", i)),
                (b + "ffn_down.weight", (F, E), mt("ffn_down", i)),
            ]
    specs += [("output_norm.weight", (E,), f32)]
    if cfg.arch != "gemma":  # Gemma ties the output projection to token_embd
        specs += [("output.weight", (E, V), mt("output"))]
    return specs
