"""Model hyper-parameters, read from GGUF metadata, plus presets for the architectures the reference
advertises (reference `README.md:43-59`: Llama 2 7B/13B/70B, Mistral, Phi-2, Mixtral ...) and the
BASELINE.json configs (Llama-2-7B Q4_K_M, Mistral-7B, Llama-2-70B, Mixtral-8x7B, Phi-2).
"""
from __future__ import annotations

from dataclasses import asdict, dataclass, field, replace
from typing import Any

ROPE_NORM = 0   # rotate adjacent pairs (x[2i], x[2i+1]) -- llama.cpp "normal" mode (llama GGUF)
ROPE_NEOX = 2   # rotate halves (x[i], x[i + n_rot/2]) -- phi2 / gpt-neox

# GGUF `general.architecture` values this engine runs, mapped to its internal arch. llama.cpp writes
# "llama" for Llama 2 / Code Llama / Vicuna / Mistral / Mixtral (MoE via expert_count).
SUPPORTED_ARCHS = {"llama": "llama", "phi2": "phi2", "gemma": "gemma"}


class UnsupportedArchitecture(ValueError):
    """A GGUF whose `general.architecture` this engine does not implement: loading must fail loudly
    rather than run the weights through the wrong graph (VERDICT r2 missing #3)."""


@dataclass
class ModelConfig:
    arch: str = "llama"            # "llama" (also Mistral / Mixtral / CodeLlama / Vicuna), "phi2", "gemma"
    n_vocab: int = 32000
    n_embd: int = 4096
    n_layer: int = 32
    n_head: int = 32
    n_head_kv: int = 32
    n_ff: int = 11008
    n_rot: int = 128
    rope_base: float = 10000.0
    rope_mode: int = ROPE_NORM
    norm_eps: float = 1e-5
    ctx_len: int = 4096
    n_expert: int = 0
    n_expert_used: int = 0
    sliding_window: int = 0
    n_embd_head: int = 0           # head dim when not n_embd / n_head (Gemma: attention.key_length = 256)
    bos_id: int = 1
    eos_id: int = 2
    name: str = ""
    extra: dict[str, Any] = field(default_factory=dict)

    @property
    def head_dim(self) -> int:
        return self.n_embd_head or self.n_embd // self.n_head

    @property
    def n_embd_q(self) -> int:
        return self.head_dim * self.n_head

    @property
    def gelu_glu(self) -> bool:
        """GeGLU FFN (gelu(gate) * up) instead of SwiGLU (Gemma)."""
        return self.arch == "gemma"

    @property
    def embed_scale(self) -> float:
        """Token embeddings are multiplied by sqrt(n_embd) (Gemma; llama.cpp build_gemma)."""
        return float(self.n_embd) ** 0.5 if self.arch == "gemma" else 1.0

    @property
    def n_embd_kv(self) -> int:
        return self.head_dim * self.n_head_kv

    @property
    def gqa(self) -> int:
        return self.n_head // self.n_head_kv

    @property
    def uses_layernorm(self) -> bool:
        return self.arch == "phi2"

    def to_dict(self) -> dict:
        return asdict(self)

    @classmethod
    def from_gguf_metadata(cls, md: dict[str, Any]) -> "ModelConfig":
        if "general.architecture" not in md:
            raise UnsupportedArchitecture("GGUF has no general.architecture")
        arch = str(md["general.architecture"])
        if arch not in SUPPORTED_ARCHS:
            raise UnsupportedArchitecture(
                f"unsupported model architecture {arch!r} (supported: {', '.join(sorted(SUPPORTED_ARCHS))})")
        p = arch + "."

        def g(k, default=None):
            return md.get(p + k, default)

        tokens = md.get("tokenizer.ggml.tokens")
        n_embd = int(g("embedding_length"))
        n_head = int(g("attention.head_count"))
        head = int(g("attention.key_length", n_embd // n_head))
        if int(g("attention.value_length", head)) != head:
            raise UnsupportedArchitecture("attention.value_length != attention.key_length")
        check_head_dim(head)
        cfg = cls(
            arch=SUPPORTED_ARCHS[arch],
            n_vocab=int(g("vocab_size", len(tokens) if tokens is not None else 32000)),
            n_embd=n_embd,
            n_layer=int(g("block_count")),
            n_head=n_head,
            n_head_kv=int(g("attention.head_count_kv", n_head)),
            n_ff=int(g("feed_forward_length")),
            n_rot=int(g("rope.dimension_count", head)),
            rope_base=float(g("rope.freq_base", 10000.0)),
            rope_mode=ROPE_NEOX if arch in ("phi2", "gemma") else ROPE_NORM,  # llama.cpp llama_rope_type
            norm_eps=float(g("attention.layer_norm_rms_epsilon", g("attention.layer_norm_epsilon", 1e-5))),
            ctx_len=int(g("context_length", 4096)),
            n_expert=int(g("expert_count", 0)),
            n_expert_used=int(g("expert_used_count", 0)),
            sliding_window=int(g("attention.sliding_window", 0) or 0),
            n_embd_head=head if head != n_embd // n_head else 0,
            bos_id=int(md.get("tokenizer.ggml.bos_token_id", 1)),
            eos_id=int(md.get("tokenizer.ggml.eos_token_id", 2)),
            name=str(md.get("general.name", "")),
        )
        return cfg

    def to_gguf_metadata(self) -> dict[str, Any]:
        a = self.arch if self.arch in ("phi2", "gemma") else "llama"
        p = a + "."
        md: dict[str, Any] = {
            "general.architecture": a,
            "general.name": self.name or a,
            p + "context_length": self.ctx_len,
            p + "embedding_length": self.n_embd,
            p + "block_count": self.n_layer,
            p + "feed_forward_length": self.n_ff,
            p + "rope.dimension_count": self.n_rot,
            p + "attention.head_count": self.n_head,
            p + "attention.head_count_kv": self.n_head_kv,
        }
        if self.n_embd_head or a == "gemma":
            md[p + "attention.key_length"] = self.head_dim
            md[p + "attention.value_length"] = self.head_dim
        if a == "phi2":
            md[p + "attention.layer_norm_epsilon"] = float(self.norm_eps)
        else:
            md[p + "attention.layer_norm_rms_epsilon"] = float(self.norm_eps)
            md[p + "rope.freq_base"] = float(self.rope_base)
        if self.n_expert:
            md[p + "expert_count"] = self.n_expert
            md[p + "expert_used_count"] = self.n_expert_used
        return md


# attention kernels (csrc/kernels/attention.hip) exist for these KV row widths; a head dim that is not
# one of them runs in the next one up (zero-padded cache rows, masked q / output): Orca Mini's 100 -> 112
ATTN_ROW_DIMS = (64, 80, 96, 112, 128, 256)


def cache_head_dim(head: int) -> int:
    """KV cache row width on the GPU for head dim `head` (the CPU backends keep `head`)."""
    for d in ATTN_ROW_DIMS:
        if head <= d:
            return d
    raise UnsupportedArchitecture(f"head dim {head} exceeds the largest attention kernel ({ATTN_ROW_DIMS[-1]})")


def check_head_dim(head: int) -> None:
    """Refuse at load what the GPU attention kernels cannot serve, instead of loading a model whose
    attention would silently not run (a head dim without a kernel used to no-op)."""
    if head <= 0 or head % 4 or cache_head_dim(head) - head >= 16:
        raise UnsupportedArchitecture(
            f"unsupported attention head dim {head} (supported: {', '.join(map(str, ATTN_ROW_DIMS))}, "
            "or a multiple of 4 up to 15 below one of them)")


PRESETS: dict[str, ModelConfig] = {
    # BASELINE headline: Llama-2-7B Q4_K_M
    "llama2-7b": ModelConfig(name="llama2-7b"),
    "llama2-13b": ModelConfig(name="llama2-13b", n_embd=5120, n_layer=40, n_head=40, n_head_kv=40,
                              n_ff=13824),
    "llama2-70b": ModelConfig(name="llama2-70b", n_embd=8192, n_layer=80, n_head=64, n_head_kv=8,
                              n_ff=28672),
    "mistral-7b": ModelConfig(name="mistral-7b", n_head_kv=8, n_ff=14336, ctx_len=32768,
                              rope_base=1000000.0),
    "mixtral-8x7b": ModelConfig(name="mixtral-8x7b", n_head_kv=8, n_ff=14336, ctx_len=32768,
                                rope_base=1000000.0, n_expert=8, n_expert_used=2),
    # Orca Mini 3B (reference README.md:55): OpenLLaMA-3B shapes, head dim 100; Q4_0 (its E = 3200 is not a
    # multiple of the 256-weight K-quant super-block)
    "orca-mini-3b": ModelConfig(name="orca-mini-3b", n_embd=3200, n_layer=26, n_head=32, n_head_kv=32,
                                n_ff=8640, n_rot=100, ctx_len=2048),
    "phi2": ModelConfig(name="phi2", arch="phi2", n_vocab=51200, n_embd=2560, n_layer=32, n_head=32,
                        n_head_kv=32, n_ff=10240, n_rot=32, rope_mode=ROPE_NEOX, norm_eps=1e-5,
                        ctx_len=2048, bos_id=50256, eos_id=50256),
    # Gemma (reference README.md:58-59): GeGLU, sqrt(E) embedding scale, head dim 256, MQA (2B),
    # NEOX RoPE, tied output. GGUF norm weights already carry Gemma's (1 + w) (llama.cpp converter)
    "gemma-2b": ModelConfig(name="gemma-2b", arch="gemma", n_vocab=256000, n_embd=2048, n_layer=18, n_head=8,
                            n_head_kv=1, n_ff=16384, n_rot=256, n_embd_head=256, rope_mode=ROPE_NEOX,
                            norm_eps=1e-6, ctx_len=8192, bos_id=2, eos_id=1),
    "gemma-7b": ModelConfig(name="gemma-7b", arch="gemma", n_vocab=256000, n_embd=3072, n_layer=28, n_head=16,
                            n_head_kv=16, n_ff=24576, n_rot=256, n_embd_head=256, rope_mode=ROPE_NEOX,
                            norm_eps=1e-6, ctx_len=8192, bos_id=2, eos_id=1),
    # small shapes of the same families for tests (K multiples of 256 so every quant type applies)
    "tiny-gemma": ModelConfig(name="tiny-gemma", arch="gemma", n_vocab=512, n_embd=256, n_layer=2, n_head=2,
                              n_head_kv=1, n_ff=512, n_rot=256, n_embd_head=256, rope_mode=ROPE_NEOX,
                              norm_eps=1e-6, ctx_len=256, bos_id=2, eos_id=1),
    "tiny-llama": ModelConfig(name="tiny-llama", n_vocab=512, n_embd=256, n_layer=2, n_head=4,
                              n_head_kv=2, n_ff=512, n_rot=64, ctx_len=256),
    # head dim 128 (the fused batch-1 attention half, attn8.hip): MHA and GQA 4
    "tiny-llama-d128": ModelConfig(name="tiny-llama-d128", n_vocab=512, n_embd=512, n_layer=3, n_head=4,
                                   n_head_kv=4, n_ff=768, n_rot=128, ctx_len=512),
    "tiny-llama-d128-gqa": ModelConfig(name="tiny-llama-d128-gqa", n_vocab=512, n_embd=512, n_layer=3, n_head=4,
                                       n_head_kv=1, n_ff=768, n_rot=128, ctx_len=512),
    # head dim 100 (Orca Mini), E not a multiple of 256: Q4_0 / Q8_0 files
    "tiny-orca": ModelConfig(name="tiny-orca", n_vocab=512, n_embd=800, n_layer=2, n_head=8, n_head_kv=8,
                             n_ff=2176, n_rot=100, ctx_len=256),
    "tiny-mixtral": ModelConfig(name="tiny-mixtral", n_vocab=512, n_embd=256, n_layer=2, n_head=4,
                                n_head_kv=2, n_ff=512, n_rot=64, ctx_len=256, n_expert=4,
                                n_expert_used=2),
    "tiny-phi2": ModelConfig(name="tiny-phi2", arch="phi2", n_vocab=512, n_embd=256, n_layer=2,
                             n_head=4, n_head_kv=4, n_ff=1024, n_rot=32, rope_mode=ROPE_NEOX,
                             ctx_len=256, bos_id=0, eos_id=0),
    # tensor-parallel test shapes: every row-parallel K spans >= 2 super-blocks per rank at TP=2
    "tiny-llama-tp": ModelConfig(name="tiny-llama-tp", n_vocab=512, n_embd=1024, n_layer=2, n_head=16,
                                 n_head_kv=4, n_ff=1024, n_rot=64, ctx_len=256),
    # n_ff = 3 super-blocks: TP=2 ranks hold an uneven 512 / 256 FFN split (as Llama-2-7B's 43 blocks)
    "tiny-llama-tp-odd": ModelConfig(name="tiny-llama-tp-odd", n_vocab=512, n_embd=1024, n_layer=2, n_head=16,
                                     n_head_kv=4, n_ff=768, n_rot=64, ctx_len=256),
    "tiny-phi2-tp": ModelConfig(name="tiny-phi2-tp", arch="phi2", n_vocab=512, n_embd=1024, n_layer=2,
                                n_head=16, n_head_kv=16, n_ff=2048, n_rot=32, rope_mode=ROPE_NEOX,
                                ctx_len=256, bos_id=0, eos_id=0),
    # TP = 8 (BASELINE config 4's degree, Llama-2-70B's 8:1 query / KV head ratio): one KV head, four query
    # heads, one FFN super-block and 64 vocab rows per rank
    "tiny-llama-tp8": ModelConfig(name="tiny-llama-tp8", n_vocab=512, n_embd=2048, n_layer=2, n_head=32,
                                  n_head_kv=8, n_ff=2048, n_rot=64, ctx_len=256),
    "tiny-mixtral-tp": ModelConfig(name="tiny-mixtral-tp", n_vocab=512, n_embd=1024, n_layer=2, n_head=16,
                                   n_head_kv=4, n_ff=1024, n_rot=64, ctx_len=256, n_expert=4,
                                   n_expert_used=2),
}


def preset(name: str, **overrides) -> ModelConfig:
    return replace(PRESETS[name], **overrides)
