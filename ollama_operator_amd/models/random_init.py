"""Random-init GGUF fixtures of real architectures (BASELINE.json: "synthetic prompts / random-init
GGUF weights"). Weights are drawn directly in quantized block form so a 4 GB Llama-2-7B Q4_K_M file
is produced in seconds, with the exact tensor-type mix of a real Q4_K_M conversion."""
from __future__ import annotations

import numpy as np

from ..gguf.constants import FileType, GGMLType
from ..gguf.writer import GGUFWriter
from ..quant import quantize, random_blocks
from ..tokenizer import synth_vocab_bpe, synth_vocab_spm
from .arch import tensor_specs
from .config import ModelConfig


def _norm_weight(n: int, rng: np.random.Generator) -> np.ndarray:
    return (1.0 + 0.05 * rng.standard_normal(n)).astype(np.float32)


def write_random_gguf(path: str, cfg: ModelConfig, ftype: FileType = FileType.MOSTLY_Q4_K_M,
                      seed: int = 0, std: float = 0.02, quantize_from_float: bool = False) -> dict:
    """Write a random-init model. `quantize_from_float` draws float weights and runs the reference
    quantizer (slow; small test models) instead of drawing random blocks."""
    rng = np.random.default_rng(seed)
    w = GGUFWriter(path)
    md = cfg.to_gguf_metadata()
    md["general.file_type"] = int(ftype)
    md["general.quantization_version"] = 2
    vocab = synth_vocab_bpe(cfg.n_vocab) if cfg.arch == "phi2" else synth_vocab_spm(cfg.n_vocab)
    md.update(vocab)
    for k, v in md.items():
        w.add(k, v)
    for name, shape, gt in tensor_specs(cfg, ftype):
        n = int(np.prod(shape))
        k = shape[0]
        rows = n // k
        tseed = int(rng.integers(0, 2**31))
        if name.endswith("norm.weight"):
            w.add_tensor(name, shape, gt, lambda n=n, s=tseed: _norm_weight(n, np.random.default_rng(s)))
        elif name.endswith(".bias"):
            w.add_tensor(name, shape, gt,
                         lambda n=n, s=tseed: (0.02 * np.random.default_rng(s).standard_normal(n)).astype(np.float32))
        elif name.endswith("ffn_gate_inp.weight"):
            w.add_tensor(name, shape, gt,
                         lambda n=n, s=tseed: (0.1 * np.random.default_rng(s).standard_normal(n)).astype(np.float32))
        elif quantize_from_float or gt in (GGMLType.F32, GGMLType.F16, GGMLType.BF16):
            w.add_tensor(name, shape, gt, lambda n=n, s=tseed, g=gt: quantize(
                (std * np.random.default_rng(s).standard_normal(n)).astype(np.float32), g))
        else:
            w.add_tensor(name, shape, gt, lambda r=rows, k=k, s=tseed, g=gt: random_blocks(
                g, r, k, np.random.default_rng(s), std))
    w.write()
    return md
