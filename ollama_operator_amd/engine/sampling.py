"""Sampling options (Ollama `options` names and defaults) and the host twin of the on-device
sampler (csrc/kernels/sampling.hip), used by the CPU backend and as the test oracle."""
from __future__ import annotations

import math
import random
from dataclasses import dataclass, fields

import numpy as np

MASK64 = (1 << 64) - 1


@dataclass
class SamplingOptions:
    temperature: float = 0.8
    top_k: int = 40
    top_p: float = 0.9
    min_p: float = 0.0
    repeat_penalty: float = 1.1
    repeat_last_n: int = 64
    presence_penalty: float = 0.0
    frequency_penalty: float = 0.0
    seed: int | None = None

    @classmethod
    def from_options(cls, opts: dict | None) -> "SamplingOptions":
        o = cls()
        if not opts:
            return o
        for f in fields(cls):
            if f.name in opts and opts[f.name] is not None:
                v = opts[f.name]
                if f.name == "seed":
                    v = int(v)
                    if v < 0:
                        v = None
                elif f.type in ("int", int):
                    v = int(v)
                else:
                    v = float(v)
                setattr(o, f.name, v)
        return o

    def resolved_seed(self) -> int:
        return (self.seed if self.seed is not None else random.getrandbits(63)) & MASK64


def splitmix64(x: int) -> int:
    x = (x + 0x9E3779B97F4A7C15) & MASK64
    x = ((x ^ (x >> 30)) * 0xBF58476D1CE4E5B9) & MASK64
    x = ((x ^ (x >> 27)) * 0x94D049BB133111EB) & MASK64
    return x ^ (x >> 31)


def uniform(seed: int, step: int) -> float:
    r = splitmix64((seed ^ ((0xD1B54A32D192ED03 * (step + 1)) & MASK64)) & MASK64)
    return (r >> 40) * (1.0 / 16777216.0)


def apply_penalties(logits: np.ndarray, history: list[int], o: SamplingOptions) -> None:
    win = history[-o.repeat_last_n:] if o.repeat_last_n > 0 else []
    if not win or (o.repeat_penalty == 1.0 and o.presence_penalty == 0.0 and o.frequency_penalty == 0.0):
        return
    counts: dict[int, int] = {}
    for t in win:
        counts[t] = counts.get(t, 0) + 1
    for t, c in counts.items():
        if 0 <= t < logits.shape[0]:
            v = float(logits[t])
            if o.repeat_penalty != 1.0:
                v = v / o.repeat_penalty if v > 0 else v * o.repeat_penalty
            v -= c * o.frequency_penalty + o.presence_penalty
            logits[t] = v


def top_k_stable(lg: np.ndarray, k: int) -> np.ndarray:
    """The first k of a stable descending argsort (ties by lower index), in O(V): partition, then
    sort only the candidates (the CPU backend samples 51,200-entry Phi-2 logits per token)."""
    if k >= lg.shape[0]:
        return np.argsort(-lg, kind="stable")[:k]
    part = np.argpartition(-lg, k - 1)[:k]
    vk = lg[part].min()
    greater = np.nonzero(lg > vk)[0]
    equal = np.nonzero(lg == vk)[0][:k - len(greater)]
    cand = np.concatenate([greater, equal])
    return cand[np.lexsort((cand, -lg[cand]))]


def sample_host(logits: np.ndarray, history: list[int], o: SamplingOptions, seed: int, step: int) -> int:
    lg = np.array(logits, dtype=np.float32, copy=True)
    apply_penalties(lg, history, o)
    if o.temperature <= 0:
        return int(np.argmax(lg))
    k = o.top_k if 0 < o.top_k <= 1024 else 1024
    k = min(k, lg.shape[0])
    idx = top_k_stable(lg, k)
    vals = lg[idx].astype(np.float64)
    top = vals[0]
    p1 = np.exp(vals - top)
    p1 /= p1.sum()
    keep = k
    if o.top_p < 1.0:
        c = np.cumsum(p1)
        hit = np.nonzero(c >= o.top_p)[0]
        if len(hit):
            keep = int(hit[0]) + 1
    if o.min_p > 0:
        j = 1
        while j < keep and math.exp(vals[j] - top) >= o.min_p:
            j += 1
        keep = j
    w = np.exp((vals[:keep] - top) / o.temperature)
    u = uniform(seed, step) * w.sum()
    c = np.cumsum(w)
    pick = int(np.searchsorted(c, u, side="right"))
    return int(idx[min(pick, keep - 1)])
