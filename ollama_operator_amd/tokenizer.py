"""Tokenizers built from GGUF `tokenizer.ggml.*` metadata.

* `SPMTokenizer`  -- `tokenizer.ggml.model == "llama"`: SentencePiece-style greedy bigram merging
  by score, "▁" space marker, `<0xNN>` byte fallback (Llama 2, Mistral, Mixtral, CodeLlama ...).
* `BPETokenizer`  -- `tokenizer.ggml.model == "gpt2"`: byte-level BPE with ranked merges (Phi-2).

Also `synth_vocab_*`: deterministic vocabularies for random-init model fixtures (no network, so no
real tokenizer files exist; BASELINE.json mandates random-init GGUF weights).
"""
from __future__ import annotations

import heapq
from functools import lru_cache
from typing import Any, Sequence

import regex

SPACE = "▁"  # ▁

TOKEN_NORMAL, TOKEN_UNKNOWN, TOKEN_CONTROL, TOKEN_USER_DEFINED, TOKEN_UNUSED, TOKEN_BYTE = 1, 2, 3, 4, 5, 6


class Tokenizer:
    bos_id: int
    eos_id: int
    n_vocab: int
    add_bos: bool = True
    tokens: list[str]

    def encode(self, text: str, add_bos: bool | None = None) -> list[int]:
        raise NotImplementedError

    def decode(self, ids: Sequence[int]) -> str:
        return self.decode_bytes(ids).decode("utf-8", errors="replace")

    def decode_bytes(self, ids: Sequence[int]) -> bytes:
        raise NotImplementedError

    def is_eog(self, tid: int) -> bool:
        return tid == self.eos_id or tid in getattr(self, "eog_ids", ())


class StreamDecoder:
    """Incremental detokenizer: yields only complete UTF-8 text (multi-byte chars can straddle
    tokens, e.g. byte-fallback pieces)."""

    def __init__(self, tok: Tokenizer, first: bool = True):
        self.tok = tok
        self.pending = b""
        self.first = first

    def push(self, tid: int) -> str:
        b = self.tok.piece_bytes(tid, self.first)  # type: ignore[attr-defined]
        self.first = False
        self.pending += b
        try:
            s = self.pending.decode("utf-8")
            self.pending = b""
            return s
        except UnicodeDecodeError as e:
            if e.start > 0:
                s = self.pending[: e.start].decode("utf-8")
                self.pending = self.pending[e.start:]
                return s
            if len(self.pending) > 8:
                s = self.pending.decode("utf-8", errors="replace")
                self.pending = b""
                return s
            return ""

    def flush(self) -> str:
        s = self.pending.decode("utf-8", errors="replace")
        self.pending = b""
        return s


class SPMTokenizer(Tokenizer):
    def __init__(self, tokens: list[str], scores: list[float] | None, types: list[int] | None,
                 bos_id: int = 1, eos_id: int = 2, unk_id: int = 0, add_bos: bool = True,
                 add_space_prefix: bool = True):
        self.tokens = tokens
        self.scores = scores or [0.0] * len(tokens)
        self.types = types or [TOKEN_NORMAL] * len(tokens)
        self.n_vocab = len(tokens)
        self.bos_id, self.eos_id, self.unk_id = bos_id, eos_id, unk_id
        self.add_bos = add_bos
        self.add_space_prefix = add_space_prefix
        self.vocab = {t: i for i, t in enumerate(tokens)}
        self.byte_ids = {}
        for i, (t, ty) in enumerate(zip(tokens, self.types)):
            if ty == TOKEN_BYTE and len(t) == 6 and t.startswith("<0x"):
                self.byte_ids[int(t[3:5], 16)] = i
        self.specials = {t: i for i, (t, ty) in enumerate(zip(tokens, self.types))
                         if ty in (TOKEN_CONTROL, TOKEN_USER_DEFINED) and len(t) > 1}

    def _encode_fragment(self, text: str) -> list[int]:
        if not text:
            return []
        syms = list(text)
        n = len(syms)
        prev = list(range(-1, n - 1))
        nxt = list(range(1, n + 1))
        nxt[-1] = -1
        alive = [True] * n
        heap: list[tuple[float, int, int, str]] = []

        def push(i: int):
            j = nxt[i]
            if j == -1:
                return
            cat = syms[i] + syms[j]
            tid = self.vocab.get(cat)
            if tid is not None:
                heapq.heappush(heap, (-self.scores[tid], i, j, cat))

        for i in range(n - 1):
            push(i)
        while heap:
            _, i, j, cat = heapq.heappop(heap)
            if not alive[i] or not alive[j] or nxt[i] != j or syms[i] + syms[j] != cat:
                continue
            syms[i] = cat
            alive[j] = False
            nxt[i] = nxt[j]
            if nxt[j] != -1:
                prev[nxt[j]] = i
            if prev[i] != -1:
                push(prev[i])
            push(i)
        out = []
        i = 0
        while i != -1 and i < n:
            if alive[i]:
                tid = self.vocab.get(syms[i])
                if tid is None:
                    for byte in syms[i].encode("utf-8"):
                        out.append(self.byte_ids.get(byte, self.unk_id))
                else:
                    out.append(tid)
            i = nxt[i]
        return out

    def encode(self, text: str, add_bos: bool | None = None) -> list[int]:
        ids: list[int] = []
        if self.add_bos if add_bos is None else add_bos:
            ids.append(self.bos_id)
        # split out special tokens written literally in the text (e.g. "</s>" in templates)
        parts = _split_specials(text, self.specials)
        first = True
        for p in parts:
            if isinstance(p, int):
                ids.append(p)
                first = False
                continue
            s = p.replace(" ", SPACE)
            if first and self.add_space_prefix:
                s = SPACE + s
            first = False
            ids.extend(self._encode_fragment(s))
        return ids

    def piece_bytes(self, tid: int, first: bool = False) -> bytes:
        if tid < 0 or tid >= self.n_vocab:
            return b""
        ty = self.types[tid]
        t = self.tokens[tid]
        if ty == TOKEN_BYTE:
            return bytes([int(t[3:5], 16)])
        if ty in (TOKEN_CONTROL, TOKEN_UNKNOWN):
            return b""
        s = t.replace(SPACE, " ")
        if first and self.add_space_prefix and s.startswith(" "):
            s = s[1:]
        return s.encode("utf-8")

    def decode_bytes(self, ids: Sequence[int]) -> bytes:
        out = bytearray()
        first = True
        for t in ids:
            if t == self.bos_id and first:
                continue
            out += self.piece_bytes(int(t), first)
            first = False
        return bytes(out)


@lru_cache(maxsize=1)
def bytes_to_unicode() -> dict[int, str]:
    bs = list(range(ord("!"), ord("~") + 1)) + list(range(ord("¡"), ord("¬") + 1)) + \
        list(range(ord("®"), ord("ÿ") + 1))
    cs = bs[:]
    n = 0
    for b in range(256):
        if b not in bs:
            bs.append(b)
            cs.append(256 + n)
            n += 1
    return {b: chr(c) for b, c in zip(bs, cs)}


GPT2_PRETOKENIZE = regex.compile(
    r"""'s|'t|'re|'ve|'m|'ll|'d| ?\p{L}+| ?\p{N}+| ?[^\s\p{L}\p{N}]+|\s+(?!\S)|\s+""")


class BPETokenizer(Tokenizer):
    def __init__(self, tokens: list[str], merges: list[str], types: list[int] | None = None,
                 bos_id: int = 50256, eos_id: int = 50256, add_bos: bool = False):
        self.tokens = tokens
        self.n_vocab = len(tokens)
        self.types = types or [TOKEN_NORMAL] * len(tokens)
        self.vocab = {t: i for i, t in enumerate(tokens)}
        self.ranks = {}
        for r, m in enumerate(merges):
            a, _, b = m.partition(" ")
            self.ranks[(a, b)] = r
        self.bos_id, self.eos_id = bos_id, eos_id
        self.add_bos = add_bos
        self.b2u = bytes_to_unicode()
        self.u2b = {v: k for k, v in self.b2u.items()}
        self.specials = {t: i for i, (t, ty) in enumerate(zip(tokens, self.types))
                         if ty in (TOKEN_CONTROL, TOKEN_USER_DEFINED)}
        self._cache: dict[str, list[int]] = {}

    def _bpe(self, word: str) -> list[int]:
        hit = self._cache.get(word)
        if hit is not None:
            return hit
        parts = list(word)
        while len(parts) > 1:
            best = None
            for k in range(len(parts) - 1):
                r = self.ranks.get((parts[k], parts[k + 1]))
                if r is not None and (best is None or r < best[0]):
                    best = (r, k)
            if best is None:
                break
            k = best[1]
            parts[k:k + 2] = [parts[k] + parts[k + 1]]
        ids = []
        for p in parts:
            tid = self.vocab.get(p)
            if tid is None:  # fall back to single byte-chars
                ids.extend(self.vocab[c] for c in p if c in self.vocab)
            else:
                ids.append(tid)
        if len(self._cache) < 100000:
            self._cache[word] = ids
        return ids

    def encode(self, text: str, add_bos: bool | None = None) -> list[int]:
        ids: list[int] = []
        if self.add_bos if add_bos is None else add_bos:
            ids.append(self.bos_id)
        for p in _split_specials(text, self.specials):
            if isinstance(p, int):
                ids.append(p)
                continue
            for w in GPT2_PRETOKENIZE.findall(p):
                ids.extend(self._bpe("".join(self.b2u[b] for b in w.encode("utf-8"))))
        return ids

    def piece_bytes(self, tid: int, first: bool = False) -> bytes:
        if tid < 0 or tid >= self.n_vocab:
            return b""
        if self.types[tid] == TOKEN_CONTROL:
            return b""
        t = self.tokens[tid]
        if self.types[tid] == TOKEN_USER_DEFINED:
            return t.encode("utf-8")
        return bytes(self.u2b[c] for c in t if c in self.u2b)

    def decode_bytes(self, ids: Sequence[int]) -> bytes:
        return b"".join(self.piece_bytes(int(t)) for t in ids)


def _split_specials(text: str, specials: dict[str, int]) -> list[Any]:
    if not specials:
        return [text]
    pat = _special_pattern(tuple(sorted(specials, key=len, reverse=True)))
    out: list[Any] = []
    pos = 0
    for m in pat.finditer(text):
        if m.start() > pos:
            out.append(text[pos:m.start()])
        out.append(specials[m.group(0)])
        pos = m.end()
    if pos < len(text):
        out.append(text[pos:])
    return out


@lru_cache(maxsize=16)
def _special_pattern(keys: tuple[str, ...]):
    return regex.compile("|".join(regex.escape(k) for k in keys))


def from_gguf_metadata(md: dict[str, Any]) -> Tokenizer:
    model = md.get("tokenizer.ggml.model", "llama")
    tokens = list(md["tokenizer.ggml.tokens"])
    types = md.get("tokenizer.ggml.token_type")
    bos = int(md.get("tokenizer.ggml.bos_token_id", 1))
    eos = int(md.get("tokenizer.ggml.eos_token_id", 2))
    if model == "gpt2":
        tok: Tokenizer = BPETokenizer(tokens, list(md.get("tokenizer.ggml.merges", [])), types, bos, eos,
                                      add_bos=bool(md.get("tokenizer.ggml.add_bos_token", False)))
    else:
        tok = SPMTokenizer(tokens, md.get("tokenizer.ggml.scores"), types, bos, eos,
                           int(md.get("tokenizer.ggml.unknown_token_id", 0)),
                           add_bos=bool(md.get("tokenizer.ggml.add_bos_token", True)),
                           add_space_prefix=bool(md.get("tokenizer.ggml.add_space_prefix", True)))
    eot = md.get("tokenizer.ggml.eot_token_id")
    tok.eog_ids = {int(eot)} if eot is not None else set()  # type: ignore[attr-defined]
    return tok


# ----------------------------------------------------------------------------------------------
# synthetic vocabularies for random-init fixtures
# ----------------------------------------------------------------------------------------------

_WORDS = (
    "the of and to in is you that it he was for on are as with his they at be this have from or one "
    "had by word but not what all were we when your can said there use an each which she do how their "
    "if will up other about out many then them these so some her would make like him into time has "
    "look two more write go see number no way could people my than first water been call who oil its "
    "now find long down day did get come made may part hello hi world model llama ollama kubernetes "
    "operator gpu amd instinct server token stream chat answer question help sure thanks good great "
    "why sky blue because light scattering sun short wavelength red yellow green code python function "
    "return print def class import value list string number data file name new old big small think "
    "know want work need very just over also back after where most only any give our under right"
).split()


def _alpha_pieces():
    letters = "etaoinshrdlcumwfgypbvkjxqz"
    for a in letters:
        for b in letters:
            yield a + b
    for a in letters[:16]:
        for b in letters[:16]:
            for c in letters[:12]:
                yield a + b + c


def synth_vocab_spm(n_vocab: int) -> dict[str, Any]:
    tokens = ["<unk>", "<s>", "</s>"]
    types = [TOKEN_UNKNOWN, TOKEN_CONTROL, TOKEN_CONTROL]
    tokens += [f"<0x{b:02X}>" for b in range(256)]
    types += [TOKEN_BYTE] * 256
    seen = set(tokens)
    pieces: list[str] = []

    def add(p: str):
        if p not in seen and len(tokens) + len(pieces) < n_vocab:
            seen.add(p)
            pieces.append(p)

    add(SPACE)
    for ch in "etaoinshrdlcumwfgypbvkjxqzETAOINSHRDLCUMWFGYPBVKJXQZ0123456789.,!?'\"-:;()":
        add(ch)
    for ch in "etaoinshrdlcumwfgypbvkjxqz":
        add(SPACE + ch)
    for w in _WORDS:
        for k in range(2, len(w) + 1):
            add(SPACE + w[:k])
    for w in _WORDS:
        for k in range(2, len(w) + 1):
            add(w[:k])
    for p in _alpha_pieces():
        add(p)
        add(SPACE + p)
    i = 0
    while len(tokens) + len(pieces) < n_vocab:
        add(f"<extra_{i}>")
        i += 1
    tokens += pieces
    types += [TOKEN_NORMAL] * len(pieces)
    scores = [0.0] * 259 + [-float(i) for i in range(len(pieces))]
    return {"tokenizer.ggml.model": "llama", "tokenizer.ggml.tokens": tokens,
            "tokenizer.ggml.scores": scores, "tokenizer.ggml.token_type": types,
            "tokenizer.ggml.bos_token_id": 1, "tokenizer.ggml.eos_token_id": 2,
            "tokenizer.ggml.unknown_token_id": 0, "tokenizer.ggml.add_bos_token": True}


def synth_vocab_bpe(n_vocab: int) -> dict[str, Any]:
    b2u = bytes_to_unicode()
    tokens = [b2u[b] for b in range(256)]
    seen = set(tokens)
    merges: list[str] = []
    G = b2u[ord(" ")]
    n_special = 1

    ranks: dict[tuple[str, str], int] = {}

    def add_word(w: str):
        # run the BPE learned so far, then add merges for what is left: keeps the merge table
        # consistent (every word merges into one token under rank-ordered application)
        parts = list(w)
        while len(parts) > 1:
            best = None
            for k in range(len(parts) - 1):
                r = ranks.get((parts[k], parts[k + 1]))
                if r is not None and (best is None or r < best[0]):
                    best = (r, k)
            if best is None:
                break
            k = best[1]
            parts[k:k + 2] = [parts[k] + parts[k + 1]]
        while len(parts) > 1:
            a, b = parts[0], parts[1]
            nxt = a + b
            if len(tokens) >= n_vocab - n_special:
                return
            ranks[(a, b)] = len(merges)
            merges.append(f"{a} {b}")
            if nxt not in seen:
                seen.add(nxt)
                tokens.append(nxt)
            parts[0:2] = [nxt]

    for w in _WORDS:
        add_word(G + w)
        add_word(w)
    for p in _alpha_pieces():
        add_word(G + p)
    i = 0
    while len(tokens) < n_vocab - n_special:
        tokens.append(f"[PAD{i}]")
        i += 1
    eos = len(tokens)
    tokens.append("<|endoftext|>")
    types = [TOKEN_NORMAL] * (len(tokens) - 1) + [TOKEN_CONTROL]
    return {"tokenizer.ggml.model": "gpt2", "tokenizer.ggml.tokens": tokens,
            "tokenizer.ggml.token_type": types, "tokenizer.ggml.merges": merges,
            "tokenizer.ggml.bos_token_id": eos, "tokenizer.ggml.eos_token_id": eos,
            "tokenizer.ggml.add_bos_token": False}
