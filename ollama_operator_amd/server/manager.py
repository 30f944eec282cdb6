"""Loaded-model manager: lazy load on first request (reference SURVEY.md §2.4 "Lazy load
semantics": readiness only checks /api/tags), keep-alive eviction, per-model request
serialisation, stop sequences, and the Ollama timing fields (`*_duration` in ns) that clients --
and our benchmark -- read tokens/s from (eval_count / eval_duration).
"""
from __future__ import annotations

import os
import threading
import time
from dataclasses import dataclass, field
from typing import Any, Iterator

import numpy as np

from ..engine.sampling import SamplingOptions
from ..tokenizer import StreamDecoder, Tokenizer, from_gguf_metadata
from .store import MT_PROJECTOR, MT_SYSTEM, MT_TEMPLATE, ModelName, ModelStore, StoreError

DEFAULT_KEEP_ALIVE = float(os.environ.get("OLLAMA_KEEP_ALIVE_SECONDS", "300"))
DEFAULT_NUM_CTX = int(os.environ.get("OLLAMA_CONTEXT_LENGTH", "2048"))


def _cuda_available() -> bool:
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:  # noqa: BLE001
        return False


def parse_keep_alive(v: Any) -> float:
    """Ollama keep_alive: number of seconds, duration string ("5m", "1h", "30s"), <0 = forever."""
    if v is None:
        return DEFAULT_KEEP_ALIVE
    if isinstance(v, (int, float)):
        return float("inf") if v < 0 else float(v)
    s = str(v).strip()
    try:
        f = float(s)
        return float("inf") if f < 0 else f
    except ValueError:
        pass
    total = 0.0
    import re
    for num, unit in re.findall(r"(-?\d+(?:\.\d+)?)(ms|s|m|h)", s):
        total += float(num) * {"ms": 1e-3, "s": 1, "m": 60, "h": 3600}[unit]
    return float("inf") if total < 0 else total


@dataclass
class LoadedModel:
    name: ModelName
    digest: str
    path: str
    runner: Any
    tokenizer: Tokenizer
    template: str | None
    system: str | None
    params: dict
    num_ctx: int
    size: int
    load_duration_ns: int
    ctx_limit: int = 1 << 30  # the model's trained context (the runner never exceeds it)
    expires_at: float = 0.0
    lock: threading.Lock = field(default_factory=threading.Lock)
    sid: int | None = None
    scheduler: Any = None  # engine.scheduler.BatchScheduler (OLLAMA_NUM_PARALLEL > 1, single rank)
    vision: Any = None     # models.clip.ClipEncoder when the manifest has a projector layer (LLaVA)
    images: Any = None     # models.clip.ImageIds: digest-keyed negative ids of this load's images


@dataclass
class GenResult:
    text: str = ""
    done_reason: str = "stop"
    prompt_eval_count: int = 0
    prompt_eval_duration: int = 0
    eval_count: int = 0
    eval_duration: int = 0
    load_duration: int = 0
    total_duration: int = 0
    context: list = field(default_factory=list)


class ModelManager:
    def __init__(self, store: ModelStore, device: str | None = None, max_loaded: int | None = None,
                 tp_world=None):
        self.store = store
        self.device = device
        self.tp_world = tp_world  # parallel.tp.TPWorld when serving with OMX_TP > 1
        self.max_loaded = max_loaded or int(os.environ.get("OLLAMA_MAX_LOADED_MODELS", "3"))
        if tp_world is not None:
            self.max_loaded = 1  # the worker ranks hold one model
        self.loaded: dict[str, LoadedModel] = {}
        self.mu = threading.Lock()
        self.stats = {"requests": 0, "tokens_generated": 0, "prompt_tokens": 0}

    # ------------------------------------------------------------------ loading
    def _evict_expired(self):
        now = time.time()
        for k, lm in list(self.loaded.items()):
            busy = lm.lock.locked() or (lm.scheduler is not None and lm.scheduler.busy)
            if lm.expires_at <= now and not busy:
                self._unload(k)

    def _unload(self, key: str):
        lm = self.loaded.pop(key, None)
        if lm is not None:
            if lm.scheduler is not None:
                lm.scheduler.close()
            if hasattr(lm.runner, "close"):  # TP: the worker ranks drop their shards too
                lm.runner.close()
            del lm.runner
            try:
                import torch
                if torch.cuda.is_available():
                    torch.cuda.empty_cache()
            except Exception:
                pass

    def unload(self, model: str) -> bool:
        with self.mu:
            key = str(ModelName.parse(model))
            if key in self.loaded:
                self._unload(key)
                return True
            return False

    def get(self, model: str, keep_alive: Any = None, num_ctx: int | None = None) -> LoadedModel:
        name = ModelName.parse(model)
        key = str(name)
        ka = parse_keep_alive(keep_alive)
        with self.mu:
            self._evict_expired()
            m = self.store.read_manifest(name)
            lm = self.loaded.get(key)
            want_ctx = num_ctx or int(self.store.params(m).get("num_ctx", DEFAULT_NUM_CTX))
            # a larger window reloads only if the loaded one is below what was asked AND below the model's
            # own limit (the runner clamps num_ctx to the trained context: comparing against the clamped
            # value alone reloaded such a model on every request, dropping its KV prefix cache)
            if lm is not None and (lm.digest != m.digest or (want_ctx > lm.num_ctx and lm.num_ctx < lm.ctx_limit)):
                self._unload(key)
                lm = None
            if lm is None:
                while len(self.loaded) >= self.max_loaded:
                    oldest = min(self.loaded.values(), key=lambda x: x.expires_at)
                    self._unload(str(oldest.name))
                lm = self._load(name, m, want_ctx)
                self.loaded[key] = lm
            lm.expires_at = time.time() + ka
            return lm

    def _load(self, name: ModelName, m, num_ctx: int) -> LoadedModel:
        from ..engine.runner import Runner
        from ..models.clip import ImageIds
        from ..gguf import read_gguf
        t0 = time.perf_counter()
        path = self.store.model_blob(name)
        g = read_gguf(path)
        tok = from_gguf_metadata(g.metadata)
        g.close()
        ctx_cap = int(os.environ.get("OMX_MAX_CTX", "0")) or None
        ctx = min(num_ctx, ctx_cap) if ctx_cap else num_ctx
        # prefill chunk = MFMA GEMM M dimension (weights cross HBM once per chunk)
        chunk = int(os.environ.get("OMX_PREFILL_CHUNK", "2048"))  # 2048-token TTFT 117 -> 94 ms vs 512
        # multimodal (LLaVA): the projector layer's CLIP encoder runs on the leader; its patch rows enter
        # the sequence as external embedding rows (room for OMX_IMAGE_ROWS, default 8 LLaVA-1.5 images)
        vision, ext_rows = None, 0
        pl = m.layer(MT_PROJECTOR)
        if pl is not None:
            from ..models.clip import ClipEncoder
            dev = self.tp_world.device if self.tp_world is not None else (self.device or (
                "cuda" if _cuda_available() else "cpu"))
            vision = ClipEncoder(self.store.blob_path(pl["digest"]), dev)
            ext_rows = int(os.environ.get("OMX_IMAGE_ROWS", str(8 * vision.cfg.max_rows)))
        scheduler = None
        # continuous batching (Ollama OLLAMA_NUM_PARALLEL): parallel rows + as many idle sequences
        # kept for prefix reuse; KV is sized for all of them at full context (288 GB HBM)
        # default 4 as Ollama; the batched path is covered on MI355X by
        # tests/test_engine_gpu.py::test_batched_decode_matches_single / test_scheduler_concurrent_gpu
        par = max(1, int(os.environ.get("OLLAMA_NUM_PARALLEL", "4")))
        # rows: par decoding + par idle prefix-cache sequences + 1 kept free for embeddings
        max_seqs = max(2, 2 * par + 1)
        if self.tp_world is not None:  # tensor parallel: every rank loads its shard (parallel/tp.py)
            from ..parallel.tp import load_tp_runner
            runner = load_tp_runner(self.tp_world, path, max_batch=chunk, max_seqs=max_seqs, ctx=ctx,
                                    ext_rows=ext_rows)
        else:
            runner = Runner(path, device=self.device, max_batch=chunk, max_seqs=max_seqs, ctx=ctx, ext_rows=ext_rows)
        if vision is not None and vision.out_dim != runner.cfg.n_embd:
            raise StoreError(f"projector output width {vision.out_dim} != model embedding width {runner.cfg.n_embd}")
        runner.warmup()
        if par > 1:  # under TP the scheduler drives the leader's proxy; followers replay every call
            from ..engine.scheduler import BatchScheduler
            runner.capture_batch_graphs(par)
            scheduler = BatchScheduler(runner, max_parallel=par)
        return LoadedModel(name=name, digest=m.digest, path=path, runner=runner, tokenizer=tok, scheduler=scheduler,
                           vision=vision, images=ImageIds() if vision is not None else None,
                           template=self.store.text_layer(m, MT_TEMPLATE), system=self.store.text_layer(m, MT_SYSTEM),
                           params=self.store.params(m), num_ctx=runner.ctx, ctx_limit=runner.cfg.ctx_len,
                           size=os.path.getsize(path),
                           load_duration_ns=int((time.perf_counter() - t0) * 1e9))

    def ps(self) -> list[LoadedModel]:
        with self.mu:
            self._evict_expired()
            return list(self.loaded.values())

    # ------------------------------------------------------------------ generation
    def options(self, lm: LoadedModel, req_opts: dict | None) -> tuple[SamplingOptions, dict]:
        merged = dict(lm.params)
        merged.update(req_opts or {})
        return SamplingOptions.from_options(merged), merged

    def generate(self, lm: LoadedModel, prompt_ids: list[int], req_opts: dict | None, load_ns: int,
                 t_start: float) -> Iterator[tuple[str, GenResult | None]]:
        """Yields (text_piece, None) while generating and ("", GenResult) at the end."""
        from ..engine.runner import StepTimes
        so, merged = self.options(lm, req_opts)
        stops = merged.get("stop") or []
        if isinstance(stops, str):
            stops = [stops]
        num_predict = int(merged.get("num_predict", -1))
        runner = lm.runner
        room = runner.ctx - 1
        if len(prompt_ids) > room:  # Ollama truncates the prompt from the front (keeps num_keep)
            keep = int(merged.get("num_keep", 4))
            prompt_ids = prompt_ids[:keep] + prompt_ids[len(prompt_ids) - (room - keep) // 2:]
        max_new = runner.ctx - len(prompt_ids)
        if num_predict >= 0:
            max_new = min(max_new, num_predict)
        res = GenResult(load_duration=load_ns, context=list(prompt_ids))
        if max_new <= 0:
            res.done_reason = "length"
            res.total_duration = int((time.perf_counter() - t_start) * 1e9)
            yield "", res
            return
        import contextlib
        # batched models: the scheduler thread owns the runner (requests share decode steps);
        # otherwise requests to one model are serialised and reuse one sequence's KV prefix
        with (contextlib.nullcontext() if lm.scheduler is not None else lm.lock):
            times = StepTimes()
            dec = StreamDecoder(lm.tokenizer, first=not prompt_ids or prompt_ids[-1] == lm.tokenizer.bos_id)
            pending = ""
            out_text = []
            if lm.scheduler is not None:
                gen = lm.scheduler.submit(prompt_ids, so, max_tokens=max_new, times=times)
            else:
                if lm.sid is None:
                    lm.sid = runner.new_sequence()
                gen = runner.generate(lm.sid, prompt_ids, so, max_tokens=max_new, times=times)
            n = 0
            reason = "length"
            try:
                for tid in gen:
                    n += 1
                    res.context.append(tid)
                    if lm.tokenizer.is_eog(tid):
                        reason = "stop"
                        break
                    pending += dec.push(tid)
                    hit = _find_stop(pending, stops)
                    if hit is not None:
                        piece = pending[:hit]
                        if piece:
                            out_text.append(piece)
                            yield piece, None
                        pending = ""
                        reason = "stop"
                        break
                    safe = _safe_len(pending, stops)
                    if safe:
                        piece = pending[:safe]
                        pending = pending[safe:]
                        out_text.append(piece)
                        yield piece, None
                else:
                    reason = "length"
                if reason == "length":
                    pending += dec.flush()
                    if pending:
                        out_text.append(pending)
                        yield pending, None
            finally:
                gen.close()
        self.stats["requests"] += 1
        self.stats["tokens_generated"] += n
        self.stats["prompt_tokens"] += times.prompt_tokens
        res.text = "".join(out_text)
        res.done_reason = reason
        res.prompt_eval_count = times.prompt_tokens or len(prompt_ids)
        res.prompt_eval_duration = int(times.prompt_s * 1e9)
        res.eval_count = n
        res.eval_duration = int(times.gen_s * 1e9)
        res.total_duration = int((time.perf_counter() - t_start) * 1e9)
        yield "", res

    @staticmethod
    def check_context(lm: LoadedModel, ids: list) -> list[int]:
        """Client-supplied `context` ids: vocabulary tokens, or image patch ids THIS load issued (a
        negative id is a row of the shared external-embedding ring; only the registry's own ids may
        name one, so a client cannot address rows of images it never sent)."""
        out = []
        V = lm.runner.cfg.n_vocab
        for t in ids:
            if not isinstance(t, int) or isinstance(t, bool) or t >= V or (
                    t < 0 and (lm.images is None or not lm.images.issued(t))):
                raise StoreError(f"invalid context token {t!r}")
            out.append(t)
        return out

    def encode_prompt(self, lm: LoadedModel, text: str, images: list[bytes] | None = None,
                      add_bos: bool = True) -> list[int]:
        """Tokenize `text`; each `[img-N]` marker becomes image N's patch rows (negative ids registered
        with the runner). Images without a marker go in front of the text, as Ollama does for LLaVA."""
        import re
        images = list(images or [])
        if not images:
            return lm.tokenizer.encode(text, add_bos=add_bos)
        if lm.vision is None:
            raise StoreError("this model does not support images (no projector layer)")
        marks = {int(x) for x in re.findall(r"\[img-(\d+)\]", text)}
        text = "".join(f"[img-{i}]" for i in range(len(images)) if i not in marks) + text
        img_ids = []
        for data in images:
            rows = lm.vision.encode(data)
            ids = lm.images.ids_for(data, rows.shape[0])
            if lm.scheduler is not None:  # between batched decode steps, on the scheduler thread
                lm.scheduler.run_exclusive(lambda r, ids=ids, rows=rows: r.set_ext(ids, rows))
            else:
                with lm.lock:
                    lm.runner.set_ext(ids, rows)
            img_ids.append(ids)
        out: list[int] = []
        pos = 0
        for mt in re.finditer(r"\[img-(\d+)\]", text):
            seg = text[pos:mt.start()]
            if seg or not out:
                out += lm.tokenizer.encode(seg, add_bos=add_bos and not out)
            k = int(mt.group(1))
            if k >= len(img_ids):
                raise StoreError(f"prompt references [img-{k}] but only {len(img_ids)} images were given")
            out += img_ids[k]
            pos = mt.end()
        if text[pos:]:
            out += lm.tokenizer.encode(text[pos:], add_bos=False)
        return out

    def embed(self, lm: LoadedModel, texts: list[str], truncate: bool = True) -> tuple[list[list[float]], int]:
        total = 0
        out = []
        for t in texts:
            ids = lm.tokenizer.encode(t)
            if len(ids) > lm.runner.ctx:
                if not truncate:
                    raise StoreError("input length exceeds context length")
                ids = ids[:lm.runner.ctx]
            total += len(ids)
            if lm.scheduler is not None:  # between batched decode steps, on the scheduler thread
                v = lm.scheduler.run_exclusive(lambda r, ids=ids: r.embed(ids))
            else:
                with lm.lock:
                    v = lm.runner.embed(ids)
            n = float(np.linalg.norm(v)) or 1.0
            out.append([float(x) / n for x in v])
        return out, total


def _find_stop(text: str, stops: list[str]) -> int | None:
    best = None
    for s in stops:
        if not s:
            continue
        i = text.find(s)
        if i >= 0 and (best is None or i < best):
            best = i
    return best


def _safe_len(text: str, stops: list[str]) -> int:
    """Length of the prefix that cannot be the start of any stop sequence."""
    hold = 0
    for s in stops:
        for k in range(min(len(s) - 1, len(text)), 0, -1):
            if text.endswith(s[:k]):
                hold = max(hold, k)
                break
    return len(text) - hold
