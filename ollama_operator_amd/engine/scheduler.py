"""Continuous batching: several requests to one loaded model decode together, one batched step per token.

Ollama serves `OLLAMA_NUM_PARALLEL` requests per model at once (its runner keeps that many "slots",
each with its own KV cache and prefix reuse). The reference operator inherits that from the external
`ollama/ollama` image (reference pkg/model/pod.go:10-12); here it is native: one scheduler thread per
loaded model owns the `Runner` and

* admits queued requests into free rows (up to `max_parallel`), reusing the idle sequence whose KV holds
  the longest common prefix with the new prompt (multi-turn chats skip the shared history);
* prefills the new prompt, samples its first token with the request's own sampler state; while other
  rows are decoding, admission is INTERLEAVED: the new prompts go through in chunks of `chunk` tokens, and
  every chunk's forward also carries each running row's next decode token (one more row of the same
  step), so running streams keep producing a token per chunk instead of stalling for the whole burst's
  prefill;
* coalesces a burst: when nothing is decoding, the first arrival waits (at most `coalesce_ms`, and only
  while requests keep arriving within `quiet_ms`) for the rest of the burst, so simultaneous clients
  prefill in one forward and start decoding together;
* runs batched decode steps for every active row (`Runner.decode_batch`: B rows through the batched
  GEMV + paged GQA attention + per-row on-device sampling, one hipGraph per B), keeping two steps in
  flight while the batch composition is stable -- the sampled tokens feed back on device, exactly as
  the batch-1 pipelined path does -- and draining only when a request joins, finishes or is cancelled;
* restores every row's sampler state (penalty history, seeded RNG counter) when rows are recomposed, so a
  request's random draws do not depend on who else is in the batch.

Failure semantics: a step that raises fails only the requests it carried (their rows are freed) and the
loop goes on; a closed or dead scheduler rejects new work immediately and fails everything queued, so no
caller ever blocks on a scheduler that will not answer.

The same code drives the torch twin on CPU (tests), where steps are simply synchronous.
"""
from __future__ import annotations

import collections
import os
import queue
import threading
import time
from dataclasses import dataclass, field
from typing import Callable, Iterator

import torch

from .runner import Runner, StepTimes
from .sampling import SamplingOptions

_DONE = object()


class SchedulerClosed(RuntimeError):
    pass


@dataclass
class _Req:
    prompt: list[int]
    opts: SamplingOptions
    seed: int
    max_tokens: int
    times: StepTimes | None
    out: "queue.Queue" = field(default_factory=queue.Queue)
    cancelled: threading.Event = field(default_factory=threading.Event)
    sid: int | None = None
    history: list[int] = field(default_factory=list)  # prompt + sampled tokens (penalties)
    n_sampled: int = 0          # RNG draws made (first token included)
    pos: int = 0                # next position to issue (input token's position)
    issued: int = 0             # decode steps issued (each yields one token)
    delivered: int = 0          # tokens handed to the consumer
    last_input: int = 0         # input token of the oldest unconsumed step
    t_gen0: float = 0.0

    def finished(self) -> bool:
        return self.delivered >= self.max_tokens or self.cancelled.is_set()


class BatchScheduler:
    """Per-model continuous-batching loop (see module docstring)."""

    def __init__(self, runner: Runner, max_parallel: int = 4, depth: int = 2, chunk: int | None = None,
                 coalesce_ms: float | None = None, quiet_ms: float | None = None):
        # tensor parallel: `runner` is the leader's TPRunnerProxy; every runner call below is mirrored to
        # the follower ranks (parallel/tp.py), which replay the leader's decisions step for step
        self.r = runner
        # one KV row stays reserved for exclusive jobs (embeddings) even when every row decodes
        self.max_parallel = max(1, min(max_parallel, runner.max_batch, runner.max_seqs - 1))
        self.max_idle = max(0, runner.max_seqs - self.max_parallel - 1)  # prefix cache rows
        self.depth = depth if runner.is_gpu else 1  # steps in flight
        # interleaved admission: prompt tokens per mixed forward (0 = one forward for the whole burst)
        env = os.environ.get
        self.chunk = int(env("OMX_ADMIT_CHUNK", "256")) if chunk is None else chunk
        # burst coalescing (0 = admit the first arrival at once)
        self.coalesce_ms = float(env("OMX_ADMIT_COALESCE_MS", "10")) if coalesce_ms is None else coalesce_ms
        self.quiet_ms = float(env("OMX_ADMIT_QUIET_MS", "3")) if quiet_ms is None else quiet_ms
        self.interleaved_chunks = 0  # mixed forwards run (tests, /api/ps diagnostics)
        self.cv = threading.Condition()
        self.pending: collections.deque[_Req] = collections.deque()
        self.jobs: collections.deque = collections.deque()  # exclusive runner work (embeddings)
        self.active: list[_Req] = []
        self.idle: list[int] = []  # sequences kept for prefix reuse, most recent last
        self.closed = False
        self.steps = 0
        self.failed_steps = 0
        self.max_batch_seen = 0
        self._ring = None
        self._thread = threading.Thread(target=self._loop, name="omx-batch", daemon=True)
        self._thread.start()

    # ------------------------------------------------------------------ public API
    def _check_open(self) -> None:
        if self.closed or not self._thread.is_alive():
            raise SchedulerClosed("scheduler closed")

    def submit(self, prompt: list[int], options: SamplingOptions | None = None, max_tokens: int = 128,
               times: StepTimes | None = None) -> Iterator[int]:
        """Queue a generation; yields its tokens as the batched steps produce them. Closing the
        iterator early (stop string, client gone) cancels the request and frees its row."""
        o = options or SamplingOptions()
        req = _Req(prompt=list(prompt), opts=o, seed=o.resolved_seed(), max_tokens=max(0, max_tokens), times=times)
        with self.cv:
            self._check_open()
            self.pending.append(req)
            self.cv.notify()
        return self._consume(req, times)

    def _consume(self, req: _Req, times: StepTimes | None) -> Iterator[int]:
        n, t1 = 0, None
        try:
            while True:
                item = req.out.get()
                if item is _DONE:
                    return
                if isinstance(item, BaseException):
                    raise item
                if t1 is None:  # eval timing as Runner.generate: from the first token on
                    t1 = time.perf_counter()
                n += 1
                yield item
        finally:
            req.cancelled.set()
            if times is not None:
                times.gen_tokens = n
                times.gen_s = time.perf_counter() - t1 if t1 is not None else 0.0
            with self.cv:
                self.cv.notify()

    def run_exclusive(self, fn: Callable[[Runner], object]):
        """Run fn(runner) on the scheduler thread between steps (embeddings share the runner)."""
        box: queue.Queue = queue.Queue()
        with self.cv:
            self._check_open()
            self.jobs.append((fn, box))
            self.cv.notify()
        ok, val = box.get()
        if not ok:
            raise val
        return val

    @property
    def busy(self) -> bool:
        return bool(self.active or self.pending or self.jobs)

    def close(self) -> None:
        with self.cv:
            self.closed = True
            self.cv.notify()
        self._thread.join(timeout=30)

    # ------------------------------------------------------------------ scheduler thread
    def _loop(self) -> None:
        err: BaseException = SchedulerClosed("scheduler closed")
        try:
            while True:
                with self.cv:
                    while not (self.closed or self.pending or self.jobs or self.active):
                        self.cv.wait()
                    if self.closed:
                        break
                    self._coalesce()
                    jobs = list(self.jobs)
                    self.jobs.clear()
                for fn, box in jobs:
                    self._run_job(fn, box)
                try:
                    self._admit()
                    if self.active:
                        self._run_stable()
                except Exception as e:  # noqa: BLE001 -- fail the rows this step carried, keep serving
                    self.failed_steps += 1
                    self._fail_active(e)
        except BaseException as e:  # noqa: BLE001 -- the loop itself died: nobody may wait on it
            err = e
            raise
        finally:
            self._shutdown(err)

    def _coalesce(self) -> None:
        """(cv held) Nothing decodes and requests are queued: give a burst's stragglers up to
        coalesce_ms to arrive, ending early once no new request came for quiet_ms or the rows are full."""
        if self.coalesce_ms <= 0 or self.active or not self.pending or self.jobs:
            return
        deadline = time.perf_counter() + self.coalesce_ms / 1e3
        while not self.closed and len(self.pending) < self.max_parallel:
            n = len(self.pending)
            left = deadline - time.perf_counter()
            if left <= 0:
                return
            self.cv.wait(min(left, self.quiet_ms / 1e3))
            if len(self.pending) == n:  # quiet: the burst is over
                return

    def _run_job(self, fn, box) -> None:
        kv = self.r.kv
        if not kv.rows_free and self.idle:  # every row taken: give the job the LRU prefix-cache row
            self.r.free_sequence(self.idle.pop(0))
        try:
            box.put((True, fn(self.r)))
        except BaseException as e:  # noqa: BLE001 -- handed to the caller
            box.put((False, e))

    def _fail_active(self, e: BaseException) -> None:
        for req in self.active:
            req.out.put(e)
            if req.sid is not None and req.sid in self.r.kv.seqs:
                self.r.free_sequence(req.sid)
        self.active.clear()

    def _shutdown(self, e: BaseException) -> None:
        with self.cv:
            self.closed = True
            reqs = list(self.active) + list(self.pending)
            jobs = list(self.jobs)
            self.active.clear()
            self.pending.clear()
            self.jobs.clear()
        for req in reqs:
            req.out.put(e)
        for _, box in jobs:
            box.put((False, e if isinstance(e, Exception) else SchedulerClosed("scheduler closed")))

    def _take_sequence(self, prompt: list[int]) -> tuple[int, int]:
        """(sid, reusable prefix length): the idle sequence sharing the longest prefix, else a fresh one
        (evicting the least recently used idle sequence when every KV row is taken)."""
        kv = self.r.kv
        best, keep = None, -1
        for sid in self.idle:
            n = kv.common_prefix(kv.seqs[sid].tokens, prompt)
            if n > keep:
                best, keep = sid, n
        if best is not None and keep > 0:
            self.idle.remove(best)
            return best, keep
        if not kv.rows_free and self.idle:
            self.r.evict(self.idle.pop(0))
        return self.r.new_sequence(), 0

    def _admit(self) -> None:
        """Admit every queued request that fits; several at once prefill in ONE forward
        (Runner.admit_many: their prompt rows are independent rows of one step), so a burst of
        arrivals stalls the running rows once, not once per request."""
        r = self.r
        while True:
            batch = []
            with self.cv:
                while self.pending and len(self.active) + len(batch) < self.max_parallel:
                    batch.append(self.pending.popleft())
            if not batch:
                return
            ready = []
            for req in batch:
                if req.cancelled.is_set() or req.max_tokens <= 0:
                    req.out.put(_DONE)
                    continue
                try:
                    sid, keep = self._take_sequence(req.prompt)
                except BaseException as e:  # noqa: BLE001 -- this request fails, the batch goes on
                    req.out.put(e)
                    continue
                req.sid = sid
                ready.append((req, min(keep, len(req.prompt) - 1)))
            if not ready:
                continue
            t0 = time.perf_counter()
            # per-request checks first (unregistered image ids, context overflow): a bad request fails
            # alone instead of failing the whole burst's shared forward
            ok = []
            for req, keep in ready:
                try:
                    r.check_admit(req.sid, keep, req.prompt[keep:])
                    ok.append((req, keep))
                except ValueError as e:
                    self._fail_req(req, e)
            if ok and self.active and self.chunk > 0:
                self._admit_interleaved(ok, t0)
                continue
            done, firsts = [], []
            if len(ok) <= 1 or sum(len(q.prompt) - k for q, k in ok) > r.max_batch or len(ok) > r.max_batch:
                for req, keep in ok:  # one forward each: a failure stays with its request
                    try:
                        r.admit(req.sid, keep, req.prompt[keep:], req.opts, req.prompt, req.seed)
                        firsts.append(int(r.s_out[0].item()))
                        done.append((req, keep))
                    except BaseException as e:  # noqa: BLE001
                        self._fail_req(req, e)
            else:
                try:
                    firsts = r.admit_many([(req.sid, keep, req.prompt[keep:], req.opts, req.prompt, req.seed)
                                           for req, keep in ok])
                    done = ok
                except BaseException as e:  # noqa: BLE001 -- the shared forward failed: its requests fail
                    for req, _ in ok:
                        self._fail_req(req, e)
            t1 = time.perf_counter()
            for (req, keep), first in zip(done, firsts):
                self._started(req, keep, first, t0, t1)

    def _started(self, req: _Req, keep: int, first: int, t0: float, t1: float) -> None:
        """A request's prompt is in: record its first token and make it a decoding row."""
        req.n_sampled = 1
        req.history = list(req.prompt) + [first]
        req.pos = self.r.kv.seqs[req.sid].length
        req.max_tokens = min(req.max_tokens, self.r.ctx - req.pos)
        req.last_input = first
        req.t_gen0 = t1
        if req.times is not None:
            req.times.prompt_tokens = len(req.prompt) - keep
            req.times.prompt_s = t1 - t0
        self._deliver(req, first)
        if req.finished():
            self._retire(req)
        else:
            self.active.append(req)

    def _admit_interleaved(self, ok: list[tuple[_Req, int]], t0: float) -> None:
        """Admit `ok` while rows are decoding: their prompts in chunks of self.chunk tokens, each chunk
        ONE forward (Runner.admit_many) that also carries every running row's next decode token. A
        running row gets its token from each chunk; an admitted request joins the running rows (and the
        next chunks) as soon as its last chunk is in."""
        r = self.r
        work = [[req, keep, 0] for req, keep in ok]  # request, prefix kept, prompt tokens done
        while work:
            rows = [q for q in self.active if not q.finished() and q.issued < q.max_tokens - 1]
            budget = max(1, min(self.chunk, r.max_batch - len(rows)))
            items, roles = [], []
            for q in rows:
                items.append((q.sid, r.kv.seqs[q.sid].length, [q.last_input], q.opts, q.history, q.seed, q.n_sampled))
                roles.append(q)
            for w in work:
                if budget <= 0:
                    break
                req, keep, off = w
                rest = len(req.prompt) - keep - off
                take = min(rest, budget)
                items.append((req.sid, keep + off, req.prompt[keep + off: keep + off + take], req.opts, req.prompt,
                              req.seed, 0))
                roles.append((w, take == rest))
                w[2] += take
                budget -= take
            try:
                outs = r.admit_many(items)
            except BaseException as e:  # noqa: BLE001 -- the shared forward failed: every row in it fails
                for w in work:
                    self._fail_req(w[0], e)
                self._fail_active(e)
                return
            self.interleaved_chunks += 1
            t1 = time.perf_counter()
            for role, tok in zip(roles, outs):
                if isinstance(role, _Req):  # a running row's decode step
                    q = role
                    q.pos += 1
                    q.issued += 1
                    q.last_input = tok
                    q.history.append(tok)
                    q.n_sampled += 1
                    if not q.cancelled.is_set():
                        self._deliver(q, tok)
                elif role[1]:  # the request's last chunk: its first token
                    w = role[0]
                    work.remove(w)
                    self._started(w[0], w[1], tok, t0, t1)
            for q in [q for q in self.active if q.finished()]:
                self.active.remove(q)
                self._retire(q)

    def _fail_req(self, req: _Req, e: BaseException) -> None:
        if req.sid is not None and req.sid in self.r.kv.seqs:
            self.r.free_sequence(req.sid)
        req.out.put(e)

    def _deliver(self, req: _Req, tok: int) -> None:
        req.delivered += 1
        req.out.put(tok)

    def _retire(self, req: _Req) -> None:
        # a sample since the last check met non-finite logits (the sampler clamped the id): that request's
        # stream is not valid output -- fail it loudly rather than end it as a normal completion
        err = getattr(self.r, "sampler_error", None)
        if err is not None and err():
            req.out.put(RuntimeError("sampling met non-finite logits (numerical fault upstream); the generated "
                                     "tokens are invalid"))
        else:
            req.out.put(_DONE)
        if req.sid is not None:
            self.idle.append(req.sid)
            while len(self.idle) > self.max_idle:  # bounded prefix cache
                self.r.free_sequence(self.idle.pop(0))

    def _recompose(self) -> None:
        """Rows changed: upload every row's next input token and sampler state (history, RNG step)."""
        self.r.recompose([(req.opts, req.history, req.seed, req.n_sampled) for req in self.active],
                         [req.last_input for req in self.active])

    def _must_drain(self, rows: list[_Req]) -> bool:
        """Stop issuing (drain in-flight steps, then recompose) only when the composition must change:
        a row finished, an exclusive job or close is waiting, or a queued request can actually be
        admitted. Under overload (every row busy) pending requests do not break the pipelining."""
        if any(q.finished() for q in rows) or self.jobs or self.closed:
            return True
        return bool(self.pending) and len(self.active) < self.max_parallel

    def _run_stable(self) -> None:
        """Decode steps for the current rows, `depth` in flight, until the composition must change;
        then drain so the next composition starts from known tokens."""
        r = self.r
        rows = list(self.active)
        B = len(rows)
        self.max_batch_seen = max(self.max_batch_seen, B)
        self._recompose()
        if self._ring is None and r.is_gpu:
            self._ring = [torch.zeros(r.max_batch, dtype=torch.int32).pin_memory() for _ in range(4)]
        inflight: collections.deque = collections.deque()
        stop_issue = False
        while True:
            # issue while every row still needs a token beyond those in flight
            while (not stop_issue and len(inflight) < self.depth and
                   all(q.issued < q.max_tokens - 1 for q in rows)):
                r.decode_batch([q.sid for q in rows], [q.pos for q in rows])
                for q in rows:
                    q.pos += 1
                    q.issued += 1
                self.steps += 1
                if r.is_gpu:
                    buf = self._ring[self.steps % len(self._ring)]
                    buf[:B].copy_(r.s_out[:B], non_blocking=True)
                    ev = torch.cuda.Event()
                    ev.record()
                    inflight.append((buf, ev))
                else:
                    inflight.append((r.s_out[:B].clone(), None))
            if not inflight:
                break
            buf, ev = inflight.popleft()
            if ev is not None:
                ev.synchronize()
            toks = buf[:B].tolist()
            for q, t in zip(rows, toks):
                r.kv.seqs[q.sid].tokens.append(q.last_input)  # its KV was written by this step
                q.last_input = t
                q.history.append(t)
                q.n_sampled += 1
                if not q.cancelled.is_set():
                    self._deliver(q, t)
            with self.cv:
                if self._must_drain(rows):
                    stop_issue = True  # drain what is in flight, then recompose
        # steps issued past a cancellation were wasted; their KV positions are not recorded
        for q in rows:
            if q.finished():
                self.active.remove(q)
                self._retire(q)
