"""Continuous batching (engine/scheduler.py) on the torch twin: concurrent requests decode in one batch
and produce what each would produce alone; cancellation frees rows; prefix reuse across turns."""
import threading
import time

import pytest

from ollama_operator_amd.engine.runner import Runner, StepTimes
from ollama_operator_amd.engine.sampling import SamplingOptions
from ollama_operator_amd.engine.scheduler import BatchScheduler


@pytest.fixture(scope="module")
def runner(tmp_path_factory):
    from ollama_operator_amd.gguf.constants import FileType
    from ollama_operator_amd.models.config import preset
    from ollama_operator_amd.models.random_init import write_random_gguf
    p = str(tmp_path_factory.mktemp("sched") / "m.gguf")
    write_random_gguf(p, preset("tiny-llama"), FileType.MOSTLY_Q8_0, seed=7, quantize_from_float=True)
    return p


def solo(path, prompt, opts, n):
    r = Runner(path, device="cpu", max_batch=16, max_seqs=2, ctx=256)
    return list(r.generate(r.new_sequence(), prompt, opts, max_tokens=n))


def test_batched_matches_solo_greedy_and_seeded(runner):
    prompts = [[1, 5, 9, 13], [1, 200, 201], [1, 7, 7, 7, 7, 7, 30], [1, 99]]
    optss = [SamplingOptions(temperature=0), SamplingOptions(temperature=0.8, seed=5),
             SamplingOptions(temperature=0), SamplingOptions(temperature=1.0, top_k=10, seed=11)]
    lens = [12, 7, 20, 16]  # rows finish at different steps -> recomposition mid-flight
    want = [solo(runner, p, o, n) for p, o, n in zip(prompts, optss, lens)]
    r = Runner(runner, device="cpu", max_batch=16, max_seqs=8, ctx=256)
    sch = BatchScheduler(r, max_parallel=4)
    got = [None] * 4
    start = threading.Barrier(4)

    def work(i):
        start.wait()
        got[i] = list(sch.submit(prompts[i], optss[i], lens[i]))

    th = [threading.Thread(target=work, args=(i,)) for i in range(4)]
    for t in th:
        t.start()
    for t in th:
        t.join(60)
    sch.close()
    assert got == want
    assert sch.max_batch_seen >= 2  # they really shared steps


def test_cancel_frees_row_and_prefix_reuse(runner):
    r = Runner(runner, device="cpu", max_batch=16, max_seqs=4, ctx=256)
    sch = BatchScheduler(r, max_parallel=2)
    gen = sch.submit([1, 2, 3, 4, 5], SamplingOptions(temperature=0), 50)
    first = [next(gen) for _ in range(3)]
    gen.close()  # client went away after 3 tokens
    t = StepTimes()
    out = list(sch.submit([1, 2, 3, 4, 5] + first[:2] + [9], SamplingOptions(temperature=0), 4, times=t))
    assert len(out) == 4
    assert t.prompt_tokens < 8  # the conversation prefix came from the cancelled request's KV
    assert t.gen_tokens == 4
    sch.close()
    assert len(r.kv.seqs) <= 2


def test_exclusive_job_between_steps(runner):
    r = Runner(runner, device="cpu", max_batch=16, max_seqs=4, ctx=256)
    sch = BatchScheduler(r, max_parallel=2)
    v = sch.run_exclusive(lambda rr: rr.embed([1, 2, 3]))
    assert v.shape == (r.cfg.n_embd,)
    sch.close()


def test_failed_step_fails_rows_and_loop_survives(runner, monkeypatch):
    """A step that raises fails the requests it carried (rows freed); later requests are served."""
    r = Runner(runner, device="cpu", max_batch=16, max_seqs=5, ctx=256)
    sch = BatchScheduler(r, max_parallel=2)
    orig = r.decode_batch
    calls = {"n": 0}

    def boom(sids, poss):
        calls["n"] += 1
        if calls["n"] == 2:
            raise RuntimeError("injected HIP error")
        return orig(sids, poss)

    monkeypatch.setattr(r, "decode_batch", boom)
    with pytest.raises(RuntimeError, match="injected"):
        list(sch.submit([1, 2, 3], SamplingOptions(temperature=0), 10))
    out = list(sch.submit([1, 4, 5], SamplingOptions(temperature=0), 5))
    assert len(out) == 5 and sch.failed_steps == 1
    sch.close()
    with pytest.raises(RuntimeError, match="closed"):
        sch.submit([1], SamplingOptions(), 2)
    with pytest.raises(RuntimeError, match="closed"):
        sch.run_exclusive(lambda rr: 1)


def test_close_fails_queued_jobs_and_requests(runner):
    r = Runner(runner, device="cpu", max_batch=16, max_seqs=5, ctx=256)
    sch = BatchScheduler(r, max_parallel=2)
    gate = threading.Event()
    res = {}

    def slow_job(rr):
        gate.wait(10)
        return 1

    t1 = threading.Thread(target=lambda: res.setdefault("a", sch.run_exclusive(slow_job)))
    t1.start()
    time.sleep(0.2)

    def second():
        try:
            sch.run_exclusive(lambda rr: 2)
        except RuntimeError as e:
            res["b"] = e

    t2 = threading.Thread(target=second)
    t2.start()
    time.sleep(0.2)
    closer = threading.Thread(target=sch.close)
    closer.start()
    time.sleep(0.1)
    gate.set()
    for t in (t1, t2, closer):
        t.join(30)
        assert not t.is_alive()
    assert res["a"] == 1 and isinstance(res["b"], RuntimeError)


def test_embed_job_with_every_row_taken(runner):
    """All rows decoding + a full idle prefix cache: an embedding job still gets a KV row."""
    r = Runner(runner, device="cpu", max_batch=16, max_seqs=5, ctx=256)  # the manager's 2*par+1
    sch = BatchScheduler(r, max_parallel=2)
    for i in range(2):  # fill the idle prefix cache
        list(sch.submit([1, 30 + i, 40 + i], SamplingOptions(temperature=0), 2))
    gens = [sch.submit([1, 50 + i], SamplingOptions(temperature=0), 40) for i in range(2)]
    firsts = [next(g) for g in gens]  # both rows active now
    v = sch.run_exclusive(lambda rr: rr.embed([1, 2, 3]))
    assert v.shape == (r.cfg.n_embd,) and len(firsts) == 2
    for g in gens:
        g.close()
    sch.close()


def test_overload_keeps_pipelining(runner):
    """More clients than rows: pending requests that cannot be admitted must not force a drain."""
    r = Runner(runner, device="cpu", max_batch=16, max_seqs=3, ctx=256)
    sch = BatchScheduler(r, max_parallel=1)
    rows = []
    sch.pending.append(object())  # a queued request while the only row is busy
    sch.active = rows = [type("Q", (), {"finished": lambda self: False})()]
    assert not sch._must_drain(rows)
    sch.active = []
    assert sch._must_drain(rows)  # a free row: admit now
    sch.pending.clear()
    sch.close()


def test_bad_request_in_a_burst_fails_alone(runner):
    """Batched admission validates each request first (advisor r3): a prompt naming an unregistered
    image id fails by itself; the other requests of the same burst are admitted and decode."""
    want = solo(runner, [1, 5, 9, 13], SamplingOptions(temperature=0), 6)
    r = Runner(runner, device="cpu", max_batch=16, max_seqs=8, ctx=256, ext_rows=8)
    sch = BatchScheduler(r, max_parallel=4)
    # queue the burst while the scheduler is busy, so all three are admitted together
    with sch.cv:
        good1 = sch.submit([1, 5, 9, 13], SamplingOptions(temperature=0), 6)
        bad = sch.submit([1, -123, 9], SamplingOptions(temperature=0), 6)
        good2 = sch.submit([1, 5, 9, 13], SamplingOptions(temperature=0), 6)
    assert list(good1) == want and list(good2) == want
    with pytest.raises(ValueError):
        list(bad)
    sch.close()


@pytest.mark.parametrize("chunk", [4, 0])
def test_interleaved_admission_matches_solo(runner, chunk):
    """A burst arriving while a row decodes: with chunk > 0 its prompts go through in chunks of `chunk`
    tokens, each chunk's forward also stepping the running row (Runner.admit_many mixed items). Every
    request must still produce exactly what it produces alone; chunk = 0 is the one-forward burst."""
    p0, p1, p2 = [1, 5, 9, 13], [1] + list(range(40, 57)), [1] + list(range(80, 91))
    o0, o1, o2 = SamplingOptions(temperature=0.8, seed=3), SamplingOptions(temperature=0), \
        SamplingOptions(temperature=1.0, top_k=20, seed=9)
    want = [solo(runner, p, o, n) for p, o, n in ((p0, o0, 30), (p1, o1, 12), (p2, o2, 9))]
    r = Runner(runner, device="cpu", max_batch=16, max_seqs=8, ctx=256)
    sch = BatchScheduler(r, max_parallel=4, chunk=chunk)
    g0 = sch.submit(p0, o0, 30)
    head = [next(g0), next(g0)]  # the first request is decoding
    with sch.cv:  # the burst lands together
        g1 = sch.submit(p1, o1, 12)
        g2 = sch.submit(p2, o2, 9)
    got = [head + list(g0), list(g1), list(g2)]
    sch.close()
    assert got == want
    if chunk:
        # 18 + 12 prompt tokens in chunks of 4 (the running row's token rides along in each)
        assert sch.interleaved_chunks >= (17 + 11) // 4
    else:
        assert sch.interleaved_chunks == 0


def test_burst_coalescing_admits_together(runner):
    """Nothing decoding: requests arriving within the quiet window are admitted in one forward."""
    r = Runner(runner, device="cpu", max_batch=16, max_seqs=8, ctx=256)
    sch = BatchScheduler(r, max_parallel=4, coalesce_ms=500, quiet_ms=200)
    calls = []
    orig = r.admit_many

    def spy(items):
        calls.append(len(items))
        return orig(items)

    r.admit_many = spy
    out = {}
    th = []
    for i in range(3):
        t = threading.Thread(target=lambda i=i: out.setdefault(i, list(sch.submit([1, 10 + i, 20 + i],
                                                                                 SamplingOptions(temperature=0), 3))))
        t.start()
        th.append(t)
        time.sleep(0.02)
    for t in th:
        t.join(60)
    sch.close()
    assert calls and calls[0] == 3, calls
    assert all(len(v) == 3 for v in out.values())
