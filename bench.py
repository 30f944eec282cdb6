"""Headline benchmark (BASELINE.json): output tokens/s, Llama-2-7B Q4_K_M, decode, 1/2/4/8 MI355X.

Data-parallel serving exactly as the reference scales (`spec.replicas` -> one replica per GPU,
reference pkg/model/model.go:72,149-186): each rank owns a full replica and one stream of
generation; `value` is the whole-job aggregate tokens/s.

One step = one decode token for the sequence on each GPU: the full 32-layer forward through the
native gfx950 executor (fused quantized GEMVs, paged attention), the LM head, and Ollama-default
sampling (temperature 0.8, top-k 40, top-p 0.9, repeat penalty 1.1) on device, replayed as one
hipGraph, plus the token hand-back to the host exactly as the server streams it.
Weights: random-init GGUF with the real Q4_K_M tensor-type mix (no network for checkpoints).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--prompt P]
    torchrun --nproc-per-node N bench.py --gpus N ...
    python bench.py --model llama2-70b --ftype Q4_0 --tp 8      # tensor parallel (BASELINE config 4)

`--gpus N` without torchrun: this process launches the N rank processes itself (one per GPU, before
it touches any GPU) and exits with their status; it refuses (non-zero) when fewer than N GPUs are
visible instead of silently measuring one. `--tp T` serves ONE sequence on T GPUs through the real
tensor-parallel serving stack (parallel/tp.py: leader + T-1 worker processes, one-shot IPC
all-reduce in the decode graph) and reports its tokens/s with parallelism `tpT`. `--device cpu`
runs the same orchestration on the CPU (gloo, torch twin executor) -- the multi-rank CPU tests use it.
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)


MODEL_LABELS = {"llama2-7b": "Llama-2-7B", "llama2-13b": "Llama-2-13B", "llama2-70b": "Llama-2-70B",
                "mistral-7b": "Mistral-7B", "mixtral-8x7b": "Mixtral-8x7B", "phi2": "Phi-2",
                "gemma-2b": "Gemma-2B", "gemma-7b": "Gemma-7B"}


def ensure_model(path: str, preset_name: str, ftype_name: str, ctx_len: int = 0) -> str:
    """ctx_len > 0: the preset's architecture with its context length metadata replaced (random-init
    weights carry no trained context; e.g. Llama-2-7B shapes at 8192 keys, --model-ctx)."""
    from ollama_operator_amd.gguf.constants import FileType
    from ollama_operator_amd.models.config import preset
    from ollama_operator_amd.models.random_init import write_random_gguf
    tag = hashlib.sha1(f"{preset_name}:{ftype_name}:{ctx_len}:v1".encode()).hexdigest()[:10]
    marker = path + "." + tag + ".ok"
    if os.path.exists(path) and os.path.exists(marker):
        return path
    os.makedirs(os.path.dirname(path), exist_ok=True)
    tmp = path + f".tmp{os.getpid()}"
    cfg = preset(preset_name, ctx_len=ctx_len) if ctx_len > 0 else preset(preset_name)
    write_random_gguf(tmp, cfg, FileType[f"MOSTLY_{ftype_name}"], seed=0)
    os.replace(tmp, path)
    open(marker, "w").close()
    return path


def start_server(a, model_path: str):
    """Spawn `ollama serve` (this framework's server, cli.py) as a child process. Called before this
    process touches the GPU: a GPU-initialised parent must never fork+exec."""
    import socket
    import subprocess
    with socket.socket() as s_:
        s_.bind(("127.0.0.1", 0))
        port = s_.getsockname()[1]
    env = dict(os.environ)
    env.update({"OLLAMA_HOST": f"127.0.0.1:{port}", "OLLAMA_MODELS": os.path.join(a.dir, "server-models"),
                "OLLAMA_NUM_PARALLEL": str(a.server_parallel), "OMX_LOG_LEVEL": "warning",
                "PYTHONPATH": ROOT + os.pathsep + env.get("PYTHONPATH", "")})
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    log = open(os.path.join(a.dir, f"server-{port}.log"), "w")
    proc = subprocess.Popen([sys.executable, "-m", "ollama_operator_amd", "serve"], env=env, cwd=ROOT,
                            stdout=log, stderr=subprocess.STDOUT, start_new_session=True)
    import atexit
    atexit.register(stop_server, proc)  # never leave the child behind, also when the bench fails
    return proc, f"http://127.0.0.1:{port}"


def bench_server(a, url: str, model_path: str, vocab_words: int = 32000):
    """Headline metric the way BASELINE.json defines it: `/api/generate` (stream=false) through the
    REST server, tok/s = eval_count / eval_duration * 1e9 (reference docs getting-started.md:135-149).
    Then `a.server_parallel` concurrent clients (continuous batching) for the aggregate."""
    import concurrent.futures as cf
    import random

    import httpx
    deadline = time.time() + 300  # a fresh box pages torch in for 1-2 min
    with httpx.Client(base_url=url, timeout=600) as c:
        while True:
            try:
                if c.get("/api/version").status_code == 200:
                    break
            except httpx.TransportError:
                pass
            if time.time() > deadline:
                raise RuntimeError("server did not come up")
            time.sleep(0.5)
        r = c.post("/api/create", json={"model": "bench", "modelfile": f"FROM {model_path}", "stream": False})
        r.raise_for_status()
        rng = random.Random(5)

        def prompt():  # synthetic prompt of a.prompt tokens, passed as Ollama `context` token ids
            return [1] + [rng.randrange(3, vocab_words) for _ in range(a.prompt - 2)]

        def gen(n, p, cc=None):
            if cc is None:
                with httpx.Client(base_url=url, timeout=600) as c1:
                    return gen(n, p, c1)
            return cc.post("/api/generate", json={"model": "bench", "prompt": " a", "context": p, "raw": True, "stream": False,
                                                  "options": {"num_predict": n, "seed": 42}}).json()

        gen(32, prompt())  # load + warm
        d = gen(a.steps, prompt())
        single = d["eval_count"] / d["eval_duration"] * 1e9
        out = {"served_tok_s": round(single, 2), "eval_count": d["eval_count"],
               "prompt_eval_count": d["prompt_eval_count"],
               "served_ttft_ms": round(d["prompt_eval_duration"] / 1e6, 2), "num_parallel": a.server_parallel}
        P = a.server_parallel
        if P > 1:
            prompts = [prompt() for _ in range(P)]
            # one connected client per simulated user, built before the clock starts: an httpx.Client
            # builds an SSL context (CA bundle load), which 4 threads contending for the GIL took
            # ~0.3 s to do -- client setup, not serving time
            clients = [httpx.Client(base_url=url, timeout=600) for _ in range(P)]
            for cc in clients:
                cc.get("/api/version")
            with cf.ThreadPoolExecutor(P) as ex:
                list(ex.map(lambda i: None, range(P)))  # worker threads started before the clock too
                t0 = time.perf_counter()
                res = list(ex.map(lambda pc: gen(a.steps, pc[0], pc[1]), zip(prompts, clients)))
                wall = time.perf_counter() - t0
            for cc in clients:
                cc.close()
            out["concurrent_clients"] = P
            out["concurrent_aggregate_tok_s"] = round(sum(x["eval_count"] for x in res) / wall, 2)
            out["concurrent_per_client_tok_s"] = [round(x["eval_count"] / x["eval_duration"] * 1e9, 2) for x in res]
            # decode-phase aggregate (what the batched steps deliver); the wall aggregate above also
            # holds the P prefills and request ramp
            out["concurrent_decode_tok_s"] = round(sum(out["concurrent_per_client_tok_s"]), 2)
            # where the wall time went, per client (server-side Ollama durations, ms)
            ms = lambda k: [round(x.get(k, 0) / 1e6, 2) for x in res]  # noqa: E731
            out["concurrent_wall_ms"] = round(wall * 1e3, 2)
            out["concurrent_total_ms"] = ms("total_duration")
            out["concurrent_prompt_eval_ms"] = ms("prompt_eval_duration")
            out["concurrent_eval_ms"] = ms("eval_duration")
    return out


def stop_server(proc):
    import signal
    if proc.poll() is not None:
        return
    try:
        os.killpg(proc.pid, signal.SIGTERM)
        proc.wait(timeout=30)
    except Exception:
        try:
            os.killpg(proc.pid, signal.SIGKILL)
        except Exception:
            pass


def bench_batched(runner, a, rank, world, sync):
    """Aggregate decode tokens/s with B = a.batch_extra sequences per GPU sharing every step (the
    server's continuous batching, engine/scheduler.py): B prompts prefilled, then exactly a.steps batched
    steps (each samples B tokens on device, Ollama-default options per row), two steps in flight."""
    import torch
    import torch.distributed as dist
    from ollama_operator_amd.engine.sampling import SamplingOptions
    B = a.batch_extra
    runner.capture_batch_graphs(B)
    g = torch.Generator().manual_seed(4321 + rank)
    sids, poss, firsts, prompts = [], [], [], []
    for b in range(B):
        p = [1] + torch.randint(3, runner.cfg.n_vocab, (a.prompt - 1,), generator=g).tolist()
        sid = runner.new_sequence()
        runner.prefill(sid, p)
        runner._set_sampler(0, SamplingOptions(seed=7 + b), p, 7 + b, 0)
        runner._sample(1)
        firsts.append(int(runner.s_out[0].item()))
        sids.append(sid)
        poss.append(len(p))
        prompts.append(p)
    for b in range(B):
        runner._set_sampler(b, SamplingOptions(seed=7 + b), prompts[b] + [firsts[b]], 7 + b, 1)
    runner.set_tokens(firsts)
    ring = [torch.zeros(B, dtype=torch.int32).pin_memory() for _ in range(4)]
    evs = []

    def step(i):
        runner.decode_batch(sids, poss)
        for b in range(B):
            poss[b] += 1
        ring[i % 4].copy_(runner.s_out[:B], non_blocking=True)
        e = torch.cuda.Event()
        e.record()
        evs.append(e)
        if len(evs) > 2:  # two steps in flight, the host reads tokens one step behind
            evs.pop(0).synchronize()

    for i in range(a.warmup):
        step(i)
    sync()
    t0 = time.perf_counter()
    for i in range(a.steps):
        step(i)
    sync()
    dt = time.perf_counter() - t0
    t = torch.tensor([dt], device="cuda")
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dt = float(t)
    for sid in sids:
        runner.free_sequence(sid)
    return {"sequences_per_gpu": B, "tokens_per_s": round(world * B * a.steps / dt, 2),
            "ms_per_step": round(dt / a.steps * 1e3, 4)}


def free_port() -> int:
    import socket
    with socket.socket() as s_:
        s_.bind(("127.0.0.1", 0))
        return s_.getsockname()[1]


def visible_devices(device: str) -> int:
    if device == "cpu":
        return 1 << 30
    import torch
    return torch.cuda.device_count()  # counts devices without initialising the GPU on this image


def launch_ranks(a) -> int:
    """`--gpus N` outside torchrun: spawn the N data-parallel ranks (one process per GPU, env
    RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* as torchrun sets them) and return the worst exit code.
    Runs before this process touches any GPU; the model file is written once, here."""
    import subprocess
    n = a.gpus
    have = visible_devices(a.device)
    if have < n:
        print(f"bench.py: --gpus {n} requested but only {have} GPU(s) are visible; refusing to report a "
              f"{have}-GPU number as {n}", file=sys.stderr, flush=True)
        return 2
    ensure_model(model_path(a), a.model, a.ftype, a.model_ctx)
    port = free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env, cwd=ROOT))
    rc = 0
    try:
        for p in procs:
            c = p.wait()
            if c != 0 and rc == 0:
                rc = c
                for q in procs:  # one rank failed: the others would hang in the next collective
                    if q.poll() is None:
                        q.kill()
    finally:
        for q in procs:
            if q.poll() is None:
                q.kill()
    return rc


def model_path(a) -> str:
    ctx = f"-ctx{a.model_ctx}" if getattr(a, "model_ctx", 0) else ""
    return os.path.join(a.dir, f"{a.model}-{a.ftype.lower()}{ctx}.gguf")


def bench_tp(a) -> None:
    """One sequence on T GPUs through the tensor-parallel serving stack: the leader (this process)
    spawns T-1 workers before touching the GPU (parallel/tp.py start_leader), loads the model sharded
    (TPRunnerProxy), and streams `generate` exactly as the server does. On a box with fewer GPUs than
    T, ranks share GPUs (gloo compute group; decode collectives stay on the one-shot IPC all-reduce)
    -- a correctness rehearsal, reported with `shared_gpus` in config."""
    T = a.tp
    have = visible_devices(a.device)
    shared = have < T
    if shared and not a.allow_shared:
        print(f"bench.py: --tp {T} needs {T} GPUs, {have} visible (pass --allow-shared to rehearse on fewer)",
              file=sys.stderr, flush=True)
        sys.exit(2)
    path = ensure_model(model_path(a), a.model, a.ftype, a.model_ctx)
    if shared or a.device == "cpu":
        os.environ["OMX_TP_BACKEND"] = "gloo"
    from ollama_operator_amd.parallel import tp
    world = tp.start_leader(T)
    import torch
    from ollama_operator_amd.engine.sampling import SamplingOptions
    gpu = world.device.startswith("cuda")

    def sync():
        if gpu:
            torch.cuda.synchronize()

    try:
        ctx = a.prompt + a.warmup + a.steps + 64
        t_load = time.perf_counter()
        r = tp.load_tp_runner(world, path, max_batch=a.chunk, max_seqs=2, ctx=ctx)
        r.warmup()
        sync()
        load_s = time.perf_counter() - t_load
        g = torch.Generator().manual_seed(1234)
        prompt = [1] + torch.randint(3, r.cfg.n_vocab, (a.prompt - 1,), generator=g).tolist()
        sid = r.new_sequence()
        gen = r.generate(sid, prompt, SamplingOptions(seed=42), max_tokens=a.warmup + a.steps + 2)
        t_p = time.perf_counter()
        next(gen)
        ttft = time.perf_counter() - t_p
        for _ in range(a.warmup):
            next(gen)
        sync()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            next(gen)
        sync()
        dt = time.perf_counter() - t0
        gen.close()
        r.free_sequence(sid)
        weights_gb = r.w.nbytes / 1e9
        r.close()
    finally:
        tp.shutdown_leader(world)
    label = MODEL_LABELS.get(a.model, a.model) + " " + a.ftype + (f" (ctx {a.model_ctx})" if a.model_ctx else "")
    print(json.dumps({
        "metric": f"output tokens/sec {label}",
        "value": round(a.steps / dt, 2),
        "unit": "tokens/s",
        "n_gpus": T,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": round(dt / a.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": f"{a.ftype} weights, int8-dot activations, fp32 accumulate, fp16 KV",
        "data": f"synthetic prompt, random-init GGUF weights (real {a.ftype} tensor-type mix)",
        "config": {"model": label, "global_batch": 1, "seq_len": a.prompt + a.warmup + a.steps,
                   "parallelism": f"tp{T}", "prompt_tokens": a.prompt, "shared_gpus": shared,
                   "device": a.device, "sampling": "temperature 0.8, top_k 40, top_p 0.9, repeat_penalty 1.1"},
        "extra": {"ttft_ms": round(ttft * 1e3, 2), "load_s": round(load_s, 2),
                  "weights_gb_rank0": round(weights_gb, 3)},
    }), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--tp", type=int, default=1, help="tensor-parallel degree: one sequence sharded over T GPUs")
    ap.add_argument("--allow-shared", action="store_true",
                    help="--tp T on fewer than T GPUs: ranks share GPUs (correctness rehearsal)")
    ap.add_argument("--device", default="cuda", choices=["cuda", "cpu"],
                    help="cpu: same orchestration on the CPU (gloo, torch twin executor) for tests")
    ap.add_argument("--steps", type=int, default=256)
    ap.add_argument("--warmup", type=int, default=16)
    ap.add_argument("--prompt", type=int, default=128)
    ap.add_argument("--model", default="llama2-7b")
    ap.add_argument("--ftype", default="Q4_K_M", type=str.upper)
    ap.add_argument("--model-ctx", type=int, default=0,
                    help="replace the preset's context length (random-init weights), e.g. 8192 for Llama-2-7B "
                         "shapes at an 8k context; 0 = the preset's (Llama-2: 4096)")
    ap.add_argument("--dir", default=os.environ.get("OMX_BENCH_DIR", "/tmp/omx_bench"))
    ap.add_argument("--batch-extra", type=int, default=4,
                    help="also measure continuous-batching throughput with this many concurrent sequences per "
                         "GPU (Ollama OLLAMA_NUM_PARALLEL default 4; reported under extra.continuous_batching, 0 = skip)")
    ap.add_argument("--via-server", type=int, default=1,
                    help="1 (default, single-GPU runs): also measure through the REST server (/api/generate) "
                         "and report it under extra.server")
    ap.add_argument("--ttft-long", type=int, default=2048,
                    help="also time prefill + first token of a prompt this long (extra.ttft_long_ms; 0 = skip)")
    ap.add_argument("--chunk", type=int, default=2048, help="prefill chunk (MFMA GEMM M) = runner max_batch")
    ap.add_argument("--long-ctx", default="2048,4096",
                    help="also measure batch-1 decode tokens/s after a prompt of each of these lengths "
                         "(extra.long_context: decode_ctx<L>_tok_s; a length past the model's context is "
                         "clipped to it, minus the timed steps; empty = skip)")
    ap.add_argument("--server-parallel", type=int, default=4,
                    help="OLLAMA_NUM_PARALLEL of the spawned server (concurrent clients measured)")
    a = ap.parse_args()
    os.makedirs(a.dir, exist_ok=True)
    if a.tp > 1:
        bench_tp(a)
        return
    if "WORLD_SIZE" not in os.environ and a.gpus > 1:
        sys.exit(launch_ranks(a))

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus:
        print(f"bench.py: WORLD_SIZE={world} but --gpus {a.gpus}", file=sys.stderr, flush=True)
        sys.exit(2)
    gpu = a.device == "cuda"
    path = model_path(a)
    server = None
    if a.via_server and world == 1 and gpu:
        server = start_server(a, path)  # before this process touches the GPU

    import torch
    import torch.distributed as dist

    if gpu:
        torch.cuda.set_device(local)
    if world > 1:
        if gpu:
            dist.init_process_group("nccl", device_id=torch.device(f"cuda:{local}"))
        else:
            dist.init_process_group("gloo")

    from ollama_operator_amd.engine.runner import Runner
    from ollama_operator_amd.engine.sampling import SamplingOptions

    if local == 0:
        ensure_model(path, a.model, a.ftype, a.model_ctx)
    if world > 1:
        dist.barrier()
    else:
        ensure_model(path, a.model, a.ftype, a.model_ctx)

    long_ctx = [int(x) for x in a.long_ctx.split(",") if x.strip()] if gpu else []
    LC_WARM, LC_STEPS = 8, 64
    ctx = max(a.prompt + a.warmup + a.steps + 64, a.ttft_long + 8 if a.ttft_long else 0,
              max(long_ctx, default=0) + LC_WARM + LC_STEPS + 64)
    t_load = time.perf_counter()
    runner = Runner(path, device=f"cuda:{local}" if gpu else "cpu", max_batch=a.chunk,
                    max_seqs=max(2, a.batch_extra), ctx=ctx)
    runner.warmup()  # load-time decode-graph capture, as the server does at model load
    if gpu:
        torch.cuda.synchronize()
    load_s = time.perf_counter() - t_load

    g = torch.Generator().manual_seed(1234 + rank)
    prompt = [1] + torch.randint(3, runner.cfg.n_vocab, (a.prompt - 1,), generator=g).tolist()
    opts = SamplingOptions(seed=42 + rank)  # Ollama defaults
    sid = runner.new_sequence()
    # decode steps per graph replay (Runner.decode_group): the timed window must hold whole groups
    G = getattr(runner, "decode_group", 1)
    if a.steps % G:
        runner.decode_group = G = 1
    gen = runner.generate(sid, prompt, opts, max_tokens=a.warmup + a.steps + 4 * G + 4)
    t_p = time.perf_counter()
    next(gen)  # prefill + first token
    ttft = time.perf_counter() - t_p
    for _ in range(a.warmup):
        next(gen)

    def sync():
        if gpu:
            torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        if gpu:
            torch.cuda.synchronize()

    # Exactly a.steps decode steps in the timed window: the sync before t0 retires every step already
    # enqueued (the generator keeps steps in flight ahead of the tokens it hands out), the loop hands out
    # tokens until a.steps more have been enqueued, and the sync after t1 retires them. Counting handed-out
    # tokens instead would credit the window with steps the GPU finished before t0.
    sync()
    s0 = runner.steps_issued
    t0 = time.perf_counter()
    while runner.steps_issued - s0 < a.steps:
        next(gen)
    sync()
    dt = time.perf_counter() - t0
    if runner.steps_issued - s0 != a.steps:
        raise RuntimeError(f"timed window ran {runner.steps_issued - s0} decode steps, not {a.steps}")
    t = torch.tensor([dt], device="cuda" if gpu else "cpu")
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dt = float(t)
    ms = dt / a.steps * 1e3
    value = world * a.steps / dt
    gen.close()
    runner.free_sequence(sid)
    ttft_long = None
    if a.ttft_long:
        p = [1] + torch.randint(3, runner.cfg.n_vocab, (a.ttft_long - 1,), generator=g).tolist()
        best = None
        for _ in range(3):  # prefill of a fresh sequence each time (no prefix reuse)
            sid = runner.new_sequence()
            if gpu:
                torch.cuda.synchronize()
            t_p = time.perf_counter()
            gl = runner.generate(sid, p, opts, max_tokens=1)
            next(gl)
            dt_l = time.perf_counter() - t_p
            gl.close()
            runner.free_sequence(sid)
            best = dt_l if best is None else min(best, dt_l)
        ttft_long = round(best * 1e3, 2)
    long_res = {}
    for L in sorted({min(x, runner.ctx - LC_WARM - LC_STEPS - 8 * G - 8) for x in long_ctx}):
        # decode after an L-token prompt: every step attends over >= L cached keys (split flash-decode);
        # exactly LC_STEPS decode steps timed, as the headline loop
        p = [1] + torch.randint(3, runner.cfg.n_vocab, (L - 1,), generator=g).tolist()
        sid = runner.new_sequence()
        gl = runner.generate(sid, p, opts, max_tokens=LC_WARM + LC_STEPS + 4 * G + 4)
        next(gl)
        for _ in range(LC_WARM):
            next(gl)
        sync()
        s_l = runner.steps_issued
        t_l = time.perf_counter()
        while runner.steps_issued - s_l < LC_STEPS:
            next(gl)
        sync()
        dt_l = time.perf_counter() - t_l
        gl.close()
        runner.free_sequence(sid)
        long_res[f"decode_ctx{L}_tok_s"] = round(LC_STEPS / dt_l, 2)
    batched = None
    if a.batch_extra > 1 and gpu:
        batched = bench_batched(runner, a, rank, world, sync)
    served = None
    # resident weight bytes: the GGUF tensors (layout v2) plus the batched-decode layout M copies
    layout_m_gb = getattr(runner, "mfma_bytes", 0) / 1e9
    prefill_f16_gb = getattr(runner, "f16_bytes", 0) / 1e9
    if server is not None:
        weights_gb = runner.w.nbytes / 1e9
        n_vocab = runner.cfg.n_vocab
        del runner
        torch.cuda.empty_cache()
        try:
            served = bench_server(a, server[1], path, vocab_words=n_vocab)
            served["vs_engine"] = round(served["served_tok_s"] / value, 4)
        except Exception as e:  # the headline line is still printed; the failure is reported
            served = {"error": f"{type(e).__name__}: {e}"}
        finally:
            stop_server(server[0])
    else:
        weights_gb = runner.w.nbytes / 1e9
    label = MODEL_LABELS.get(a.model, a.model) + " " + a.ftype + (f" (ctx {a.model_ctx})" if a.model_ctx else "")
    if rank == 0:
        print(json.dumps({
            "metric": f"output tokens/sec {label}",
            "value": round(value, 2),
            "unit": "tokens/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(ms, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": f"{a.ftype} weights, int8-dot activations, fp32 accumulate, fp16 KV",
            "data": f"synthetic prompt, random-init GGUF weights (real {a.ftype} tensor-type mix)",
            "config": {"model": label, "global_batch": world, "seq_len": a.prompt + a.warmup + a.steps,
                       "parallelism": f"dp{world}", "prompt_tokens": a.prompt, "decode_batch_per_gpu": 1,
                       "device": a.device,
                       "sampling": "temperature 0.8, top_k 40, top_p 0.9, repeat_penalty 1.1 (on device)"},
            "extra": {"ttft_ms": round(ttft * 1e3, 2), f"ttft_{a.ttft_long}_ms": ttft_long, "prefill_chunk": a.chunk,
                      "load_s": round(load_s, 2),
                      "weights_gb": round(weights_gb, 3), "layout_m_gb": round(layout_m_gb, 3),
                      "prefill_f16_gb": round(prefill_f16_gb, 3),
                      "resident_weights_gb": round(weights_gb + layout_m_gb + prefill_f16_gb, 3),
                      "long_context": long_res or None, "continuous_batching": batched, "server": served},
        }), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
