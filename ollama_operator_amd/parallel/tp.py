"""Tensor-parallel serving: one pod, one process per GPU.

`ollama serve` with `OMX_TP=N` (set by the operator from `spec.tensorParallelSize`,
ollama_operator_amd/operator/resources.py) runs rank 0 inside the HTTP server process and spawns
ranks 1..N-1 as worker processes -- BEFORE anything in the server touches the GPU (no process is
forked or exec'ed from a GPU-initialised parent). All ranks then join:
  * the compute group (RCCL = backend "nccl" on ROCm, over xGMI): the runner's all-reduce of the
    row-parallel partial sums and the all-gather of vocab-sharded logits (engine/runner.py);
  * a gloo control group: rank 0 broadcasts every runner call (load / new_sequence / generate /
    embed / ...) to the workers as int32 frames (no pickling; `TPControl`), and a host shared-memory
    doorbell carries the continue/stop flag of each single-stream decode step (`Doorbell`).
Sampling needs no token broadcast: every rank holds the all-gathered full logits and the same
sampler state with the same resolved seed, so every rank samples the same token; only the stop
decision (taken by the server on detokenised text) crosses the control group, which keeps the
pipelined generate (engine/runner.py `generate`) in lockstep even when the client stops early.
A failed rank kills the pod (no partial recovery inside a TP group).
"""
from __future__ import annotations

import dataclasses
import os
import socket
import subprocess
import sys
import threading
import time

import torch
import torch.distributed as dist

ENV_TP = "OMX_TP"


def tp_size_from_env() -> int:
    return max(1, int(os.environ.get(ENV_TP, "1") or 1))


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


# ---- control channel -------------------------------------------------------------------------------
# Commands travel as int32 frames over the gloo group -- no pickling: the per-step ops (decode_batch,
# evict, new/free_sequence) are ONE fixed-size tensor broadcast; the rare structured ones (load, admit,
# set_ext, ...) add one uint8 broadcast of a JSON document (numpy arrays and SamplingOptions encoded
# explicitly, nothing executable). The per-token continue/stop flag of single-stream generation does not
# use the group at all: a host shared-memory doorbell (all TP ranks of a pod share one node).
FRAME_ROWS = 128                     # decode_batch rows carried inline
_FRAME = 2 + 2 * FRAME_ROWS          # [op, n, sids..., poss...]
_OPS = {"decode_batch": 1, "evict": 2, "new_sequence": 3, "free_sequence": 4, "warmup": 5, "unload": 6, "exit": 7}
_OP_JSON = 100
_NAMES = {v: k for k, v in _OPS.items()}
ENV_DOORBELL = "OMX_TP_DOORBELL"


def _enc(o):
    import numpy as np
    from ..engine.sampling import SamplingOptions
    if isinstance(o, SamplingOptions):
        return {"__opts__": dataclasses.asdict(o)}
    if isinstance(o, np.ndarray):
        import base64
        a = np.ascontiguousarray(o)
        return {"__nd__": [a.dtype.str, list(a.shape), base64.b64encode(a.tobytes()).decode("ascii")]}
    if isinstance(o, (np.integer,)):
        return int(o)
    if isinstance(o, (np.floating,)):
        return float(o)
    raise TypeError(f"TP control: cannot encode {type(o).__name__}")


def _dec(d):
    if "__opts__" in d:
        from ..engine.sampling import SamplingOptions
        return SamplingOptions(**d["__opts__"])
    if "__nd__" in d:
        import base64

        import numpy as np
        dt, shape, b = d["__nd__"]
        return np.frombuffer(base64.b64decode(b), dtype=np.dtype(dt)).reshape(shape).copy()
    return d


def encode_cmd(cmd: dict) -> bytes:
    import json
    return json.dumps(cmd, default=_enc, separators=(",", ":")).encode()


def decode_cmd(blob: bytes) -> dict:
    import json
    return json.loads(blob.decode(), object_hook=_dec)


class Doorbell:
    """Leader -> follower step flags in host shared memory: a 64-slot ring of values plus a sequence
    number (x86 stores are not reordered with other stores, so a follower that sees the sequence sees the
    value); followers publish the last sequence they consumed so the leader never overwrites an unread
    slot. Replaces one gloo broadcast per generated token."""
    SLOTS = 64

    def __init__(self, name: str, create: bool, rank: int = 0, world: int = 1):
        import numpy as np
        from multiprocessing import shared_memory
        self.shm = shared_memory.SharedMemory(name=name, create=create, size=8 * (2 + self.SLOTS + 64))
        if not create:  # the creator owns the segment (Python 3.10 would unlink it at a follower's exit)
            try:
                from multiprocessing import resource_tracker
                resource_tracker.unregister(self.shm._name, "shared_memory")  # noqa: SLF001
            except Exception:  # noqa: BLE001
                pass
        self.a = np.ndarray((2 + self.SLOTS + 64,), dtype=np.int64, buffer=self.shm.buf)
        if create:
            self.a[:] = 0
        self.rank, self.world = rank, world
        self.seen = int(self.a[0])

    def ring(self, value: int) -> None:
        seq = int(self.a[0]) + 1
        # the slowest follower must have consumed seq - SLOTS before its slot is reused
        while self.world > 1 and seq - min(int(self.a[2 + self.SLOTS + r]) for r in range(1, self.world)) > self.SLOTS:
            time.sleep(0)
        self.a[2 + seq % self.SLOTS] = value
        self.a[0] = seq

    def wait(self, alive=lambda: True) -> int:
        target = self.seen + 1
        spins, t0 = 0, time.monotonic()
        while int(self.a[0]) < target:
            spins += 1
            if spins > 2000:
                time.sleep(50e-6)
                if time.monotonic() - t0 > 5.0:
                    if not alive():
                        raise RuntimeError("TP doorbell: leader gone")
                    t0 = time.monotonic()
        v = int(self.a[2 + target % self.SLOTS])
        self.seen = target
        self.a[2 + self.SLOTS + self.rank] = target
        return v

    def close(self, unlink: bool = False) -> None:
        self.a = None
        try:
            self.shm.close()
            if unlink:
                self.shm.unlink()
        except Exception:  # noqa: BLE001
            pass


class TPControl:
    """Leader -> follower command / step-flag channel: int32 frames over a gloo group (commands) and a
    shared-memory doorbell (step flags; gloo broadcast when no doorbell is configured)."""

    def __init__(self, group, leader: bool, doorbell: "Doorbell | None" = None):
        self.group = group
        self.leader = leader
        self.bell = doorbell
        self._flag = torch.zeros(1, dtype=torch.int32)
        self._frame = torch.zeros(_FRAME, dtype=torch.int32)

    def send_cmd(self, cmd: dict) -> None:
        assert self.leader
        op = cmd["op"]
        code = _OPS.get(op)
        f = self._frame
        f.zero_()
        fast = code is not None and set(cmd) <= {"op", "sid", "sids", "poss"}
        if fast and code == 1 and len(cmd["sids"]) > FRAME_ROWS:
            fast = False
        if fast:
            f[0] = code
            if code == 1:
                n = len(cmd["sids"])
                f[1] = n
                f[2:2 + n] = torch.tensor(cmd["sids"], dtype=torch.int32)
                f[2 + FRAME_ROWS:2 + FRAME_ROWS + n] = torch.tensor(cmd["poss"], dtype=torch.int32)
            elif "sid" in cmd:
                f[1] = 1
                f[2] = int(cmd["sid"])
            dist.broadcast(f, src=0, group=self.group)
            return
        blob = encode_cmd(cmd)
        f[0] = _OP_JSON
        f[1] = len(blob)
        dist.broadcast(f, src=0, group=self.group)
        dist.broadcast(torch.frombuffer(bytearray(blob), dtype=torch.uint8), src=0, group=self.group)

    def recv_cmd(self) -> dict:
        f = self._frame
        dist.broadcast(f, src=0, group=self.group)
        code, n = int(f[0]), int(f[1])
        if code == _OP_JSON:
            t = torch.empty(n, dtype=torch.uint8)
            dist.broadcast(t, src=0, group=self.group)
            return decode_cmd(t.numpy().tobytes())
        op = _NAMES.get(code)
        if op is None:
            raise RuntimeError(f"TP control: unknown frame op {code}")
        cmd = {"op": op}
        if code == 1:
            cmd["sids"] = f[2:2 + n].tolist()
            cmd["poss"] = f[2 + FRAME_ROWS:2 + FRAME_ROWS + n].tolist()
        elif n:
            cmd["sid"] = int(f[2])
        return cmd

    def signal(self, go: bool) -> None:  # leader: one decode step will follow (1) / generation over (0)
        if self.bell is not None:
            self.bell.ring(1 if go else 0)
            return
        self._flag[0] = 1 if go else 0
        dist.broadcast(self._flag, src=0, group=self.group)

    def wait(self) -> bool:  # follower
        if self.bell is not None:
            return bool(self.bell.wait(alive=_parent_alive))
        dist.broadcast(self._flag, src=0, group=self.group)
        return bool(self._flag[0])


_PPID = os.getppid()


def _parent_alive() -> bool:
    return os.getppid() == _PPID


@dataclasses.dataclass
class TPWorld:
    rank: int
    size: int
    device: str
    compute_group: object
    ctrl: TPControl
    workers: list
    stopping: threading.Event = dataclasses.field(default_factory=threading.Event)
    # leader's custom all-reduce error probe (CustomAllReduce.error, a host-mapped read): set while a
    # TP model is loaded
    ar_probe: object = None


def _device_for(local_rank: int) -> str:
    if torch.cuda.is_available():
        return f"cuda:{local_rank % torch.cuda.device_count()}"
    return "cpu"


def _backend() -> str:
    b = os.environ.get("OMX_TP_BACKEND")
    if b:
        return b
    return "nccl" if torch.cuda.is_available() else "gloo"


def _init_groups(rank: int, size: int, addr: str, port: int) -> tuple:
    dev = _device_for(rank)
    if dev.startswith("cuda"):
        torch.cuda.set_device(torch.device(dev))
    dist.init_process_group(_backend(), init_method=f"tcp://{addr}:{port}", rank=rank, world_size=size)
    ctrl_group = dist.new_group(backend="gloo")
    return dev, dist.group.WORLD, ctrl_group


def start_leader(size: int) -> TPWorld:
    """Server process (rank 0): spawn workers first (GPU untouched so far), then join the groups."""
    addr, port = "127.0.0.1", _free_port()
    workers = []
    pkg_root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    bell_name = f"omx_tp_{os.getpid()}_{port}"
    bell = Doorbell(bell_name, create=True, rank=0, world=size)
    for r in range(1, size):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(size), MASTER_ADDR=addr,
                   MASTER_PORT=str(port), **{ENV_DOORBELL: bell_name},
                   PYTHONPATH=pkg_root + os.pathsep + os.environ.get("PYTHONPATH", ""))
        workers.append(subprocess.Popen([sys.executable, "-m", "ollama_operator_amd.parallel.tp_worker"], env=env))
    world = TPWorld(0, size, "", None, None, workers)
    # watch the workers from the start: one that dies before the rendezvous would otherwise leave the
    # leader blocked in init_process_group
    threading.Thread(target=_watchdog, args=(world,), name="tp-watchdog", daemon=True).start()
    dev, compute, ctrl = _init_groups(0, size, addr, port)
    world.device, world.compute_group, world.ctrl = dev, compute, TPControl(ctrl, leader=True, doorbell=bell)
    return world


WATCHDOG_PERIOD_S = 1.0


def _watchdog(world: TPWorld, period: float = WATCHDOG_PERIOD_S, exit_fn=os._exit) -> None:
    """A TP group cannot lose a rank: a dead worker leaves the leader blocked in (or timing out of)
    the next collective while /api/tags keeps answering. Any worker exit outside shutdown, and any
    all-reduce barrier timeout on the leader (a wedged peer: the device skips every later collective,
    allreduce.hip), ends the server with a non-zero code, so the pod restarts (SURVEY.md §5.3;
    liveness alone would not see it)."""
    def die(msg: str, rc: int) -> None:
        print(f"tp watchdog: {msg}; terminating the TP group", file=sys.stderr, flush=True)
        for q in world.workers:
            if q.poll() is None:
                q.kill()
        exit_fn(rc)

    while not world.stopping.wait(period):
        for r, p in enumerate(world.workers, start=1):
            rc = p.poll()
            if rc is not None and not world.stopping.is_set():
                die(f"rank {r} exited with code {rc}", rc if rc else 1)
                return
        probe = world.ar_probe
        if probe is not None and not world.stopping.is_set():
            e = probe()
            if e:
                die(f"rank 0: peer {e - 1} missed a one-shot all-reduce barrier", 1)
                return


def shutdown_leader(world: TPWorld) -> None:
    world.stopping.set()
    try:
        world.ctrl.send_cmd({"op": "exit"})
    except Exception:  # noqa: BLE001 - workers may already be gone
        pass
    for p in world.workers:
        try:
            p.wait(timeout=30)
        except subprocess.TimeoutExpired:
            p.kill()
    if world.ctrl is not None and world.ctrl.bell is not None:
        world.ctrl.bell.close(unlink=True)


class TPRunnerProxy:
    """Rank-0 face of a tensor-parallel model: mirrors each call to the workers, then runs it on
    the local rank-0 `Runner` (duck-types the Runner API the server uses)."""

    def __init__(self, world: TPWorld, runner, load_cmd: dict):
        self.world = world
        self.r = runner
        self.load_cmd = load_cmd

    def __getattr__(self, name):  # read-only attributes (cfg, ctx, is_gpu, ...)
        return getattr(self.r, name)

    def _mirror(self, op: str, **kw):
        self.world.ctrl.send_cmd({"op": op, **kw})

    def new_sequence(self) -> int:
        self._mirror("new_sequence")
        return self.r.new_sequence()

    def free_sequence(self, sid: int) -> None:
        self._mirror("free_sequence", sid=sid)
        self.r.free_sequence(sid)

    def warmup(self) -> None:
        self._mirror("warmup")
        self.r.warmup()

    def embed(self, tokens: list[int]):
        self._mirror("embed", tokens=list(tokens))
        return self.r.embed(tokens)

    def set_ext(self, ids: list[int], rows) -> None:  # image patch rows: every rank embeds them
        import numpy as np
        rows = np.ascontiguousarray(rows.detach().float().cpu().numpy() if hasattr(rows, "detach") else rows,
                                    dtype=np.float32)
        self._mirror("set_ext", ids=list(ids), rows=rows)
        self.r.set_ext(ids, rows)

    def generate(self, sid: int, prompt: list[int], options=None, max_tokens: int = 128, stop=None, times=None):
        from ..engine.sampling import SamplingOptions
        o = options or SamplingOptions()
        o = dataclasses.replace(o, seed=o.resolved_seed())  # every rank must draw the same stream
        self._mirror("generate", sid=sid, prompt=list(prompt), options=o, max_tokens=max_tokens)
        return self.r.generate(sid, prompt, o, max_tokens=max_tokens, stop=stop, times=times)

    # continuous batching (engine/scheduler.py drives the leader's runner through these)
    def _prefixes(self, sids) -> dict:
        """The leader's token record of each reused sequence: the scheduler appends generated tokens on
        the leader only, so a follower's record stops at its prompt; admit truncates to `keep`, which may
        reach into generated tokens -- followers adopt the leader's record first (same KV positions)."""
        seqs = self.r.kv.seqs
        return {str(sid): list(seqs[sid].tokens) for sid in sids if sid in seqs and seqs[sid].tokens}

    def admit(self, sid: int, keep: int, tokens: list[int], opts, history: list[int], seed: int,
              n_sampled: int = 0) -> None:
        self._mirror("admit", sid=sid, keep=keep, tokens=list(tokens), opts=opts, history=list(history), seed=seed,
                     n_sampled=n_sampled, prefixes=self._prefixes([sid]))
        self.r.admit(sid, keep, tokens, opts, history, seed, n_sampled)

    def admit_many(self, items: list[tuple]) -> list[int]:
        items = [(it[0], it[1], list(it[2]), it[3], list(it[4]), *it[5:]) for it in items]
        self._mirror("admit_many", items=items, prefixes=self._prefixes([it[0] for it in items]))
        return self.r.admit_many(items)

    def recompose(self, rows: list[tuple], tokens: list[int]) -> None:
        rows = [(o, list(h), sd, n) for o, h, sd, n in rows]
        self._mirror("recompose", rows=rows, tokens=list(tokens))
        self.r.recompose(rows, tokens)

    def decode_batch(self, sids: list[int], poss: list[int]) -> None:
        self._mirror("decode_batch", sids=list(sids), poss=list(poss))
        self.r.decode_batch(sids, poss)

    def evict(self, sid: int) -> None:
        self._mirror("evict", sid=sid)
        self.r.evict(sid)

    def capture_batch_graphs(self, max_B: int) -> None:
        self._mirror("capture_batch_graphs", max_B=max_B)
        self.r.capture_batch_graphs(max_B)

    def close(self) -> None:
        self.world.ar_probe = None
        self._mirror("unload")
        self.r.close()


def load_tp_runner(world: TPWorld, path: str, max_batch: int, max_seqs: int, ctx: int, ext_rows: int = 0):
    from ..engine.runner import Runner
    cmd = dict(path=path, max_batch=max_batch, max_seqs=max_seqs, ctx=ctx, ext_rows=ext_rows)
    world.ctrl.send_cmd({"op": "load", **cmd})
    r = Runner(path, device=world.device, max_batch=max_batch, max_seqs=max_seqs, ctx=ctx, tp_rank=0,
               tp_size=world.size, tp_group=world.compute_group, tp_ctrl=world.ctrl, ext_rows=ext_rows)
    if r.ar is not None:
        world.ar_probe = r.ar.error
    return TPRunnerProxy(world, r, cmd)


def adopt_prefixes(runner, prefixes: dict | None) -> None:
    """Follower side of TPRunnerProxy._prefixes: take the leader's token record of reused sequences."""
    for sid, toks in (prefixes or {}).items():
        seq = runner.kv.seqs.get(int(sid))
        if seq is not None:
            seq.tokens = list(toks)


def worker_main() -> None:
    rank, size = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dev, compute, ctrl_group = _init_groups(rank, size, os.environ["MASTER_ADDR"], int(os.environ["MASTER_PORT"]))
    bell = Doorbell(os.environ[ENV_DOORBELL], create=False, rank=rank, world=size) if os.environ.get(ENV_DOORBELL) else None
    ctrl = TPControl(ctrl_group, leader=False, doorbell=bell)
    from ..engine.runner import Runner
    runner = None
    while True:
        try:
            cmd = ctrl.recv_cmd()
        except RuntimeError as e:  # the leader (server process) is gone: the TP group is over
            print(f"tp rank {rank}: control channel closed ({e.__class__.__name__}); exiting", flush=True)
            os._exit(0)
        op = cmd["op"]
        if op == "exit":
            break
        if op == "load":
            runner = Runner(cmd["path"], device=dev, max_batch=cmd["max_batch"], max_seqs=cmd["max_seqs"],
                            ctx=cmd["ctx"], tp_rank=rank, tp_size=size, tp_group=compute, tp_ctrl=ctrl,
                            ext_rows=cmd.get("ext_rows", 0))
        elif op == "unload":
            if runner is not None:
                runner.close()
            runner = None
            if dev.startswith("cuda"):
                torch.cuda.empty_cache()
        elif op == "warmup":
            runner.warmup()
        elif op == "new_sequence":
            runner.new_sequence()
        elif op == "free_sequence":
            runner.free_sequence(cmd["sid"])
        elif op == "embed":
            runner.embed(cmd["tokens"])
        elif op == "set_ext":
            runner.set_ext(cmd["ids"], cmd["rows"])
        elif op == "generate":
            for _ in runner.generate(cmd["sid"], cmd["prompt"], cmd["options"], max_tokens=cmd["max_tokens"]):
                pass
        elif op == "admit":
            adopt_prefixes(runner, cmd.get("prefixes"))
            runner.admit(cmd["sid"], cmd["keep"], cmd["tokens"], cmd["opts"], cmd["history"], cmd["seed"],
                         cmd.get("n_sampled", 0))
        elif op == "admit_many":
            adopt_prefixes(runner, cmd.get("prefixes"))
            runner.admit_many(cmd["items"])
        elif op == "recompose":
            runner.recompose(cmd["rows"], cmd["tokens"])
        elif op == "decode_batch":
            runner.decode_batch(cmd["sids"], cmd["poss"])
        elif op == "evict":
            runner.evict(cmd["sid"])
        elif op == "capture_batch_graphs":
            runner.capture_batch_graphs(cmd["max_B"])
        else:
            raise RuntimeError(f"unknown TP command {op}")
    dist.barrier(group=ctrl_group)
    time.sleep(0.1)
