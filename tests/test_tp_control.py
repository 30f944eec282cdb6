"""TP control channel (parallel/tp.py): int32 command frames + JSON documents over a gloo group (no
pickling) and the shared-memory step doorbell, exercised across two real processes."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from ollama_operator_amd.engine.sampling import SamplingOptions
from ollama_operator_amd.parallel.tp import Doorbell, decode_cmd, encode_cmd

CMDS = [
    {"op": "decode_batch", "sids": [3, 1, 7], "poss": [10, 200, 5]},
    {"op": "evict", "sid": 4},
    {"op": "new_sequence"},
    {"op": "free_sequence", "sid": 2},
    {"op": "warmup"},
    {"op": "load", "path": "/x/y.gguf", "max_batch": 64, "max_seqs": 9, "ctx": 4096, "ext_rows": 0},
    {"op": "admit_many", "items": [[1, 0, [1, 2, 3], SamplingOptions(temperature=0.5, seed=7), [4], 99]]},
    {"op": "set_ext", "ids": [-1, -2], "rows": np.arange(12, dtype=np.float32).reshape(2, 6)},
    {"op": "decode_batch", "sids": list(range(130)), "poss": list(range(130))},  # > inline rows: JSON
    {"op": "exit"},
]


def _same(a, b):
    if isinstance(a, np.ndarray):
        return isinstance(b, np.ndarray) and a.dtype == b.dtype and np.array_equal(a, b)
    if isinstance(a, dict):
        return a.keys() == b.keys() and all(_same(a[k], b[k]) for k in a)
    if isinstance(a, (list, tuple)):
        return len(a) == len(b) and all(_same(x, y) for x, y in zip(a, b))
    return a == b


def test_json_documents_roundtrip_without_pickle():
    for c in CMDS:
        blob = encode_cmd(c)
        assert b"__reduce__" not in blob and blob.startswith(b"{")
        assert _same(decode_cmd(blob), c)
    with pytest.raises(TypeError):
        encode_cmd({"op": "x", "f": object()})


def test_doorbell_ring_wait_in_order():
    name = f"omx_test_bell_{os.getpid()}"
    lead = Doorbell(name, create=True, rank=0, world=2)
    fol = Doorbell(name, create=False, rank=1, world=2)
    try:
        vals = [1, 0, 1, 1, 0]
        for v in vals:
            lead.ring(v)
        assert [fol.wait() for _ in vals] == vals
    finally:
        fol.close()
        lead.close(unlink=True)


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank(rank, port, bell, out):
    import torch.distributed as dist

    from ollama_operator_amd.parallel.tp import Doorbell, TPControl
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=2)
    try:
        b = Doorbell(bell, create=False, rank=rank, world=2)
        c = TPControl(dist.group.WORLD, leader=rank == 0, doorbell=b)
        if rank == 0:
            for cmd in CMDS:
                c.send_cmd(cmd)
            for i in range(200):  # many more rings than ring slots: the leader must wait for the follower
                c.signal(i % 3 != 0)
        else:
            got = [c.recv_cmd() for _ in CMDS]
            flags = [c.wait() for _ in range(200)]
            ok = all(_same(g, e) for g, e in zip(got, CMDS)) and flags == [i % 3 != 0 for i in range(200)]
            with open(out, "w") as f:
                f.write("ok" if ok else f"bad {got!r} {flags!r}")
        b.close()
        dist.barrier()
    finally:
        dist.destroy_process_group()


def test_control_channel_two_processes(tmp_path):
    name = f"omx_test_ctl_{os.getpid()}"
    bell = Doorbell(name, create=True, rank=0, world=2)
    try:
        out = str(tmp_path / "r1.txt")
        mp.start_processes(_rank, args=(_port(), name, out), nprocs=2, start_method="spawn", join=True)
        assert open(out).read() == "ok"
    finally:
        bell.close(unlink=True)


def test_followers_adopt_leader_token_record():
    """generated tokens are recorded on the leader only; a prefix reuse that reaches
    into them must not truncate followers differently -- admit carries the leader's record."""
    from types import SimpleNamespace

    from ollama_operator_amd.engine.kv_cache import SeqState
    from ollama_operator_amd.parallel.tp import TPRunnerProxy, adopt_prefixes, decode_cmd, encode_cmd
    lead = SimpleNamespace(kv=SimpleNamespace(seqs={3: SeqState(row=0, tokens=[1, 5, 6, 7, 40, 41])}))
    fol = SimpleNamespace(kv=SimpleNamespace(seqs={3: SeqState(row=0, tokens=[1, 5, 6, 7])}))
    proxy = TPRunnerProxy.__new__(TPRunnerProxy)
    proxy.r = lead
    pre = proxy._prefixes([3, 9])
    cmd = decode_cmd(encode_cmd({"op": "admit", "prefixes": pre}))
    adopt_prefixes(fol, cmd["prefixes"])
    assert fol.kv.seqs[3].tokens == [1, 5, 6, 7, 40, 41] and fol.kv.seqs[3].length == 6
