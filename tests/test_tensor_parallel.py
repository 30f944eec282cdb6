"""Tensor parallelism on CPU: world_size=2 gloo ranks run the sharded runner (Megatron column/row
splits on head / 256-block boundaries, all-reduce after O and down, vocab-sharded LM head +
all-gather) and must reproduce the TP=1 logits and greedy tokens (SURVEY.md §4 "TP correctness on
CPU with a gloo fake RCCL")."""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from ollama_operator_amd.gguf.constants import FileType
from ollama_operator_amd.models.config import preset
from ollama_operator_amd.models.random_init import write_random_gguf

PROMPT = [1, 17, 42, 99, 7, 300, 12, 5, 77]


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, path, out_dir):
    import faulthandler
    faulthandler.enable()
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from ollama_operator_amd.engine.runner import Runner
        from ollama_operator_amd.engine.sampling import SamplingOptions
        r = Runner(path, device="cpu", max_batch=4, max_seqs=2, ctx=64, tp_rank=rank, tp_size=world,
                   tp_group=dist.group.WORLD)
        sid = r.new_sequence()
        r.prefill(sid, PROMPT)
        logits = r.full_logits[0, :r.cfg.n_vocab].clone()
        toks = list(r.generate(r.new_sequence(), PROMPT, SamplingOptions(temperature=0, repeat_penalty=1.0),
                               max_tokens=5))
        np.save(os.path.join(out_dir, f"logits{rank}.npy"), logits.numpy())
        np.save(os.path.join(out_dir, f"toks{rank}.npy"), np.array(toks))
    finally:
        # gloo's background threads can abort the process if one rank tears the pair down while
        # the other is still exiting; synchronise, then leave without running C++ destructors
        dist.barrier()
        os._exit(0)


@pytest.mark.parametrize("name,ft,world", [("tiny-llama-tp", FileType.MOSTLY_Q4_K_M, 2),
                                           ("tiny-llama-tp-odd", FileType.MOSTLY_Q4_K_M, 2),
                                           ("tiny-phi2-tp", FileType.MOSTLY_Q4_0, 2),
                                           ("tiny-mixtral-tp", FileType.MOSTLY_Q8_0, 2),
                                           ("tiny-llama-tp8", FileType.MOSTLY_Q4_K_M, 8)])
def test_tp2_matches_tp1(tmp_path, name, ft, world):
    path = str(tmp_path / f"{name}.gguf")
    write_random_gguf(path, preset(name), ft, seed=5)
    from ollama_operator_amd.engine.runner import Runner
    from ollama_operator_amd.engine.sampling import SamplingOptions
    r1 = Runner(path, device="cpu", max_batch=4, max_seqs=2, ctx=64)
    sid = r1.new_sequence()
    r1.prefill(sid, PROMPT)
    ref = r1.logits[0, :r1.cfg.n_vocab].numpy().copy()
    ref_toks = list(r1.generate(r1.new_sequence(), PROMPT, SamplingOptions(temperature=0, repeat_penalty=1.0),
                                max_tokens=5))
    mp.start_processes(_worker, args=(world, _port(), path, str(tmp_path)), nprocs=world, start_method="spawn",
                       join=True)
    for rank in range(world):
        got = np.load(tmp_path / f"logits{rank}.npy")
        np.testing.assert_allclose(got, ref, rtol=1e-3, atol=1e-3)
        assert np.load(tmp_path / f"toks{rank}.npy").tolist() == ref_toks


def test_tp_rejects_indivisible(tmp_path):
    from ollama_operator_amd.engine.weights import DeviceWeights
    path = str(tmp_path / "t.gguf")
    write_random_gguf(path, preset("tiny-llama"), FileType.MOSTLY_Q4_K_M, seed=1)
    with pytest.raises(ValueError):
        DeviceWeights(path, "cpu", tp_rank=0, tp_size=2)  # K=256: one super-block cannot be split


def test_tp_watchdog_exits_when_a_worker_dies():
    """A dead TP worker must take the server down (non-zero), not leave it answering while hung."""
    import subprocess
    import sys
    import threading

    from ollama_operator_amd.parallel.tp import TPWorld, _watchdog
    dead = subprocess.Popen([sys.executable, "-c", "import sys; sys.exit(3)"])
    alive = subprocess.Popen([sys.executable, "-c", "import time; time.sleep(30)"])
    dead.wait()
    world = TPWorld(0, 3, "cpu", None, None, [alive, dead])
    codes = []
    t = threading.Thread(target=_watchdog, args=(world, 0.05, codes.append))
    t.start()
    t.join(10)
    assert codes == [3]
    assert alive.wait(10) is not None  # the surviving rank is killed with the group


def test_tp_watchdog_quiet_on_shutdown():
    import subprocess
    import sys
    import threading

    from ollama_operator_amd.parallel.tp import TPWorld, _watchdog
    done = subprocess.Popen([sys.executable, "-c", "pass"])
    done.wait()
    world = TPWorld(0, 2, "cpu", None, None, [done])
    world.stopping.set()
    codes = []
    t = threading.Thread(target=_watchdog, args=(world, 0.05, codes.append))
    t.start()
    t.join(5)
    assert codes == []


def test_tp_watchdog_exits_on_allreduce_error():
    """A one-shot all-reduce barrier timeout on the leader (a wedged peer) must end the
    server non-zero even though every worker process is still alive."""
    import subprocess
    import sys
    import threading

    from ollama_operator_amd.parallel.tp import TPWorld, _watchdog
    alive = subprocess.Popen([sys.executable, "-c", "import time; time.sleep(30)"])
    world = TPWorld(0, 2, "cpu", None, None, [alive])
    err = [0]
    world.ar_probe = lambda: err[0]
    codes = []
    t = threading.Thread(target=_watchdog, args=(world, 0.05, codes.append))
    t.start()
    import time
    time.sleep(0.2)
    assert codes == []  # healthy: quiet
    err[0] = 2  # peer 1 missed a barrier
    t.join(10)
    assert codes == [1]
    assert alive.wait(10) is not None


def test_tp_collective_error_is_a_device_fault():
    from ollama_operator_amd.parallel.custom_ar import TPCollectiveError
    from ollama_operator_amd.server.app import is_device_fault
    assert is_device_fault(TPCollectiveError("peer 1 missed an all-reduce barrier"))
    assert not is_device_fault(RuntimeError("out of KV blocks"))
