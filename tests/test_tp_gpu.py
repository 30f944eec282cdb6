"""GPU: the native executor's tensor-parallel path (partial sums -> all-reduce -> residual add,
vocab-sharded head + all-gather) with 2 ranks sharing one GPU over gloo (RCCL needs one GPU per
rank; the 8-GPU RCCL run is the driver's). Logits must match the TP=1 native run."""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from ollama_operator_amd.gguf.constants import FileType
from ollama_operator_amd.models.config import preset
from ollama_operator_amd.models.random_init import write_random_gguf

pytestmark = pytest.mark.gpu
PROMPT = [1, 17, 42, 99, 7, 300, 12, 5, 77]


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, path, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from ollama_operator_amd.engine.runner import Runner
        r = Runner(path, device="cuda:0", max_batch=4, max_seqs=2, ctx=64, tp_rank=rank, tp_size=world,
                   tp_group=dist.group.WORLD, use_graphs=False)
        sid = r.new_sequence()
        r.prefill(sid, PROMPT)
        np.save(os.path.join(out_dir, f"g{rank}.npy"), r.full_logits[0, :r.cfg.n_vocab].cpu().numpy())
    finally:
        dist.barrier()
        os._exit(0)


@pytest.mark.parametrize("name,ft", [("tiny-llama-tp", FileType.MOSTLY_Q4_K_M),
                                     ("tiny-mixtral-tp", FileType.MOSTLY_Q8_0),
                                     ("tiny-phi2-tp", FileType.MOSTLY_Q4_0)])
def test_native_tp2_matches_tp1(tmp_path, name, ft):
    path = str(tmp_path / f"{name}.gguf")
    write_random_gguf(path, preset(name), ft, seed=5)
    from ollama_operator_amd.engine.runner import Runner
    r1 = Runner(path, device="cuda:0", max_batch=4, max_seqs=2, ctx=64)
    r1.prefill(r1.new_sequence(), PROMPT)
    ref = r1.logits[0, :r1.cfg.n_vocab].cpu().numpy()
    del r1
    mp.start_processes(_worker, args=(2, _port(), path, str(tmp_path)), nprocs=2, start_method="spawn", join=True)
    for rank in range(2):
        got = np.load(tmp_path / f"g{rank}.npy")
        err = np.linalg.norm(got - ref) / np.linalg.norm(ref)
        assert err < 2e-2, err
