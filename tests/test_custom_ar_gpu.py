"""GPU: the one-shot IPC all-reduce (csrc/kernels/allreduce.hip, parallel/custom_ar.py) with 2 and 4
ranks sharing one GPU through hipIpc handles -- the same code path as one rank per GPU over xGMI,
except that the peer pointers resolve to the local device. 1,000 back-to-back hipGraph replays of
two all-reduces each (slab rotation + epoch reuse) must match a torch sum bit for bit on every rank;
then a TP=2 model runs its whole decode step as one graph and matches TP=1 logits."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from ollama_operator_amd.gguf.constants import FileType
from ollama_operator_amd.models.config import preset
from ollama_operator_amd.models.random_init import write_random_gguf

pytestmark = pytest.mark.gpu
N = 4096 + 192  # not a multiple of the block tile: partial last block
REPLAYS = 1000


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _ar_worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.cuda.set_device(0)
        from ollama_operator_amd.ops import native
        from ollama_operator_amd.parallel.custom_ar import CustomAllReduce
        C = native()
        ar = CustomAllReduce(dist.group.WORLD, rank, world, N, timeout_s=10)
        g = torch.Generator().manual_seed(0)
        x0 = [torch.randn(N, generator=g) for _ in range(world)]  # every rank draws all ranks' inputs
        x = x0[rank].cuda()
        xs = [t.cuda() for t in x0]  # local replica of every rank's evolution (same ops, same bits)
        y = torch.zeros(N, device="cuda")
        z = torch.zeros(N, device="cuda")

        def body():
            s = torch.cuda.current_stream().cuda_stream
            x.mul_(0.999).add_(0.5)
            C.copy_d2d(ar.slab_ptr(0), x.data_ptr(), 4 * N, s)
            y.zero_()
            ar.all_reduce_add(0, y.data_ptr(), N, s)
            C.copy_d2d(ar.slab_ptr(1), y.data_ptr(), 4 * N, s)
            z.zero_()
            ar.all_reduce_add(1, z.data_ptr(), N, s)

        body()
        torch.cuda.synchronize()
        ar.check()
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            body()
        for i in range(REPLAYS):
            graph.replay()
            if i % 250 == 249:
                torch.cuda.synchronize()
                ar.check()
        torch.cuda.synchronize()
        ar.check()
        for t in xs:
            for _ in range(REPLAYS + 1):
                t.mul_(0.999).add_(0.5)
        acc = xs[0].clone()
        for t in xs[1:]:
            acc = acc + t
        zz = acc.clone()
        for _ in range(world - 1):
            zz = zz + acc
        np.save(os.path.join(out_dir, f"y{rank}.npy"), y.cpu().numpy())
        np.save(os.path.join(out_dir, f"z{rank}.npy"), z.cpu().numpy())
        np.save(os.path.join(out_dir, f"ref{rank}.npy"), acc.cpu().numpy())
        np.save(os.path.join(out_dir, f"zref{rank}.npy"), zz.cpu().numpy())
        ar.close()
    finally:
        dist.barrier()
        os._exit(0)


@pytest.mark.parametrize("world", [2, 4, 8])
def test_custom_allreduce_graph_replays(tmp_path, world):
    mp.start_processes(_ar_worker, args=(world, _port(), str(tmp_path)), nprocs=world, start_method="spawn",
                       join=True)
    y0 = np.load(tmp_path / "y0.npy")
    for r in range(world):
        y, z = np.load(tmp_path / f"y{r}.npy"), np.load(tmp_path / f"z{r}.npy")
        assert np.array_equal(y, y0), f"rank {r} differs from rank 0"  # bit-identical across ranks
        np.testing.assert_allclose(y, np.load(tmp_path / f"ref{r}.npy"), rtol=1e-6, atol=1e-6)
        np.testing.assert_allclose(z, np.load(tmp_path / f"zref{r}.npy"), rtol=1e-5, atol=1e-5)


def _stall_worker(rank, world, port, out_dir):
    """rank 1 never enters the collective: rank 0's barrier must time out into the error word (host
    mirror), leave y untouched, and fail fast (no second wait) on the next call."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import time

    import torch
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.cuda.set_device(0)
        from ollama_operator_amd.ops import native
        from ollama_operator_amd.parallel.custom_ar import CustomAllReduce, TPCollectiveError
        C = native()
        ar = CustomAllReduce(dist.group.WORLD, rank, world, N, timeout_s=0.5)
        res = {}
        if rank == 0:
            s = torch.cuda.current_stream().cuda_stream
            x = torch.ones(N, device="cuda")
            y = torch.full((N,), 7.0, device="cuda")
            C.copy_d2d(ar.slab_ptr(0), x.data_ptr(), 4 * N, s)
            t0 = time.perf_counter()
            ar.all_reduce_add(0, y.data_ptr(), N, s)
            torch.cuda.synchronize()
            res["first_s"] = time.perf_counter() - t0
            res["err"] = ar.error()
            t0 = time.perf_counter()
            ar.all_reduce_add(1, y.data_ptr(), N, s)  # fail fast: no second 0.5 s wait
            torch.cuda.synchronize()
            res["second_s"] = time.perf_counter() - t0
            res["y_untouched"] = bool(torch.all(y == 7.0).item())
            try:
                ar.check()
                res["raised"] = False
            except TPCollectiveError:
                res["raised"] = True
            np.save(os.path.join(out_dir, "stall.npy"), np.array([res["first_s"], res["err"], res["second_s"],
                                                                   res["y_untouched"], res["raised"]], float))
        dist.barrier()
        ar.close()
    finally:
        dist.barrier()
        os._exit(0)


def test_custom_allreduce_stalled_peer_times_out(tmp_path):
    mp.start_processes(_stall_worker, args=(2, _port(), str(tmp_path)), nprocs=2, start_method="spawn", join=True)
    first_s, err, second_s, untouched, raised = np.load(tmp_path / "stall.npy")
    assert err == 2, "error word must name peer 1 (1 + rank)"
    assert 0.4 < first_s < 10
    assert second_s < 0.4, "a failed group must not wait again"
    assert untouched == 1.0, "slab reads must be skipped after a failed barrier"
    assert raised == 1.0


def _emit_worker(rank, world, port, out_dir):
    """the fused all-reduce + residual + int8-chain emission (ar_allreduce_add_emit), 2 batch rows"""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.cuda.set_device(0)
        from ollama_operator_amd.ops import native
        from ollama_operator_amd.parallel.custom_ar import CustomAllReduce
        C = native()
        E, B = 4096, 2
        ar = CustomAllReduce(dist.group.WORLD, rank, world, B * E, timeout_s=10)
        g = torch.Generator().manual_seed(3)
        parts = [torch.randn(B * E, generator=g) for _ in range(world)]
        y0 = torch.randn(B * E, generator=g)
        nw = torch.rand(E, generator=g) + 0.5
        s = torch.cuda.current_stream().cuda_stream
        x = parts[rank].cuda()
        y = y0.cuda()
        nwd = nw.cuda()
        img = torch.zeros(B * C.x8_bytes(E), dtype=torch.uint8, device="cuda")
        st = torch.zeros(B * C.x8_stat_ld(E) + 4, device="cuda")
        C.copy_d2d(ar.slab_ptr(1), x.data_ptr(), 4 * B * E, s)
        ar.all_reduce_add_emit(1, y.data_ptr(), E, B, img.data_ptr(), nwd.data_ptr(), st.data_ptr(), s)
        torch.cuda.synchronize()
        ar.check()
        ref = y0.clone()
        for t in parts:
            ref = ref + t
        np.save(os.path.join(out_dir, f"ey{rank}.npy"), y.cpu().numpy())
        np.save(os.path.join(out_dir, f"eref{rank}.npy"), ref.numpy())
        np.save(os.path.join(out_dir, f"eimg{rank}.npy"), img.cpu().numpy())
        np.save(os.path.join(out_dir, f"est{rank}.npy"), st.cpu().numpy())
        np.save(os.path.join(out_dir, "enw.npy"), nw.numpy())
        ar.close()
    finally:
        dist.barrier()
        os._exit(0)


@pytest.mark.parametrize("world", [2, 8])
def test_allreduce_emits_int8_chain_image(tmp_path, world):
    """TP decode on the int8 chain: the all-reduce itself writes the next GEMV's image + RMS partials
    (world 8: the ar_add_emit_kernel<8> instantiation TP=8 decode runs)."""
    from test_gemv8_gpu import decode_image
    from ollama_operator_amd.ops import native
    E, B = 4096, 2
    mp.start_processes(_emit_worker, args=(world, _port(), str(tmp_path)), nprocs=world, start_method="spawn",
                       join=True)
    C = native()
    nw = np.load(tmp_path / "enw.npy")
    img0 = np.load(tmp_path / "eimg0.npy")
    for r in range(world):
        y, ref = np.load(tmp_path / f"ey{r}.npy"), np.load(tmp_path / f"eref{r}.npy")
        np.testing.assert_allclose(y, ref, rtol=1e-6, atol=1e-6)
        assert np.array_equal(np.load(tmp_path / f"eimg{r}.npy"), img0)  # identical on every rank
    st = np.load(tmp_path / "est0.npy")
    nb, sl = C.x8_bytes(E), C.x8_stat_ld(E)
    import torch
    for b in range(B):
        yb = ref[b * E:(b + 1) * E]
        got = decode_image(torch.from_numpy(img0[b * nb:(b + 1) * nb].copy()), E).numpy()
        want = yb * nw
        assert np.linalg.norm(got - want) / np.linalg.norm(want) < 1.5e-2
        np.testing.assert_allclose(st[b * sl:b * sl + E // 16], (yb.reshape(-1, 16) ** 2).sum(1), rtol=1e-4)


PROMPT = [1, 17, 42, 99, 7, 300, 12, 5, 77]


def _tp_worker(rank, world, port, path, out_dir, mode="custom"):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    if mode == "eager":  # every stage through the eager collective path (torch.distributed)
        os.environ["OMX_CUSTOM_AR"] = "0"
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from ollama_operator_amd.engine.runner import Runner
        # "long": prefill chunks of 32 rows exceed the 16-row all-reduce slabs, so prefill takes the
        # eager collective path and decode the one-shot graph path
        mb = 32 if mode == "long" else 4
        r = Runner(path, device="cuda:0", max_batch=mb, max_seqs=2, ctx=96, tp_rank=rank, tp_size=world,
                   tp_group=dist.group.WORLD)
        if mode == "eager":
            assert r.ar is None and not r.use_graphs
        else:
            assert r.ar is not None and r.use_graphs
        if mode == "long":
            assert not r.exe.ar_fits(32)
        from ollama_operator_amd.ops import native
        native().reset_launch_counts()
        np.save(os.path.join(out_dir, f"p{rank}.npy"), _run(r, LONG_PROMPT if mode == "long" else PROMPT))
        n = native().launch_counts()  # decode graph captured inside _run: its forward_tp kernels counted
        np.save(os.path.join(out_dir, f"n{rank}.npy"), np.array([n["gemv8_row1"] + n["gemv8_dual"], r.exe.exe.x8_on]))
        if r.ar is not None:
            r.ar.check()
        r.close()
    finally:
        dist.barrier()
        os._exit(0)


LONG_PROMPT = [1] + [(7 * i + 3) % 250 + 2 for i in range(40)]


def _run(r, prompt=PROMPT):
    """prefill (chunks of max_batch through forward_tp or the eager stages), then 3 decode steps with
    fixed input tokens"""
    sid = r.new_sequence()
    r.prefill(sid, prompt)
    out = [r.full_logits[0, :r.cfg.n_vocab].cpu().numpy()]
    for i, tok in enumerate([5, 9, 11]):
        r.set_tokens([tok])
        r.decode_step(sid, len(prompt) + i)
        out.append(r.full_logits[0, :r.cfg.n_vocab].cpu().numpy())
    return np.stack(out)


@pytest.mark.parametrize("name,ft", [("tiny-llama-tp", FileType.MOSTLY_Q4_K_M),
                                     ("tiny-llama-tp-odd", FileType.MOSTLY_Q4_K_M),
                                     ("tiny-mixtral-tp", FileType.MOSTLY_Q8_0)])
def test_tp2_graph_decode_matches_tp1(tmp_path, name, ft):
    path = str(tmp_path / f"{name}.gguf")
    write_random_gguf(path, preset(name), ft, seed=5)
    from ollama_operator_amd.engine.runner import Runner
    r1 = Runner(path, device="cuda:0", max_batch=4, max_seqs=2, ctx=64)
    ref = _run(r1)
    del r1
    mp.start_processes(_tp_worker, args=(2, _port(), path, str(tmp_path)), nprocs=2, start_method="spawn",
                       join=True)
    _check_tp(tmp_path, ref)
    if "mixtral" not in name:  # dense llama ranks decode on the int8 chain (the all-reduce emits its images)
        for rank in range(2):
            n8, on = np.load(tmp_path / f"n{rank}.npy")
            assert on == 1 and n8 > 0, (rank, n8, on)


def _check_tp(tmp_path, ref, world=2):
    p0 = np.load(tmp_path / "p0.npy")
    for rank in range(world):
        got = np.load(tmp_path / f"p{rank}.npy")
        assert np.array_equal(got, p0), "TP ranks must hold bit-identical logits"
        for i in range(len(ref)):
            err = np.linalg.norm(got[i] - ref[i]) / np.linalg.norm(ref[i])
            assert err < 2e-2, (i, err)


@pytest.mark.parametrize("mode", ["eager", "long"])
def test_tp2_collective_stage_paths_match_tp1(tmp_path, mode):
    """The eager (torch.distributed) stage path: forced for every step (OMX_CUSTOM_AR=0), and taken by
    prefill chunks wider than the one-shot slabs."""
    path = str(tmp_path / "tiny.gguf")
    write_random_gguf(path, preset("tiny-llama-tp"), FileType.MOSTLY_Q4_K_M, seed=5)
    from ollama_operator_amd.engine.runner import Runner
    prompt = LONG_PROMPT if mode == "long" else PROMPT
    r1 = Runner(path, device="cuda:0", max_batch=32 if mode == "long" else 4, max_seqs=2, ctx=96)
    ref = _run(r1, prompt)
    del r1
    mp.start_processes(_tp_worker, args=(2, _port(), path, str(tmp_path), mode), nprocs=2, start_method="spawn",
                       join=True)
    _check_tp(tmp_path, ref)


def test_tp8_graph_decode_matches_tp1(tmp_path):
    """TP = 8 (BASELINE config 4's degree) with 8 ranks sharing one GPU: the whole decode step of every rank
    is one graph on the int8 chain with the fused all-reduce emission at world 8, and the logits match
    TP = 1. No cross-GPU run exists here (one GPU per box); the collective code path is the same."""
    path = str(tmp_path / "tiny-tp8.gguf")
    write_random_gguf(path, preset("tiny-llama-tp8"), FileType.MOSTLY_Q4_K_M, seed=5)
    from ollama_operator_amd.engine.runner import Runner
    r1 = Runner(path, device="cuda:0", max_batch=4, max_seqs=2, ctx=64)
    ref = _run(r1)
    del r1
    mp.start_processes(_tp_worker, args=(8, _port(), path, str(tmp_path)), nprocs=8, start_method="spawn",
                       join=True)
    _check_tp(tmp_path, ref, world=8)
    for rank in range(8):
        n8, on = np.load(tmp_path / f"n{rank}.npy")
        assert on == 1 and n8 > 0, (rank, n8, on)
