"""bench.py's multi-rank orchestration (the driver's contract), rehearsed on the CPU:
`--gpus N` without torchrun launches the N data-parallel ranks itself and reports `n_gpus == N`;
fewer visible GPUs than requested is a non-zero exit, never a silent 1-GPU number; `--tp T` runs
the tensor-parallel serving stack and reports `tpT`."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TINY = ["--model", "tiny-llama-tp", "--ftype", "Q4_K_M", "--steps", "3", "--warmup", "1", "--prompt", "8",
        "--chunk", "16", "--via-server", "0", "--ttft-long", "0"]


def _run(args, tmp_path, timeout=300):
    env = dict(os.environ)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args, "--dir", str(tmp_path)],
                          capture_output=True, text=True, timeout=timeout, env=env, cwd=str(tmp_path))


def _json_lines(out: str):
    return [json.loads(l) for l in out.splitlines() if l.startswith("{")]


def test_bench_gpus2_launches_two_ranks(tmp_path):
    p = _run(["--gpus", "2", "--device", "cpu", *TINY], tmp_path)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = _json_lines(p.stdout)
    assert len(lines) == 1, p.stdout  # rank 0 only
    d = lines[0]
    assert d["n_gpus"] == 2 and d["config"]["parallelism"] == "dp2" and d["config"]["global_batch"] == 2
    assert d["value"] > 0 and d["steps"] == 3 and d["warmup"] == 1


@pytest.mark.skipif(__import__("torch").cuda.device_count() >= 2, reason="needs a box with < 2 GPUs")
def test_bench_refuses_more_gpus_than_visible(tmp_path):
    p = _run(["--gpus", "2", *TINY], tmp_path, timeout=120)
    assert p.returncode != 0
    assert "refusing" in p.stderr
    assert not _json_lines(p.stdout)


def test_bench_world_size_mismatch_fails(tmp_path):
    env_args = ["--gpus", "2", "--device", "cpu", *TINY]
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *env_args, "--dir", str(tmp_path)],
                       capture_output=True, text=True, timeout=120, env=env, cwd=str(tmp_path))
    assert p.returncode != 0 and "WORLD_SIZE" in p.stderr


def test_bench_tp2_cpu(tmp_path):
    p = _run(["--tp", "2", "--device", "cpu", *TINY], tmp_path)
    assert p.returncode == 0, p.stderr[-3000:]
    (d,) = _json_lines(p.stdout)
    assert d["n_gpus"] == 2 and d["config"]["parallelism"] == "tp2" and d["scaling"] == "strong"
    assert d["value"] > 0
