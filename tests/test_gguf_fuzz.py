"""GGUF parser robustness: model files are untrusted input.
  * the Python reader must accept or raise ValueError/EOFError-style errors on mutated files;
  * the native C++ loader is built host-only with AddressSanitizer + UBSan (g++) and run over the
    same mutated corpus -- it must reject bad files with an exception, never touch memory outside
    the mapping (any sanitizer report fails the test)."""
import os
import shutil
import subprocess

import numpy as np
import pytest
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

from ollama_operator_amd.gguf import read_gguf
from ollama_operator_amd.gguf.constants import FileType
from ollama_operator_amd.models.config import preset
from ollama_operator_amd.models.random_init import write_random_gguf

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def seed_gguf(tmp_path_factory):
    p = str(tmp_path_factory.mktemp("fuzz") / "seed.gguf")
    cfg = preset("tiny-llama", n_layer=1, n_vocab=64)
    write_random_gguf(p, cfg, FileType.MOSTLY_Q4_K_M, seed=3)
    return p


def mutate(data: bytes, rng: np.random.Generator) -> bytes:
    b = bytearray(data)
    kind = rng.integers(0, 4)
    if kind == 0:  # truncate
        return bytes(b[: rng.integers(0, len(b))])
    if kind == 1:  # flip bytes in the header / metadata / tensor-info region
        for _ in range(rng.integers(1, 16)):
            i = int(rng.integers(0, min(len(b), 4096)))
            b[i] ^= int(rng.integers(1, 256))
        return bytes(b)
    if kind == 2:  # overwrite a 64-bit field with an extreme value
        i = int(rng.integers(4, min(len(b), 2048) - 8))
        vals = [0, 2**31 - 1, 2**32, 2**63 - 1, 2**64 - 1]
        b[i:i + 8] = vals[int(rng.integers(0, len(vals)))].to_bytes(8, "little")
        return bytes(b)
    i = int(rng.integers(0, len(b)))  # splice garbage
    return bytes(b[:i]) + rng.bytes(int(rng.integers(1, 512))) + bytes(b[i:])


@settings(max_examples=150, deadline=None, suppress_health_check=[HealthCheck.function_scoped_fixture])
@given(seed=st.integers(0, 2**31 - 1))
def test_python_reader_rejects_cleanly(seed, seed_gguf, tmp_path):
    data = open(seed_gguf, "rb").read()
    p = tmp_path / "m.gguf"
    p.write_bytes(mutate(data, np.random.default_rng(seed)))
    try:
        g = read_gguf(str(p))
        for name in list(g.tensors)[:4]:
            g.raw(name)
    except (ValueError, EOFError, KeyError, UnicodeDecodeError, OverflowError, MemoryError):
        pass


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_native_loader_under_asan(seed_gguf, tmp_path):
    exe = str(tmp_path / "gguf_fuzz")
    cmd = ["g++", "-std=c++17", "-O1", "-g", "-fsanitize=address,undefined", "-fno-omit-frame-pointer",
           "-fno-sanitize-recover=undefined", os.path.join(ROOT, "csrc/tools/gguf_fuzz_main.cpp"),
           os.path.join(ROOT, "csrc/gguf/gguf.cpp"), "-I", os.path.join(ROOT, "csrc"), "-lpthread", "-o", exe]
    subprocess.run(cmd, check=True, capture_output=True, timeout=300)
    data = open(seed_gguf, "rb").read()
    rng = np.random.default_rng(0)
    files = [seed_gguf]
    for i in range(200):
        p = tmp_path / f"m{i}.gguf"
        p.write_bytes(mutate(data, rng))
        files.append(str(p))
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1", UBSAN_OPTIONS="print_stacktrace=1")
    env.pop("LD_PRELOAD", None)
    r = subprocess.run([exe, *files], capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stderr[-4000:]
    assert "AddressSanitizer" not in r.stderr and "runtime error" not in r.stderr, r.stderr[-4000:]
    assert f"{seed_gguf}: ok" in r.stdout
    assert "rejected" in r.stdout  # the corpus does exercise the error paths
