import os
import sys
import zlib

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (gfx950) GPU and the built HIP extension")
    config.addinivalue_line("markers", "slow: long-running test")


def pytest_collection_modifyitems(config, items):
    try:
        import torch
        has_gpu = torch.cuda.is_available()
    except Exception:
        has_gpu = False
    if has_gpu:
        return
    skip = pytest.mark.skip(reason="no GPU in this environment")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)


@pytest.fixture(scope="session")
def tiny_models(tmp_path_factory):
    """Random-init GGUF fixtures for each architecture family (quantized from float weights)."""
    from ollama_operator_amd.gguf.constants import FileType
    from ollama_operator_amd.models.config import preset
    from ollama_operator_amd.models.random_init import write_random_gguf
    d = tmp_path_factory.mktemp("models")
    out = {}
    for name, ft in [("tiny-llama", FileType.MOSTLY_Q4_K_M), ("tiny-mixtral", FileType.MOSTLY_Q4_K_M),
                     ("tiny-phi2", FileType.MOSTLY_Q4_0), ("tiny-llama-q8", FileType.MOSTLY_Q8_0),
                     ("tiny-llama-q40", FileType.MOSTLY_Q4_0), ("tiny-llama-q5km", FileType.MOSTLY_Q5_K_M),
                     ("tiny-mixtral-q5ks", FileType.MOSTLY_Q5_K_S), ("tiny-gemma", FileType.MOSTLY_Q4_K_M),
                     ("tiny-orca", FileType.MOSTLY_Q4_0)]:
        base = name.replace("-q8", "").replace("-q40", "").replace("-q5km", "").replace("-q5ks", "")
        p = str(d / f"{name}.gguf")
        write_random_gguf(p, preset(base), ft, seed=zlib.crc32(name.encode()) % 1000, quantize_from_float=True)
        out[name] = p
    return out

# CPU runners in the test suite default to the fp32 torch twin (the numerical oracle the GPU engine
# is checked against); the native CPU backend has its own tests (tests/test_cpu_backend.py), which
# ask for it explicitly.
os.environ.setdefault("OMX_CPU_BACKEND", "torch")
