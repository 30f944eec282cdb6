"""Native CPU serving backend (csrc/cpu, module `_cpu`; BASELINE config 1: Phi-2 on a CPU-only node).

Weights stay quantised (the repacked streams the GPU uses); every projection is an int8 dot product
against Q8_K-style activations. Checked against plain fp32 math on the dequantised weights: the
GEMM per quant type, then whole models (prefill logits + greedy decode) against the torch twin."""
import numpy as np
import pytest
import torch

from ollama_operator_amd.gguf import GGMLType
from ollama_operator_amd.gguf.constants import FileType
from ollama_operator_amd.models.config import preset
from ollama_operator_amd.models.random_init import write_random_gguf
from ollama_operator_amd.ops.cpu import cpu_module
from ollama_operator_amd.quant import REPACK_STREAMS, dequantize, random_blocks, repack

C = cpu_module()
pytestmark = pytest.mark.skipif(C is None, reason="CPU backend module not built")


@pytest.mark.parametrize("qt", [GGMLType.Q4_0, GGMLType.Q8_0, GGMLType.Q4_K, GGMLType.Q5_K, GGMLType.Q6_K])
@pytest.mark.parametrize("K", [256, 1024 + 512, 2560])
def test_cpu_gemm_matches_fp32(qt, K):
    if qt in (GGMLType.Q4_K, GGMLType.Q5_K, GGMLType.Q6_K) and K % 256:
        pytest.skip("K-quants need whole super-blocks")
    N, B = 37, 3
    rng = np.random.default_rng(int(qt) * 1000 + K)
    raw = random_blocks(qt, N, K, rng)
    st = repack(raw, qt, N, K)
    ts = [torch.from_numpy(np.ascontiguousarray(st[n])) for n in REPACK_STREAMS[qt]]
    p = [t.data_ptr() for t in ts] + [0] * (4 - len(ts))
    tup = (p[0], p[1], p[2], p[3], N, K, int(qt))
    W = dequantize(raw, qt, N * K).reshape(N, K).astype(np.float64)
    x = torch.randn(B, K)
    y = torch.zeros(B, N)
    C.gemm(tup, 0, N, x.data_ptr(), K, B, y.data_ptr(), N, False)
    ref = x.double().numpy() @ W.T
    err = np.linalg.norm(y.numpy() - ref) / np.linalg.norm(ref)
    assert err < 1.5e-2, err
    # accumulate mode and a single row
    y1 = torch.ones(1, N)
    C.gemm(tup, 0, N, x[1:2].data_ptr(), K, 1, y1.data_ptr(), N, True)
    err1 = np.linalg.norm(y1.numpy()[0] - 1.0 - ref[1]) / np.linalg.norm(ref[1])
    assert err1 < 1.5e-2, err1
    # one dequantised row
    row = torch.zeros(((K + 255) // 256) * 256)
    C.dequant_row(tup, 5, row.data_ptr())
    np.testing.assert_allclose(row.numpy()[:K], W[5], rtol=1e-5, atol=1e-5)


PROMPT = [1, 17, 42, 99, 7, 300, 12, 5, 77, 3, 250, 11]


@pytest.mark.parametrize("name,ft", [("tiny-llama", FileType.MOSTLY_Q4_K_M), ("tiny-llama", FileType.MOSTLY_Q5_K_M),
                                     ("tiny-phi2", FileType.MOSTLY_Q4_0), ("tiny-mixtral", FileType.MOSTLY_Q8_0),
                                     ("tiny-llama", FileType.MOSTLY_Q6_K), ("tiny-gemma", FileType.MOSTLY_Q4_K_M),
                                     ("tiny-orca", FileType.MOSTLY_Q4_0)])
def test_native_cpu_runner_matches_torch_twin(tmp_path, name, ft):
    from ollama_operator_amd.engine.runner import Runner
    from ollama_operator_amd.engine.sampling import SamplingOptions
    path = str(tmp_path / "m.gguf")
    write_random_gguf(path, preset(name), ft, seed=3)
    rn = Runner(path, device="cpu", max_batch=8, max_seqs=2, ctx=64, cpu_backend="native")
    rt = Runner(path, device="cpu", max_batch=8, max_seqs=2, ctx=64, cpu_backend="torch")
    assert rn.cpu_backend == "native" and rt.cpu_backend == "torch"
    V = rn.cfg.n_vocab
    sn, st = rn.new_sequence(), rt.new_sequence()
    rn.prefill(sn, PROMPT)  # chunks of 8 + 4 rows
    rt.prefill(st, PROMPT)
    a, b = rn.logits[0, :V].numpy().copy(), rt.logits[0, :V].numpy()
    err = np.linalg.norm(a - b) / np.linalg.norm(b)
    assert err < 3e-2, err
    # teacher-forced decode steps through the same stage API
    for r in (rn, rt):
        r._set_sampler(0, SamplingOptions(temperature=0), PROMPT, 0)
    for i, tok in enumerate([5, 9, 11, 40]):
        rn.set_tokens([tok])
        rt.set_tokens([tok])
        rn.decode_step(sn, len(PROMPT) + i)
        rt.decode_step(st, len(PROMPT) + i)
        a, b = rn.logits[0, :V].numpy(), rt.logits[0, :V].numpy()
        err = np.linalg.norm(a - b) / np.linalg.norm(b)
        assert err < 3e-2, (i, err)
    toks = list(rn.generate(rn.new_sequence(), PROMPT, SamplingOptions(temperature=0), max_tokens=6))
    assert len(toks) == 6 and all(0 <= t < V for t in toks)
