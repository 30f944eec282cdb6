"""Probe: B=4 int8 batch GEMV with / without a layout-M copy attached (test_mb_path_is_taken failure)."""
import sys
import torch
sys.path.insert(0, "tests")
sys.path.insert(0, ".")
from ollama_operator_amd.gguf import GGMLType  # noqa: E402
from test_kernels_gpu import QM, C, S, gemv, rel  # noqa: E402

for qt in [GGMLType.Q4_0, GGMLType.Q4_K]:
    m = QM(qt, 64, 512, seed=1)
    x = torch.randn(4, 512, device="cuda")
    for mode in ["plain", "mt_zero"]:
        tup0 = m.tup
        if mode == "mt_zero":
            mt = torch.zeros(C().mfma_layout_bytes(int(qt), 64, 512), dtype=torch.uint8, device="cuda")
            m.tup = tup0 + (0, mt.data_ptr())
        for en in (1, 0):
            C().set_mb_enable(en)
            y = torch.full((4, 64), 7.0, device="cuda")
            gemv(m, x, y=y)
            torch.cuda.synchronize()
            print(qt.name, mode, "mb", en, "rel", rel(y, x @ m.w.T), "max", float(y.abs().max()), flush=True)
        C().set_mb_enable(1)
        m.tup = tup0
