"""The debug kernel build: `build_native.py --debug` compiles the gfx950 kernels with
the in-kernel bounds assertions (OMX_KASSERT -> device assert) at -O1 -g. This CPU-side check compiles
the kernels that carry assertions (GEMV index math, matrix-core GEMV records, attention block table)
and confirms the assertion text is in the device code; the release objects must not contain it."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

pytestmark = pytest.mark.skipif(not os.path.exists("/opt/rocm/bin/hipcc"), reason="needs hipcc")


def _strings(obj):
    return subprocess.run(["strings", obj], capture_output=True, text=True).stdout


def test_debug_kernels_compile_with_asserts(tmp_path, monkeypatch):
    import sys
    sys.path.insert(0, ROOT)
    import build_native
    monkeypatch.setattr(build_native, "DEBUG_BUILD", str(tmp_path / "debug"))
    srcs = ["kernels/attention.hip", "kernels/gemv_mfma.hip"]
    d = build_native.build(debug=True, sources=srcs, jobs=2)
    objs = [os.path.join(d, s.replace("/", "_") + ".o") for s in srcs]
    for o in objs:
        assert os.path.exists(o)
    if shutil.which("strings"):
        txt = _strings(objs[0]) + _strings(objs[1])
        assert "blk >= 0" in txt and "tile < (w.N + 15) / 16" in txt
