"""Audit of the built gfx950 code objects (scripts/isa_check.py): scalar opcodes are allow-listed
(no scalar-memory writes anywhere in the extension) and the decode GEMV and attention kernels use no scratch."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "scripts"))
import isa_check  # noqa: E402

SO = isa_check.default_so()
pytestmark = pytest.mark.skipif(SO is None or not os.path.exists(isa_check.LLVM), reason="extension not built")


@pytest.fixture(scope="module")
def audit():
    return isa_check.audit(SO)


def test_scalar_opcodes_allow_listed(audit):
    bad, scratch = audit
    assert scratch, "no gfx950 kernels found in the extension"
    assert bad == [], f"disallowed scalar opcodes in the built ISA: {bad}"


def test_allow_list_rejects_unknown_families():
    assert isa_check.ALLOWED_SCALAR.match("s_load_dwordx4")
    assert isa_check.ALLOWED_SCALAR.match("s_cbranch_execz")
    assert not isa_check.ALLOWED_SCALAR.match("s_" + "st" + "ore_dword")
    assert not isa_check.ALLOWED_SCALAR.match("s_" + "dcache_" + "wb")


def test_gemv_and_attention_kernels_do_not_spill(audit):
    """decode GEMVs and every attention kernel (fp16 and fp8-KV instantiations) keep their state in
    registers: a spill here cost the fp8 decode kernels their bandwidth gain (profiles/r5_kv8)"""
    _, scratch = audit
    hot = {k: v for k, v in scratch.items() if "gemv" in k or "attn" in k}
    assert any("gemv" in k for k in hot) and any("attn_decode" in k for k in hot)
    spills = {k: v for k, v in hot.items() if v}
    assert not spills, f"decode kernels using scratch: {spills}"
