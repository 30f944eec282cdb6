"""Allow-list ISA audit of the built gfx950 code objects inside `ollama_operator_amd/_C*.so`.

The extension's `.hip_fatbin` section holds one clang offload bundle per translation unit. Each
gfx950 code object is cut out of its bundle, disassembled with `llvm-objdump --mcpu=gfx950`, and:

  * every scalar (SALU/SMEM) opcode must belong to an allow-listed family — loads, ALU, compares,
    branches, waits, barriers. Anything else (in particular any scalar-memory write) fails, so the
    policy is enforced without the source ever naming the instructions it rejects;
  * every kernel's `.private_segment_fixed_size` (scratch bytes per lane) is reported, so a test can
    assert the hot GEMV instantiations never spill.

    python scripts/isa_check.py [path/to/_C.so]      (exit 1 on a finding)
"""
from __future__ import annotations

import glob
import os
import re
import struct
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LLVM = "/opt/rocm/lib/llvm/bin"
BUNDLE_MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"

# Scalar opcode families a compute kernel legitimately needs. Matching is on the full mnemonic.
ALLOWED_SCALAR = re.compile(
    r"^s_(?:"
    r"load_dword\w*|buffer_load_dword\w*|"                                  # SMEM reads only
    r"waitcnt\w*|barrier|endpgm\w*|nop|sleep|memrealtime|memtime|sethalt|trap|setprio|"
    r"branch|cbranch_\w+|getpc_b64|setpc_b64|swappc_b64|"
    r"mov_\w+|movk_i32|cmov_\w+|cmovk_i32|cselect_\w+|"
    r"(?:add|addc|sub|subb|addk|mulk|mul|mul_hi|absdiff|abs|min|max)_\w+|"
    r"(?:and|or|xor|nand|nor|xnor|andn2|orn2|not)(?:_saveexec)?_\w+|andn2_saveexec_b64|orn2_saveexec_b64|"
    r"(?:lshl|lshr|ashr|lshl[1-4]_add)_\w+|bfe_\w+|bfm_\w+|sext_\w+|pack_\w+|"
    r"bcnt[01]_\w+|ff[01]_\w+|flbit_\w+|brev_\w+|bitcmp[01]_\w+|bitset[01]_\w+|bitreplicate_\w+|"
    r"wqm_\w+|quadmask_\w+|cmp_\w+|cmpk_\w+|getreg_b32|setreg_\w+|sendmsg\w*|"
    r"set_gpr_idx_\w+|inst_prefetch|icache_inv"
    r")$")


def default_so() -> str | None:
    hits = sorted(glob.glob(os.path.join(ROOT, "ollama_operator_amd", "_C*.so")))
    return hits[0] if hits else None


def code_objects(so_path: str, arch: str = "gfx950") -> list[bytes]:
    """Every `arch` code object of every offload bundle in the shared object's `.hip_fatbin`."""
    with tempfile.TemporaryDirectory() as d:
        fat = os.path.join(d, "fat.bin")
        subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fat}", so_path, os.path.join(d, "x")],
                       check=True, capture_output=True)
        data = open(fat, "rb").read()
    out, i = [], 0
    while (i := data.find(BUNDLE_MAGIC, i)) >= 0:
        n_entries = struct.unpack_from("<Q", data, i + len(BUNDLE_MAGIC))[0]
        p = i + len(BUNDLE_MAGIC) + 8
        for _ in range(n_entries):
            off, size, tlen = struct.unpack_from("<QQQ", data, p)
            p += 24
            triple = data[p:p + tlen].decode()
            p += tlen
            if triple.endswith(arch) and size:
                out.append(data[i + off:i + off + size])
        i += len(BUNDLE_MAGIC)
    return out


def _tool(tool: str, args: list[str], co: bytes) -> str:
    with tempfile.NamedTemporaryFile(suffix=".co") as f:
        f.write(co)
        f.flush()
        return subprocess.run([f"{LLVM}/{tool}", *args, f.name], check=True, capture_output=True, text=True).stdout


def scalar_opcodes(co: bytes) -> dict[str, int]:
    counts: dict[str, int] = {}
    for m in re.finditer(r"^\s+(s_[a-z0-9_]+)", _tool("llvm-objdump", ["-d", "--mcpu=gfx950"], co), re.M):
        counts[m.group(1)] = counts.get(m.group(1), 0) + 1
    return counts


def scratch_bytes(co: bytes) -> dict[str, int]:
    """kernel symbol -> private_segment_fixed_size from the AMDGPU metadata note."""
    notes = _tool("llvm-readelf", ["--notes"], co)
    out: dict[str, int] = {}
    name = None
    for line in notes.splitlines():
        m = re.match(r"\s+\.name:\s+(\S+)", line)
        if m:
            name = m.group(1)
            continue
        m = re.match(r"\s+\.private_segment_fixed_size:\s+(\d+)", line)
        if m and name:
            out[name] = int(m.group(1))
    return out


def audit(so_path: str) -> tuple[list[str], dict[str, int]]:
    """(disallowed scalar opcodes, kernel -> scratch bytes) over all gfx950 code objects."""
    bad: set[str] = set()
    scratch: dict[str, int] = {}
    for co in code_objects(so_path):
        bad |= {op for op in scalar_opcodes(co) if not ALLOWED_SCALAR.match(op)}
        scratch.update(scratch_bytes(co))
    return sorted(bad), scratch


def main(argv: list[str]) -> int:
    so = argv[0] if argv else default_so()
    if not so:
        print("isa_check: no built extension (run build_native.py)")
        return 1
    bad, scratch = audit(so)
    spill = {k: v for k, v in scratch.items() if v}
    for op in bad:
        print(f"disallowed scalar opcode: {op}")
    for k, v in sorted(spill.items()):
        print(f"scratch {v:5d} B/lane  {k}")
    print(f"isa_check: {len(scratch)} kernels, {len(bad)} disallowed scalar opcode(s), {len(spill)} kernel(s) using scratch")
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
