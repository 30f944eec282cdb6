"""Disassemble the gfx950 kernels of the built extension whose (mangled) name matches a regex.

    python scripts/disasm.py REGEX [--so path] [--stats]   (--stats: opcode histogram per kernel)
"""
from __future__ import annotations

import argparse
import collections
import os
import re
import subprocess
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import isa_check  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("pattern")
    ap.add_argument("--so", default=isa_check.default_so())
    ap.add_argument("--stats", action="store_true")
    a = ap.parse_args()
    rx = re.compile(a.pattern)
    for co in isa_check.code_objects(a.so):
        with tempfile.NamedTemporaryFile(suffix=".co") as f:
            f.write(co)
            f.flush()
            txt = subprocess.run([f"{isa_check.LLVM}/llvm-objdump", "-d", "--mcpu=gfx950", f.name],
                                 capture_output=True, text=True).stdout
        cur, body = None, []
        blocks = []
        for line in txt.splitlines():
            m = re.match(r"^[0-9a-f]+ <(.+)>:$", line)
            if m:
                if cur:
                    blocks.append((cur, body))
                cur, body = m.group(1), []
            elif cur:
                body.append(line)
        if cur:
            blocks.append((cur, body))
        for name, body in blocks:
            if not rx.search(name):
                continue
            print(f"==== {name} ({len(body)} lines)")
            if a.stats:
                c = collections.Counter()
                for l in body:
                    t = l.strip().split()
                    if t and not t[0].startswith("//"):
                        c[t[0]] += 1
                for op, n in c.most_common(40):
                    print(f"  {n:6d} {op}")
            else:
                print("\n".join(body))


if __name__ == "__main__":
    main()
