"""Scratch / wait / branch census of the innermost loops of one kernel in a hipcc --save-temps .s file:
  python scripts/loopscan.py file.s <kernel-name-substring>"""
import re
import sys

s = open(sys.argv[1]).read()
for m in re.finditer(r"^(_Z\w+):", s, re.M):
    if sys.argv[2] not in m.group(1):
        continue
    body = s[m.end():s.find(".Lfunc_end", m.end())].split("\n")
    labels = {l.split(":")[0]: i for i, l in enumerate(body) if re.match(r"^\.LBB\w+:", l)}
    print(m.group(1)[:100])
    for i, l in enumerate(body):
        mm = re.search(r"s_cbranch_\w+\s+(\.LBB\w+)", l)
        if mm and mm.group(1) in labels and labels[mm.group(1)] < i:  # back edge
            a, b = labels[mm.group(1)], i
            seg = body[a:b + 1]
            pats = {"mfma": r"v_mfma", "scratch": r"scratch_", "vmcnt0": r"s_waitcnt vmcnt\(0\)",
                    "branches": r"s_cbranch", "valu": r"^\s+v_(?!mfma)", "ds_read": r"ds_read",
                    "ds_write": r"ds_write", "gload": r"global_load"}
            res = " ".join(f"{k}={sum(1 for x in seg if re.search(p, x))}" for k, p in pats.items())
            print(f"  loop {mm.group(1)} lines {a}-{b}: {res}")
