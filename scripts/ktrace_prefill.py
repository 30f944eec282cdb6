"""Prefill-phase breakdown from a rocprofv3 kernel_trace.csv: kernels before the first sampler launch
(the prompt pass of the first request), grouped by kernel, plus the wall span.
Usage: python scripts/ktrace_prefill.py gpurun_out/prof/bench_kernel_trace.csv"""
import collections
import csv
import re
import sys

from ktrace_step import short

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
samp = [i for i, r in enumerate(rows) if re.search(r"sample(_fast)?_kernel", r["Kernel_Name"])]
# the prompt pass: the longest span from an embedding gather to the next sampler launch (warm-up
# graph captures and decode steps are short; the timed prompt is the long one)
best = None
for a, b in zip([-1] + samp[:-1], samp):
    emb = [i for i in range(a + 1, b) if "embed_rows" in rows[i]["Kernel_Name"]]
    if not emb:
        continue
    st = emb[0]
    dur = int(rows[b]["End_Timestamp"]) - int(rows[st]["Start_Timestamp"])
    if best is None or dur > best[0]:
        best = (dur, st, b)
_, start, first = best
seg = rows[start:first + 1]
span = int(seg[-1]["End_Timestamp"]) - int(seg[0]["Start_Timestamp"])
busy = collections.Counter()
calls = collections.Counter()
for r in seg:
    k = short(r["Kernel_Name"])
    busy[k] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    calls[k] += 1
print(f"prefill span {span / 1e3:.1f} us, kernel busy {sum(busy.values()) / 1e3:.1f} us, {len(seg)} kernels")
for k, v in busy.most_common(20):
    print(f"{k[:50]:50s} calls={calls[k]:5d} total_us={v / 1e3:9.1f} avg_us={v / calls[k] / 1e3:8.2f}")
