"""Prefill-phase breakdown from a rocprofv3 kernel_trace.csv: kernels before the first sampler launch
(the prompt pass of the first request), grouped by kernel, plus the wall span.
Usage: python scripts/ktrace_prefill.py gpurun_out/prof/bench_kernel_trace.csv"""
import collections
import csv
import sys

from ktrace_step import short

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
first = next(i for i, r in enumerate(rows) if "sample_kernel" in r["Kernel_Name"])
# the prompt pass: from the embedding gather that precedes the first sampler
start = max(i for i in range(first) if "embed_rows" in rows[i]["Kernel_Name"])
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
