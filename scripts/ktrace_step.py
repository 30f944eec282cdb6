"""Per-decode-step breakdown from a rocprofv3 kernel_trace.csv: kernel busy time vs idle gaps between
consecutive kernels, per kernel kind. Decode steps are delimited by the sampler kernel.
Usage: python scripts/ktrace_step.py gpurun_out/prof/bench_kernel_trace.csv"""
import collections
import csv
import re
import sys


def short(name: str) -> str:
    m = re.match(r"void omx::(\w+)<([^>]*)>", name)
    if m:
        return f"{m.group(1)}<{m.group(2)}>"
    m = re.match(r"omx::(\w+)", name)
    return m.group(1) if m else name[:40]


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if re.search(r"sample(_fast)?_kernel", r["Kernel_Name"])]
    # steady-state decode steps: between consecutive sampler launches, skip the first few
    steps = list(zip(idx[4:-1], idx[5:]))
    # drop steps that contain a prefill (bench runs a ttft probe after the decode loop)
    spans = sorted(int(rows[b]["Start_Timestamp"]) - int(rows[a]["Start_Timestamp"]) for a, b in steps)
    med = spans[len(spans) // 2] if spans else 0
    steps = [(a, b) for a, b in steps
             if int(rows[b]["Start_Timestamp"]) - int(rows[a]["Start_Timestamp"]) <= 1.5 * med][-16:]
    busy = collections.Counter()
    calls = collections.Counter()
    gap_after = collections.Counter()
    tot_span = tot_busy = 0
    for a, b in steps:
        span = int(rows[b]["Start_Timestamp"]) - int(rows[a]["Start_Timestamp"])
        tot_span += span
        for i in range(a, b):
            r = rows[i]
            d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
            k = short(r["Kernel_Name"])
            busy[k] += d
            calls[k] += 1
            tot_busy += d
            gap_after[k] += int(rows[i + 1]["Start_Timestamp"]) - int(r["End_Timestamp"])
    n = len(steps)
    print(f"{n} decode steps: {tot_span / n / 1e3:.1f} us/step, kernel busy {tot_busy / n / 1e3:.1f} us, "
          f"idle gaps {(tot_span - tot_busy) / n / 1e3:.1f} us")
    print(f"{'kernel':44s} {'calls':>6s} {'us/step':>9s} {'avg us':>8s} {'gap after us':>12s}")
    for k, v in busy.most_common():
        print(f"{k[:44]:44s} {calls[k] / n:6.1f} {v / n / 1e3:9.1f} {v / calls[k] / 1e3:8.2f} "
              f"{gap_after[k] / calls[k] / 1e3:12.2f}")


if __name__ == "__main__":
    main()
