"""Per-decode-step launch counts of a TP rank from a rocprofv3 kernel trace: how many all-reduce
(ar_add_kernel; ar_add_emit_kernel on the int8 chain) and all-gather (ar_gather_kernel) launches one
token costs, per layer half, and how many GEMVs ran on the int8 chain (qgemv8) vs the fp32 prologue.
Usage: python scripts/tp_trace_count.py <kernel_trace.csv> <n_layer>"""
import collections
import csv
import re
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    n_layer = int(sys.argv[2])
    by_pid = collections.defaultdict(list)
    for r in rows:
        by_pid[r.get("Process_Id") or r.get("Agent_Id") or r.get("Queue_Id")].append(r)
    for pid, rs in by_pid.items():
        rs.sort(key=lambda r: int(r["Start_Timestamp"]))
        idx = [i for i, r in enumerate(rs) if re.search(r"sample(_fast)?_kernel", r["Kernel_Name"])]
        steps = list(zip(idx[4:-1], idx[5:]))[-8:]
        if not steps:
            continue
        cnt = collections.Counter()
        dur = collections.Counter()
        for a, b in steps:
            for r in rs[a + 1:b + 1]:
                n = r["Kernel_Name"]
                key = ("ar_add_emit" if "ar_add_emit_kernel" in n else "ar_add" if "ar_add_kernel" in n else
                       "ar_gather" if "ar_gather_kernel" in n else "qgemv8" if "qgemv8" in n else
                       "qgemv_flight" if "qgemv_flight" in n else "other")
                cnt[key] += 1
                dur[key] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        k = len(steps)
        print(f"process {pid}: {k} decode steps; per step: ar_add {cnt['ar_add'] / k:.1f} launches, "
              f"ar_add_emit {cnt['ar_add_emit'] / k:.1f} "
              f"({cnt['ar_add_emit'] / k / (2 * n_layer):.2f} per layer half, "
              f"{dur['ar_add_emit'] / max(cnt['ar_add_emit'], 1):.2f} us each), "
              f"ar_gather {cnt['ar_gather'] / k:.1f}, qgemv8 {cnt['qgemv8'] / k:.1f}, "
              f"qgemv_flight {cnt['qgemv_flight'] / k:.1f}, other kernels {cnt['other'] / k:.1f}")


if __name__ == "__main__":
    main()
