"""Average PMC counters per dispatch of kernels matching a name filter.
usage: python scripts/pmc_summary.py gpurun_out/pmc_gemm qgemm"""
import collections
import csv
import glob
import sys

d, pat = sys.argv[1], sys.argv[2]
agg = collections.defaultdict(list)
for f in sorted(glob.glob(f"{d}/p*_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        if pat in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in sorted(agg.items()):
    print(f"{k:32s} dispatches={len(v):4d} mean={sum(v) / len(v):16.1f}")
