"""Per-call durations of the last decode steps' kernels (rocprofv3 kernel_trace.csv), in launch order:
python scripts/mb_trace.py <kernel_trace.csv> [n_last]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 24
prev = None
for r in rows[-n:]:
    st, en = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    gap = (st - prev) / 1e3 if prev else 0.0
    prev = en
    print(f"{r['Kernel_Name'][:58]:58s} grid={r['Grid_Size_X']:>7} lds={r['LDS_Block_Size']:>6} "
          f"vgpr={r['VGPR_Count']:>4} dur={(en - st) / 1e3:7.2f} gap={gap:5.2f}")
