"""Export the kernel dispatches of a rocprofv3 rocpd database (`*_results.db`, the default output
format of ROCm 7.2) to the kernel_trace.csv columns scripts/ktrace_step.py reads.
Usage: python scripts/rocpd2csv.py k_results.db out_kernel_trace.csv"""
import csv
import sqlite3
import sys


def main():
    c = sqlite3.connect(sys.argv[1])
    rows = c.execute("select name, start, end, grid_x, workgroup_x, vgpr_count, scratch_size from kernels order by start")
    with open(sys.argv[2], "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Kernel_Name", "Start_Timestamp", "End_Timestamp", "Grid_Size", "Workgroup_Size", "VGPR_Count",
                    "Scratch_Size"])
        for r in rows:
            w.writerow(r)


if __name__ == "__main__":
    main()
