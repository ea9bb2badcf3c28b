#!/usr/bin/env python3
"""Print the kernel timeline of the last rep of a rocprofv3 kernel trace (gaps between kernels),
starting at the last launch of a marker kernel.

    python3 tools/timeline.py <run_kernel_trace.csv> [marker=k_len_count] [min_gap_us=0]
"""
import csv
import sys


def main():
    path = sys.argv[1]
    mark = sys.argv[2] if len(sys.argv) > 2 else "k_len_count"
    min_gap = float(sys.argv[3]) if len(sys.argv) > 3 else 0.0
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    st = max(i for i, r in enumerate(rows) if mark in r["Kernel_Name"])
    t0 = prev = int(rows[st]["Start_Timestamp"])
    busy = 0
    for r in rows[st:]:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        busy += e - s
        gap = (s - prev) / 1e3
        n = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "")[:60]
        if gap >= min_gap or (e - s) / 1e3 >= 20:
            print(f"{(s - t0) / 1e3:9.1f}  gap {gap:7.1f}  dur {(e - s) / 1e3:8.1f}  {n}")
        prev = e
    print(f"span {(prev - t0) / 1e3:.1f} us, kernels busy {busy / 1e3:.1f} us")


if __name__ == "__main__":
    main()
