#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc passes (scripts/pmc_f2.sh layout: <dir>/p<i>/**/run_counter_collection.csv):
per kernel name, the mean of each counter over its dispatches.

    python tools/pmc_table.py gpurun_out/pmc_<tag> [kernel-regex]
"""
import collections
import csv
import glob
import re
import sys


def main():
    d = sys.argv[1]
    pat = re.compile(sys.argv[2] if len(sys.argv) > 2 else ".")
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        per = collections.defaultdict(float)
        names = {}
        for r in csv.DictReader(open(f)):
            key = (r["Dispatch_Id"], r["Counter_Name"])
            per[key] += float(r["Counter_Value"])
            names[r["Dispatch_Id"]] = r["Kernel_Name"]
        for (disp, ctr), v in per.items():
            vals[names[disp]][ctr].append(v)
    for k in sorted(vals):
        if not pat.search(k):
            continue
        print(k[:110])
        for ctr in sorted(vals[k]):
            xs = vals[k][ctr]
            print(f"    {ctr:28s} {sum(xs) / len(xs):16.4g}  (n={len(xs)})")


if __name__ == "__main__":
    main()
