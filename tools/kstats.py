#!/usr/bin/env python3
"""Print a rocprofv3 run_kernel_stats.csv compactly: kernel (short name), calls, average us, share."""
import csv
import re
import sys

for path in sys.argv[1:]:
    print(path)
    for r in csv.DictReader(open(path)):
        n = r["Name"].replace("(anonymous namespace)::", "")
        n = re.sub(r"^void ", "", n)
        n = n.split("(")[0]
        print(f"  {n[:70]:70s} calls {r['Calls']:>5s} avg {float(r['AverageNs']) / 1e3:9.1f} us  {float(r['Percentage']):5.1f} %")
