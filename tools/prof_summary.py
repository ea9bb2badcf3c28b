#!/usr/bin/env python3
"""Summarise rocprofv3 CSV output: per (kernel, grid size) dispatch stats from the kernel trace and
HBM traffic per dispatch from separate --pmc FETCH_SIZE / WRITE_SIZE passes.

FETCH_SIZE / WRITE_SIZE are in KB (x1024).  gfx950 correction (MI355X_MICROARCH.md §HBM): FETCH_SIZE
reports exactly half the bytes of a wide (16 B/lane) coalesced streaming read -> doubled here.
WRITE_SIZE is exact for 16 B/lane stores; narrower stores are uncalibrated (noted in the output).

usage: prof_summary.py <prof_dir> [--json out.json]
  <prof_dir>/trace/*kernel_trace.csv, <prof_dir>/fetch/*counter_collection.csv, <prof_dir>/write/...
"""
import csv
import glob
import json
import os
import statistics
import sys


def short(name):
    n = name.replace("(anonymous namespace)::", "")
    return n.split("(")[0] if "(" in n and "<" not in n.split("(")[0] else n[: n.find(">(") + 1] if ">(" in n else n


def load_trace(d):
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                rows.append((short(r["Kernel_Name"]), int(r.get("Grid_Size") or r["Grid_Size_X"]),
                             int(r["End_Timestamp"]) - int(r["Start_Timestamp"])))
    return rows


def load_pmc(d, counter):
    out = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                if r["Counter_Name"] != counter:
                    continue
                k = (short(r["Kernel_Name"]), int(r.get("Grid_Size") or r["Grid_Size_X"]))
                out.setdefault(k, []).append(float(r["Counter_Value"]))
    return out


def main():
    d = sys.argv[1]
    rows = load_trace(os.path.join(d, "trace"))
    groups = {}
    for k, g, ns in rows:
        groups.setdefault((k, g), []).append(ns)
    fetch = load_pmc(os.path.join(d, "fetch"), "FETCH_SIZE")
    write = load_pmc(os.path.join(d, "write"), "WRITE_SIZE")
    summary = []
    for (k, g), v in sorted(groups.items(), key=lambda x: -sum(x[1])):
        e = {"kernel": k, "grid": g, "calls": len(v), "avg_ms": statistics.mean(v) / 1e6,
             "min_ms": min(v) / 1e6, "max_ms": max(v) / 1e6}
        if (k, g) in fetch:
            e["fetch_kb_raw"] = statistics.mean(fetch[(k, g)])
            e["hbm_read_bytes_corrected"] = 2 * e["fetch_kb_raw"] * 1024
        if (k, g) in write:
            e["write_kb_raw"] = statistics.mean(write[(k, g)])
            e["hbm_write_bytes"] = e["write_kb_raw"] * 1024
        if "hbm_read_bytes_corrected" in e and "hbm_write_bytes" in e:
            e["hbm_bytes_per_launch"] = e["hbm_read_bytes_corrected"] + e["hbm_write_bytes"]
        summary.append(e)
    for e in summary[:25]:
        t = f"  traffic {e['hbm_bytes_per_launch'] / 1e9:.3f} GB" if "hbm_bytes_per_launch" in e else ""
        print(f"{e['avg_ms']:9.4f} ms avg  x{e['calls']:<4d} grid {e['grid']:>10d}  {e['kernel'][:90]}{t}")
    if "--json" in sys.argv:
        with open(sys.argv[sys.argv.index("--json") + 1], "w") as f:
            json.dump(summary, f, indent=1)


if __name__ == "__main__":
    main()
