#!/usr/bin/env python3
"""Summarise scripts/pmc_c5.sh (rocprofv3 --pmc passes over tools/c5_only.py) per C5 kernel: HBM read
= FETCH_SIZE KB x 2 (gfx950 wide-read correction) x 1024, write = WRITE_SIZE KB x 1024, and the 8
SQ counters; the median over that kernel's launches.

usage: pmc_c5_summary.py <gpurun_out/pmc_c5> > profiles/r1/pmc_c5_<tag>.txt
"""
import csv
import os
import statistics
import sys
from collections import defaultdict

KERNELS = ["k_pf_coarse", "k_pf_count", "k_pf_scatter", "k_pc_aggregate_slice", "k_spill_insert", "k_pf_order"]


def per_dispatch(path):
    """{kernel: {counter: [value per dispatch]}} for the C5 kernels."""
    acc = defaultdict(float)
    names = {}
    with open(path) as f:
        for r in csv.DictReader(f):
            k = next((k for k in KERNELS if k in r["Kernel_Name"]), None)
            if k is None:
                continue
            key = (r["Dispatch_Id"], r["Counter_Name"])
            acc[key] += float(r["Counter_Value"])
            names[r["Dispatch_Id"]] = (k, r["Kernel_Name"])
    out = defaultdict(lambda: defaultdict(list))
    for (d, c), v in acc.items():
        out[names[d][0]][c].append(v)
    full = {k: n for (k, n) in names.values()}
    return out, full


def main():
    root = sys.argv[1]
    save = "--save-traffic" in sys.argv
    fetch, full = per_dispatch(os.path.join(root, "fetch", "run_counter_collection.csv"))
    write, _ = per_dispatch(os.path.join(root, "write", "run_counter_collection.csv"))
    sq, _ = per_dispatch(os.path.join(root, "sq", "run_counter_collection.csv"))
    p2 = os.path.join(root, "sq2", "run_counter_collection.csv")
    if os.path.exists(p2):
        sq2, _ = per_dispatch(p2)
        for k, v in sq2.items():
            sq.setdefault(k, {}).update(v)
    print("C5 counter kernels (tools/c5_only.py: 125M x 32-nt reads, pool 2^24 uniform, lazy reset), rocprofv3 --pmc,")
    print("separate passes (FETCH_SIZE | WRITE_SIZE | 8 SQ counters | 8 SQ counters), median over launches.")
    print("HBM read = FETCH_SIZE KB x2 (gfx950 wide-read correction) x1024; write = WRITE_SIZE KB x1024.")
    print("Algorithmic per launch: coarse 4.0 GB in / 1.5 GB out; count 1.0 GB in; scatter 1.5 / 1.5 GB;")
    print("aggregate 1.5 GB in + whole 0.5-GB table written (fresh slices, 16-B slots).\n")
    per_kernel = {}
    for k in KERNELS:
        if k not in fetch:
            continue
        rd = statistics.median(fetch[k]["FETCH_SIZE"]) * 2 * 1024 / 1e9
        wr = statistics.median(write[k]["WRITE_SIZE"]) * 1024 / 1e9 if k in write else float("nan")
        name = full[k].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
        print(f"{name}: HBM read {rd:.3f} GB, write {wr:.3f} GB")
        for c in sorted(sq.get(k, {})):
            print(f"   {c:24s} {statistics.median(sq[k][c]):.4g}")
        d = {c: statistics.median(v) for c, v in sq.get(k, {}).items()}
        if d.get("SQ_INSTS_LDS"):
            print(f"   -> LDS bank-conflict cycles per LDS instruction {d.get('SQ_LDS_BANK_CONFLICT', 0) / d['SQ_INSTS_LDS']:.2f}")
        per_kernel[k] = rd + wr
    total = sum(per_kernel.values())
    print(f"per insert: {total:.3f} GB HBM ({total * 1e9 / 125e6:.1f} B per read)")
    if save:
        import json
        path = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles", "pmc_traffic.json")
        t = json.load(open(path)) if os.path.exists(path) else {}
        t["counter32_insert"] = {"kernels": {k: v * 1e9 for k, v in per_kernel.items()},
                                 "hbm_bytes_per_launch": total * 1e9, "reads": 125_000_000,
                                 "hbm_bytes_per_read": total * 1e9 / 125e6, "source": sys.argv[2] if len(sys.argv) > 2 else root,
                                 "method": "scripts/pmc_c5.sh: rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes over "
                                           "tools/c5_only.py (125M x 32 nt, pool 2^24 uniform); FETCH x2 (gfx950), x1024"}
        # the variants' passes (scripts/pmc_c5.sh: var_<name>/fetch, var_<name>/write)
        for d in sorted(os.listdir(root)):
            if not d.startswith("var_") or not os.path.isdir(os.path.join(root, d, "write")):
                continue
            vf, _ = per_dispatch(os.path.join(root, d, "fetch", "run_counter_collection.csv"))
            vw, _ = per_dispatch(os.path.join(root, d, "write", "run_counter_collection.csv"))
            vk = {k: statistics.median(vf[k]["FETCH_SIZE"]) * 2 * 1024 + statistics.median(vw[k]["WRITE_SIZE"]) * 1024
                  for k in KERNELS if k in vf and k in vw}
            vt = sum(vk.values())
            print(f"variant {d[4:]}: {vt / 1e9:.3f} GB HBM per insert ({vt / 125e6:.1f} B per read)")
            t["counter32_insert_" + d[4:]] = {"kernels": vk, "hbm_bytes_per_launch": vt, "reads": 125_000_000,
                                              "hbm_bytes_per_read": vt / 125e6,
                                              "source": sys.argv[2] if len(sys.argv) > 2 else root,
                                              "method": t["counter32_insert"]["method"].replace(
                                                  "pool 2^24 uniform", d[4:])}
        with open(path, "w") as f:
            json.dump(t, f, indent=1)
        print()


if __name__ == "__main__":
    main()
