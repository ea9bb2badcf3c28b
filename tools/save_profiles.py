#!/usr/bin/env python3
"""Copy the rocprofv3 summaries of one GPU run into profiles/<round>/<tag>/ (tracked) and refresh
profiles/pmc_traffic.json (HBM bytes per launch of the bench's roofline kernels), which bench.py
reads for roofline.traffic.

usage: save_profiles.py <gpurun_out/prof_TAG> <round> [bench.log]
"""
import json
import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
READS = 100_000_000   # the profiled command is the default bench (C2: 100M x 32 nt per launch)
REPO = os.path.dirname(HERE)


def main():
    src, rnd = sys.argv[1], sys.argv[2]
    tag = os.path.basename(src.rstrip("/")).replace("prof_", "")
    dst = os.path.join(REPO, "profiles", rnd, tag)
    os.makedirs(dst, exist_ok=True)
    for sub in ("trace", "all/trace"):
        for f in ("run_kernel_stats.csv", "run_domain_stats.csv"):
            p = os.path.join(src, sub, f)
            if os.path.exists(p):
                shutil.copy(p, os.path.join(dst, sub.replace("/", "_") + "_" + f))
    summ = {}
    for sub, name in (("", "c2"), ("all", "all")):
        d = os.path.join(src, sub) if sub else src
        if not os.path.isdir(os.path.join(d, "trace")):
            continue
        out = os.path.join(dst, f"summary_{name}.json")
        txt = subprocess.run([sys.executable, os.path.join(HERE, "prof_summary.py"), d, "--json", out],
                             capture_output=True, text=True, check=True).stdout
        with open(os.path.join(dst, f"summary_{name}.txt"), "w") as f:
            f.write(txt)
        with open(out) as f:
            summ[name] = json.load(f)
    if len(sys.argv) > 3 and os.path.exists(sys.argv[3]):
        shutil.copy(sys.argv[3], os.path.join(dst, "bench.log"))
    # roofline-kernel traffic table for bench.py
    traffic = {}
    for e in summ.get("c2", []):
        if e["kernel"].startswith("void k_encode_g16<false, true, 1") and "hbm_bytes_per_launch" in e:
            traffic["encode32"] = {"kernel": e["kernel"], "hbm_bytes_per_launch": e["hbm_bytes_per_launch"],
                                   "reads": READS, "hbm_bytes_per_read": e["hbm_bytes_per_launch"] / READS,
                                   "fetch_kb_raw": e.get("fetch_kb_raw"), "write_kb_raw": e.get("write_kb_raw"),
                                   "avg_ms_rocprof": e["avg_ms"], "source": os.path.relpath(dst, REPO),
                                   "method": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE separate passes; "
                                             "FETCH_SIZE x2 (gfx950 wide-read correction), x1024 (KB)"}
    for e in summ.get("all", []):
        k = e["kernel"]
        if "hbm_bytes_per_launch" not in e:
            continue
        if k.startswith("void k_encode_ham_dense"):
            traffic["encode_hamming96"] = {"kernel": k, "hbm_bytes_per_launch": e["hbm_bytes_per_launch"],
                                           "avg_ms_rocprof": e["avg_ms"]}
        elif k.startswith("void k_decode_g16") and e["grid"] >= 400000000:
            traffic["decode512"] = {"kernel": k, "hbm_bytes_per_launch": e["hbm_bytes_per_launch"],
                                    "avg_ms_rocprof": e["avg_ms"]}
        elif k.startswith("void k_encode_g16<false, true, 2") and e["grid"] >= 400000000:
            traffic["encode512"] = {"kernel": k, "hbm_bytes_per_launch": e["hbm_bytes_per_launch"],
                                    "avg_ms_rocprof": e["avg_ms"]}
        elif k.startswith("void k_count_g16"):
            traffic["counter32_insert"] = {"kernel": k, "hbm_bytes_per_launch": e["hbm_bytes_per_launch"],
                                           "avg_ms_rocprof": e["avg_ms"],
                                           "note": "random 32-B slot traffic; the x2 FETCH correction is calibrated "
                                                   "for wide streaming reads only"}
    if traffic:
        with open(os.path.join(REPO, "profiles", "pmc_traffic.json"), "w") as f:
            json.dump(traffic, f, indent=1)
    print("saved", dst, sorted(traffic))


if __name__ == "__main__":
    main()
