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
    # roofline-kernel traffic table for bench.py: HBM bytes per launch of every bench line's kernel,
    # with the launch's read count so bench.py scales it to its own launch (bytes per read x reads)
    traffic = {}
    method = ("rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE separate passes; FETCH_SIZE x2 (gfx950 wide-read "
              "correction), x1024 (KB)")

    def put(name, e, reads, note=None):
        # several bench launches share a kernel template (one-off parity re-runs at other read
        # lengths): the roofline launch of each line is the one the timed loop repeats (most calls)
        if name in traffic and traffic[name]["calls"] >= e.get("calls", 0):
            return
        traffic[name] = {"kernel": e["kernel"], "grid": e["grid"], "calls": e.get("calls", 0), "hbm_bytes_per_launch": e["hbm_bytes_per_launch"],
                         "reads": reads, "hbm_bytes_per_read": e["hbm_bytes_per_launch"] / reads,
                         "fetch_kb_raw": e.get("fetch_kb_raw"), "write_kb_raw": e.get("write_kb_raw"),
                         "avg_ms_rocprof": e["avg_ms"], "source": os.path.relpath(dst, REPO), "method": method}
        if note:
            traffic[name]["note"] = note

    for e in summ.get("c2", []):
        if e["kernel"].startswith("void k_encode_g16<false, true, 1") and "hbm_bytes_per_launch" in e:
            put("encode32", e, READS)
    big = lambda e: e["grid"] >= 1_000_000   # noqa: E731  (the bench's launches, not the 1-read reference encode)
    for e in summ.get("all", []):
        k = e["kernel"]
        if "hbm_bytes_per_launch" not in e or not big(e):
            continue
        if k.startswith("void k_encode_ham_dense"):
            put("encode_hamming96", e, READS)
        elif k.startswith("void k_ham_dense3"):
            put("hamming_ref_96", e, READS)
        elif k.startswith("void k_ham_dense<"):
            # C3' 32 nt: 100M pairs, 2048 per 256-thread block; 512 nt: 50M pairs, 128 per block
            if e["grid"] < 50_000_000:
                put("hamming_ref_32", e, READS)
            else:
                put("hamming_ref_512", e, READS // 2)
        elif k.startswith("void k_decode_g16"):
            put("decode512", e, READS // 2)
        elif k.startswith("void k_encode_g16<false, true, 2"):
            put("encode512", e, READS // 2)
        elif k.startswith("k_encode_var_dense") or "k_encode_var_dense" in k:
            put("encode_var_ragged", e, 50_000_000)   # F2: 50M ragged 50-150-nt reads
    # F1: the one-pass FASTQ index (k_fq_nlpos + k_fq_place per call; 8 Mi records of the bench's
    # synthetic 100-nt file)
    fq = []
    for kname in ("k_fq_nlpos", "k_fq_place"):      # the bench's launch: the one repeated most
        cand = [e for e in summ.get("all", []) if "hbm_bytes_per_launch" in e and e["kernel"].startswith(kname)]
        if cand:
            fq.append(max(cand, key=lambda e: e.get("calls", 0)))
    if len(fq) == 2:
        nrec = 8 << 20
        tot = sum(e["hbm_bytes_per_launch"] for e in fq)
        traffic["fastq_index_onepass"] = {"kernel": "k_fq_nlpos + k_fq_place", "grid": None, "calls": None,
                                          "hbm_bytes_per_launch": tot, "reads": nrec,
                                          "hbm_bytes_per_read": tot / nrec,
                                          "avg_ms_rocprof": sum(e["avg_ms"] for e in fq),
                                          "source": os.path.relpath(dst, REPO), "method": method}
    if traffic:
        path = os.path.join(REPO, "profiles", "pmc_traffic.json")
        old = json.load(open(path)) if os.path.exists(path) else {}
        keep = {k: v for k, v in old.items() if k.startswith("counter32")}   # from tools/pmc_c5_summary.py
        with open(path, "w") as f:
            json.dump({**traffic, **keep}, f, indent=1)
    print("saved", dst, sorted(traffic))


if __name__ == "__main__":
    main()
