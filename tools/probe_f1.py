#!/usr/bin/env python3
"""F1 timing alone: ss_fastq_scan + ss_fastq_index over the bench's 1.98-GB synthetic FASTQ."""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402
import shortseq_amd.batch as B  # noqa: E402
from shortseq_amd._native import lib  # noqa: E402

dev = torch.device("cuda", 0)
for _ in range(2):
    print(bench.bench_fastq_index(B, lib(), dev, reps=20), flush=True)
