#!/usr/bin/env python3
"""The C5 exchange rehearsal of bench.py alone (pack / merge ms on one GPU)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch, json, bench
import shortseq_amd.batch as B
dev = torch.device("cuda", 0)
r = bench.bench_exchange(B, dev)
print("exchange pack %.3f merge %.3f ms" % (r["pack_ms"], r["merge_ms"]))
