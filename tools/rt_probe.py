import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
order = sys.argv[1]
if order == "torch_first":
    import torch
    print("torch avail", torch.cuda.is_available())
    import shortseq_amd as sq
elif order == "sq_first":
    import shortseq_amd as sq
    import torch
    print("torch avail", torch.cuda.is_available())
else:
    import shortseq_amd as sq
reads = [b"ACGT" * 8] * 70000
try:
    c = sq.ShortSeqCounter(reads, device="cuda")
    print(order, "ok", len(c))
except Exception as e:
    print(order, "FAIL", e)
libs = sorted({l.split()[-1] for l in open("/proc/self/maps") if ("amdhip" in l or "hsa-runtime" in l)})
print(libs)
