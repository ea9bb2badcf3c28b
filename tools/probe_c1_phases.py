import os, sys, time
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO); sys.path.insert(0, os.path.join(REPO, "oracle"))
import numpy as np, torch
import oracle, shortseq_amd as sq
from shortseq_amd import ingest, batch as B
n, L = 1_000_000, 32
a = oracle.gen_reads(11, 0, n, L)
reads = [a[i * L:(i + 1) * L].tobytes() for i in range(n)]
dev = torch.device("cuda", 0)
sq.ShortSeqCounter(reads[:100_000]); sq.ShortSeqCounter(reads)
torch.cuda.synchronize()
for rep in range(4):
    T = [time.perf_counter()]
    torch.cuda.synchronize(); T.append(time.perf_counter())
    lens_np = np.full(n, L, dtype=np.int64); T.append(time.perf_counter())
    host = ingest._staging(n * L); hv = host.numpy(); hv[:n * L] = a; T.append(time.perf_counter())
    src = ingest._device_staging(n * L, dev)[:n * L]; T.append(time.perf_counter())
    src.copy_(host[:n * L], non_blocking=True); T.append(time.perf_counter())
    torch.cuda.current_stream(dev).synchronize(); T.append(time.perf_counter())
    gc = ingest.LengthGroupCounter(dev)
    t = gc._table(L, n); T.append(time.perf_counter())
    gc._insert(t, L, (0, n), n, src, L, lambda r: r, None, 0); T.append(time.perf_counter())
    res = gc.finish_ordered(); T.append(time.perf_counter())
    names = ["presync", "lens", "stage", "devbuf", "copy_", "sync", "table", "insert+sync", "finish_ordered"]
    print("  ".join(f"{nm} {1e3*(T[i+1]-T[i]):.1f}" for i, nm in enumerate(names)), flush=True)
for rep in range(3):
    t0 = time.perf_counter(); c = sq.ShortSeqCounter(reads); t1 = time.perf_counter(); c = None
    print(f"full {1e3*(t1-t0):.1f} ms", flush=True)
