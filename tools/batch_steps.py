#!/usr/bin/env python3
"""Per-step wall time of the batch workload (development): fill, traceback and results of 4096
2048^2 pairs, each step synchronised, to see whether step times drift."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sequence-alignment-gpu_amd", "python"))
import torch  # noqa: E402
from sa_amd import synthetic  # noqa: E402
from sa_amd.batch import DeviceBatch  # noqa: E402

L, npairs = 2048, 4096
texts = [synthetic.random_sequence(1000 + 2 * i, L, 4) for i in range(npairs)]
pats = [synthetic.random_sequence(1001 + 2 * i, L, 4) for i in range(npairs)]
job = DeviceBatch(0, synthetic.blast_matrix(), 5, texts, pats)
for k in range(int(sys.argv[1]) if len(sys.argv) > 1 else 20):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    job.fill()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    job.traceback()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    r = job.results()
    t3 = time.perf_counter()
    print(f"step {k}: fill {1e3 * (t1 - t0):.2f} ms  traceback {1e3 * (t2 - t1):.2f} ms  results {1e3 * (t3 - t2):.2f} ms", flush=True)
