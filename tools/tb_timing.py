#!/usr/bin/env python3
"""Traceback phase timing (GPU, debug): runs fill + traceback of one pair with SA_TB_TIMING and prints
the time of the walk, the op-counting pass and the letter pass (s_memrealtime, 100 MHz)."""
import argparse
import os
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sequence-alignment-gpu_amd", "python"))
ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=32768)
ap.add_argument("--m", type=int, default=32768)
ap.add_argument("--mode", type=int, default=0)
args = ap.parse_args()
from sa_amd import synthetic
from sa_amd.batch import DeviceBatch

S = synthetic.blast_matrix()
b = DeviceBatch(args.mode, S, 5, [synthetic.random_sequence(6, args.n, 4)], [synthetic.random_sequence(7, args.m, 4)])
b.fill()
b.traceback()
path = os.path.join(tempfile.mkdtemp(), "tm.bin")
os.environ["SA_TB_TIMING"] = path
b.traceback()
del os.environ["SA_TB_TIMING"]
r = b.results()[0]
tm = np.fromfile(path, dtype=np.uint64).reshape(-1, 4).astype(np.int64)
d = np.diff(tm[0]) * 0.01
print({"n": args.n, "m": args.m, "mode": args.mode, "ops": r["num_bytes"], "walk_us": round(d[0], 1),
       "count_pass_us": round(d[1], 1), "letter_pass_us": round(d[2], 1),
       "walk_ns_per_op": round(d[0] * 1000 / max(1, r["num_bytes"]), 1)})
b.close()
