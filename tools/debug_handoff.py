#!/usr/bin/env python3
"""Debug aid (GPU): direction matrix of one pair vs the oracle's, cell by cell; prints the first
wrong cell per strip (strip = 64*R rows). The oracle is used only as the checker."""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sequence-alignment-gpu_amd", "python"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=3903)
ap.add_argument("--m", type=int, default=1428)
ap.add_argument("--mode", type=int, default=0)
ap.add_argument("--R", type=int, default=1)
args = ap.parse_args()
import oracle
from sa_amd import synthetic
from sa_amd.batch import DeviceBatch

S = synthetic.blast_matrix()
t = synthetic.random_sequence(11, args.n, 4)
p = synthetic.random_sequence(12, args.m, 4)
b = DeviceBatch(args.mode, S, 5, [t], [p], rows_per_lane=args.R)
b.fill()
M = b.directions(0).reshape(args.m + 1, args.n + 1)
E = np.empty((args.m + 1) * (args.n + 1), np.uint8)
oracle.fill_only(args.mode, t, p, S, 5, E)
E = E.reshape(args.m + 1, args.n + 1)
bad = np.argwhere(M != E)
print("W", os.environ.get("SA_WAVES_PER_GROUP"), "wrong cells", len(bad), "of", M.size)
RB = 64 * args.R
seen = set()
for i, j in bad:
    st = (i - 1) // RB
    if st in seen:
        continue
    seen.add(st)
    print(f"  strip {st}: first wrong cell i={i} j={j} (row in strip {(i - 1) % RB}) got {M[i, j]} want {E[i, j]}")
    if len(seen) > 6:
        break
