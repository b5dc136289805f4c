#!/usr/bin/env python3
"""Traceback walk timing (GPU, debug): runs fill + traceback of one pair with SA_TB_TIMING and prints
the walk's duration from its in-kernel timestamps (s_memrealtime, 100 MHz; sa_walk.hip writes the
start / end pair of each pair's walk). The expansion kernel's time comes from rocprofv3."""
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
# the engine reads its knobs once per process: set before the first call
path = os.path.join(tempfile.mkdtemp(), "tm.bin")
os.environ["SA_TB_TIMING"] = path
from sa_amd import synthetic
from sa_amd.batch import DeviceBatch

S = synthetic.blast_matrix()
b = DeviceBatch(args.mode, S, 5, [synthetic.random_sequence(6, args.n, 4)], [synthetic.random_sequence(7, args.m, 4)])
b.fill()
b.traceback()
b.traceback()  # the file holds the last call's timestamps
r = b.results()[0]
tm = np.fromfile(path, dtype=np.uint64).astype(np.int64)
walk_us = (tm[1] - tm[0]) * 0.01
rec = {"n": args.n, "m": args.m, "mode": args.mode, "ops": r["num_bytes"], "walk_us": round(walk_us, 1),
       "walk_ns_per_op": round(walk_us * 1000 / max(1, r["num_bytes"]), 2)}
if len(tm) >= 4 and tm[2] > 0:
    # experiment builds with SA_EXP_WALK_TIMING: shader clocks in staging / in the row walk proper
    rec.update({"stage_clk_per_row": round(tm[2] / args.m, 1), "batch_clk_per_row": round(tm[3] / args.m, 1)})
    if len(tm) >= 8 and tm[6] > 0:
        rec.update({"stage_load_clk_per_strip": round(tm[4] / tm[6], 1), "pf_miss": int(tm[5]),
                    "strips": int(tm[6]), "restages": int(tm[7])})
    if len(tm) >= 9:
        rec["stager_hits"] = int(tm[8])  # strips whose windows came from the stager wave
print(rec)
b.close()
