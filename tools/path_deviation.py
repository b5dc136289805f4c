#!/usr/bin/env python3
"""Traceback path deviation (GPU box, development): aligns synthetic DNA pairs and reports how far the
path strays from the line the table traceback centres its windows on (global: through (m, n) and
(0, 0); local: slope 1 through the best cell) at the strip boundaries -- the window half-width
kTbK / 2 must cover it for the table path to resolve (sa_walk.h)."""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sequence-alignment-gpu_amd", "python"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="32768,120000,250000")
    ap.add_argument("--mode", type=int, default=0)
    ap.add_argument("--related", action="store_true")
    args = ap.parse_args()
    from sa_amd import engine, synthetic
    S = synthetic.blast_matrix()
    for N in (int(x) for x in args.sizes.split(",")):
        t = synthetic.random_sequence(6, N, 4)
        p = synthetic.mutate(t, 7, 4, N) if args.related else synthetic.random_sequence(7, N, 4)
        r = engine.align_pair(args.mode, t, p, S, 5)
        at = np.frombuffer(r["aligned_text"].encode(), np.uint8)
        apn = np.frombuffer(r["aligned_pattern"].encode(), np.uint8)
        gap = ord("-")
        # forward walk from the start indices: row i / column j after each op
        i = np.cumsum(apn != gap) + int(r["start_pattern"]) if r["num_bytes"] else np.zeros(1, int)
        j = np.cumsum(at != gap) + int(r["start_text"]) if r["num_bytes"] else np.zeros(1, int)
        if args.mode == 0:
            i, j = np.cumsum(apn != gap), np.cumsum(at != gap)
            dev = j - i * N / N
        else:
            i0, j0 = i[-1], j[-1]
            dev = j - (j0 - (i0 - i))
        sel = (i % 64) == 0
        d = np.abs(dev[sel]) if sel.any() else np.abs(dev)
        print(json.dumps({"n": N, "mode": args.mode, "related": args.related, "ops": int(r["num_bytes"]),
                          "max_dev_at_strip_rows": float(d.max()), "p99": float(np.percentile(d, 99))}), flush=True)


if __name__ == "__main__":
    main()
