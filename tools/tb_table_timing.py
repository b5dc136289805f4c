#!/usr/bin/env python3
"""Per-phase times of tb_table_kernel (debug, GPU box): one DNA pair aligned with SA_TB_TABLE_TIMING
set; prints the mean per-strip time of each phase (staging, walk phases, compactions, output) and
the distinct chains left after each compaction. Times: [mean, p90, max] us. Stamps are s_memrealtime (100 MHz)."""
import argparse
import json
import os
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sequence-alignment-gpu_amd", "python"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=32768)
    ap.add_argument("--m", type=int, default=32768)
    ap.add_argument("--mode", type=int, default=0)
    args = ap.parse_args()
    path = os.path.join(tempfile.mkdtemp(), "tbt.bin")
    os.environ["SA_TB_TABLE_TIMING"] = path
    from sa_amd import synthetic
    from sa_amd.batch import DeviceBatch
    S = synthetic.blast_matrix()
    t = synthetic.random_sequence(6, args.n, 4)
    p = synthetic.random_sequence(7, args.m, 4) if args.mode == 0 else synthetic.mutate(t, 7, 4, args.m)
    b = DeviceBatch(args.mode, S, 5, [t], [p], rows_per_lane=1)
    for _ in range(3):
        b.fill()
        b.traceback()
    import torch
    torch.cuda.synchronize()
    v = np.fromfile(path, dtype=np.uint64).reshape(-1, 12).astype(np.int64)
    v = v[v[:, 10] > 0]
    ent, stg, e0, c0, d0, e1, c1, d1, e2, end = (v[:, i] for i in (11, 0, 1, 2, 3, 4, 5, 6, 7, 10))
    us = lambda x: [round(float(np.mean(x)) * 0.01, 2), round(float(np.percentile(x, 90)) * 0.01, 2), round(float(np.max(x)) * 0.01, 2)]
    print(json.dumps({"strips": len(v), "kernel_span_us": round((end.max() - ent.min()) * 0.01, 2),
                      "entry_spread_us": round((ent.max() - ent.min()) * 0.01, 2),
                      "staging_us": us(stg - ent), "phase0_us": us(e0 - stg), "compact0_us": us(c0 - e0),
                      "phase1_us": us(e1 - c0), "compact1_us": us(c1 - e1), "phase2_us": us(e2 - c1),
                      "output_us": us(end - e2), "chains_after_c0": float(np.mean(d0)),
                      "chains_after_c1": float(np.mean(d1)),
                      "slowest_phase0_strips": [[int(x), round(float(e0[x] - stg[x]) * 0.01, 1), round(float(stg[x] - ent.min()) * 0.01, 1)]
                                                for x in np.argsort(stg - e0)[:4]],
                      "entry_us_every64": [round(float(x - ent.min()) * 0.01, 1) for x in ent[::64]]}))
    b.close()


if __name__ == "__main__":
    main()
