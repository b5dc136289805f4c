#!/usr/bin/env python3
"""Fill-kernel timing sweep (GPU): isolates per-step cost (one strip, long text) and the strip
hand-off lag (many strips, short text) for each strip height R. Times with HIP events on the stream
the engine launches on."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sequence-alignment-gpu_amd", "python"))


def time_fill(b, reps=5):
    import torch
    s = torch.cuda.current_stream()
    b.fill()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        b.fill()
        e1.record(s)
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    return min(ts)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cases", default="")
    ap.add_argument("--rs", default="1,2,4,8")
    ap.add_argument("--mode", type=int, default=0)
    args = ap.parse_args()
    from sa_amd import synthetic
    from sa_amd.batch import DeviceBatch
    S = synthetic.blast_matrix()
    cases = [tuple(int(x) for x in c.split("x")) for c in args.cases.split(",")] if args.cases else \
        [(32768, 0), (256, 32768), (32768, 32768)]
    out = []
    for R in [int(r) for r in args.rs.split(",")]:
        for n, m in cases:
            if m == 0:
                m = 64 * R  # exactly one strip
            t = synthetic.random_sequence(6, n, 4)
            p = synthetic.random_sequence(7, m, 4)
            b = DeviceBatch(args.mode, S, 5, [t], [p], rows_per_lane=R)
            ms = time_fill(b)
            info = b.plan.info()
            steps = n + 63
            rec = {"R": R, "n": n, "m": m, "strips": info["num_strips"], "ms": round(ms, 4),
                   "gcups": round(n * m / ms / 1e6, 2), "ns_per_step_1strip": round(ms * 1e6 / steps, 2)}
            out.append(rec)
            print(json.dumps(rec), flush=True)
            b.close()


if __name__ == "__main__":
    main()
