#!/usr/bin/env python3
"""Per-strip fill timeline (GPU, debug): runs one fill with SA_TIMELINE set and reports, for a
chain of strips, the hand-off lag (start of strip k's first body minus that of strip k-1), the
per-step time and where the strips ran (XCC / CU). Timestamps are s_memrealtime (100 MHz)."""
import argparse
import json
import os
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sequence-alignment-gpu_amd", "python"))


def max_overlap(xcc, se, cu, simd, fed, end):
    """Largest number of strips whose [fed, end) windows overlap on one SIMD."""
    best = 0
    groups = {}
    for i, k in enumerate(zip(xcc.tolist(), se.tolist(), cu.tolist(), simd.tolist())):
        groups.setdefault(k, []).append(i)
    for idx in groups.values():
        ev = sorted([(int(fed[i]), 1) for i in idx] + [(int(end[i]), -1) for i in idx], key=lambda e: (e[0], e[1]))
        cur = 0
        for _, d in ev:
            cur += d
            best = max(best, cur)
    return best


def summarize(tl, n, W, t0=None):
    """Chain statistics of consecutive records (strips, or bands) of one pair."""
    start, fed, end = (tl[:, i].astype(np.int64) for i in range(3))
    xcc = (tl[:, 3] >> 32).astype(np.int64)
    hw = (tl[:, 3] & 0xffffffff).astype(np.int64)
    cu = (hw >> 8) & 0xF
    se = (hw >> 13) & 0x7
    t0 = start.min() if t0 is None else t0
    nsteps = n + 63
    lag = np.diff(fed) * 10.0 if len(fed) > 1 else np.zeros(1)  # ns
    step_ns = (end - fed) * 10.0 / nsteps
    clk = (tl[:, 5].astype(np.int64) - tl[:, 4].astype(np.int64))
    mhz = clk / np.maximum(1, (end - fed)) * 100.0  # s_memtime ticks per s_memrealtime (100 MHz) tick
    k = np.arange(1, len(fed))
    cross = (k % W) == 0
    return {
        "records": len(fed),
        "total_us": round((end.max() - t0) * 0.01, 2),
        "first_fed_us": round((fed[0] - t0) * 0.01, 3),
        "last_start_us": round((start[-1] - t0) * 0.01, 2),
        "last_end_us": round((end[-1] - t0) * 0.01, 2),
        "ns_per_step_mean": round(float(step_ns.mean()), 2),
        "ns_per_step_min": round(float(step_ns.min()), 2),
        "ns_per_step_max": round(float(step_ns.max()), 2),
        "lag_ns_in_group_mean": round(float(lag[~cross].mean()), 1) if (~cross).any() else None,
        "lag_ns_cross_group_mean": round(float(lag[cross].mean()), 1) if cross.any() else None,
        "lag_ns_p50": round(float(np.percentile(lag, 50)), 1),
        "lag_ns_p90": round(float(np.percentile(lag, 90)), 1),
        "lag_ns_max": round(float(lag.max()), 1),
        "start_wait_ns_mean": round(float(((fed - start) * 10.0).mean()), 1),
        "shader_mhz_mean": round(float(mhz.mean()), 1),
        "clk_per_step_mean": round(float((clk / nsteps).mean()), 1),
        "ns_per_step_by_strip": [round(float(x), 1) for x in step_ns[:: max(1, len(step_ns) // 16)]],
        "lag_ns_by_strip": [round(float(x), 1) for x in lag[:: max(1, len(lag) // 16)]],
        "fed_us_by_strip": [round(float((x - t0) * 0.01), 2) for x in fed[:: max(1, len(fed) // 16)]],
        "cus_used": int(len(set(zip(xcc.tolist(), se.tolist(), cu.tolist())))),
        "max_strips_on_one_simd_concurrently": max_overlap(xcc, se, cu, (hw >> 4) & 3, fed, end),
        "ns_per_step_by_wave_in_group": [round(float(step_ns[w::W].mean()), 2) for w in range(W)],
        "simd_by_wave_in_group": [sorted(set(((hw[w::W] >> 4) & 3).tolist())) for w in range(W)],
        # cross-group hand-offs whose two groups ran on the same XCD / on different XCDs
        "lag_ns_cross_same_xcd": round(float(lag[cross & (xcc[1:] == xcc[:-1])].mean()), 1) if (cross & (xcc[1:] == xcc[:-1])).any() else None,
        "lag_ns_cross_other_xcd": round(float(lag[cross & (xcc[1:] != xcc[:-1])].mean()), 1) if (cross & (xcc[1:] != xcc[:-1])).any() else None,
        "cross_same_xcd_count": int((cross & (xcc[1:] == xcc[:-1])).sum()),
        "xcc_by_record_first32": [int(x) for x in xcc[:32]],
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=32768)
    ap.add_argument("--m", type=int, default=32768)
    ap.add_argument("--R", type=int, default=1)
    ap.add_argument("--mode", type=int, default=0)
    ap.add_argument("--waves", type=int, default=0)
    ap.add_argument("--pairs", type=int, default=1, help="independent copies of the pair (contention test)")
    ap.add_argument("--score", default="blast", help="blast (+5/-4) or MATCH,MISMATCH (e.g. 1,-3)")
    ap.add_argument("--protein", action="store_true", help="BLOSUM50, letters 0..21 (the harness's dummy requests)")
    ap.add_argument("--letters", type=int, default=0, help="--protein: draw the sequences from letters 0..K-1 only")
    args = ap.parse_args()
    if args.waves:
        os.environ["SA_WAVES_PER_GROUP"] = str(args.waves)
    # the engine reads its knobs once per process: every fill of this process dumps its timeline
    path = os.path.join(tempfile.mkdtemp(), "tl.bin")
    os.environ["SA_TIMELINE"] = path
    from sa_amd import synthetic
    from sa_amd.batch import DeviceBatch
    S = synthetic.blast_matrix()
    if args.score != "blast":
        mt, mm = (int(x) for x in args.score.split(","))
        S = np.full((4, 4), mm, dtype=np.int32)
        np.fill_diagonal(S, mt)
    A = 4
    if args.protein:
        S = np.array(json.load(open(os.path.join(ROOT, "tests", "golden", "matrices.json")))["blosum50"],
                     np.int32).reshape(23, 23)
        A = 22
        if args.letters > 0:
            A = args.letters
    t = synthetic.random_sequence(6, args.n, A)
    p = synthetic.random_sequence(7, args.m, A)
    b = DeviceBatch(args.mode, S, 5, [t] * args.pairs, [p] * args.pairs, rows_per_lane=args.R)
    b.fill()
    b.fill()
    b.fill()  # the file holds the last fill's timeline
    import torch
    torch.cuda.synchronize()
    tl = np.fromfile(path, dtype=np.uint64).reshape(-1, 48)
    if os.environ.get("SA_TL_SAVE"):
        np.save(os.environ["SA_TL_SAVE"], tl)  # raw records for offline analysis
    W = int(os.environ.get("SA_WAVES_PER_GROUP", "4"))
    ns = args.pairs * ((args.m + 64 * args.R - 1) // (64 * args.R))
    t0 = int(tl[:, 0].astype(np.int64).min())
    rec = {"n": args.n, "m": args.m, "R": args.R, "W": W, "pairs": args.pairs, "strips": ns}
    rec.update(summarize(tl[:ns], args.n, W, t0))
    if len(tl) > ns:
        # band fill: the band records follow the strips' (one pair's chain)
        nb = (len(tl) - ns) // args.pairs
        rec["bands"] = summarize(tl[ns:ns + nb], args.n, W, t0)
    prog = tl[:ns, 6:16].astype(np.int64)
    iop = tl[:ns, 16:26].astype(np.int64)
    if prog[:, 1].any():
        # experiment builds (SA_EXP_PROGRESS): time at columns 0, 4096, ... per strip; the lag between
        # consecutive strips at each checkpoint shows whether a consumer falls behind its producer
        ok = (prog > 0).all(axis=0)
        pl = np.diff(prog[:, ok], axis=0) * 10.0
        rec["progress_lag_ns_by_checkpoint"] = [round(float(x), 1) for x in pl.mean(axis=0)]
        kk = np.arange(1, len(prog))
        okr = (prog[1:, 1:9] > 0).all(axis=1) & (prog[:-1, 1:9] > 0).all(axis=1)
        lagq = (prog[1:, 1:9] - prog[:-1, 1:9]) * 10.0  # ns, lag of strip k behind k-1 at checkpoints 1..8
        for nm, sel in (("in_group", (kk % W) != 0), ("cross_group", (kk % W) == 0)):
            L = lagq[sel & okr]
            rec[f"lag_ns_by_checkpoint_{nm}"] = [round(float(x), 1) for x in L.mean(axis=0)]
        rec["progress_lag_ns_first_strips"] = [[round(float(x), 1) for x in r] for r in pl[:6]]
        seg = np.diff(prog[:, ok], axis=1) * 10.0 / 4096
        rec["ns_per_step_by_segment_first"] = [round(float(x), 2) for x in seg[1]]
        rec["ns_per_step_by_segment_last"] = [round(float(x), 2) for x in seg[-2]]
        rec["ns_per_step_by_segment_every32"] = [[k] + [round(float(x), 1) for x in seg[k]] for k in range(0, len(seg), 32)]
        # I/O wave: time ring[0] of group g got column 4096q minus the time the group's first strip
        # reached column 4096q (negative: the feed was there first, the strip was the bottleneck)
        gi = [k for k in range(W, len(prog), W) if iop[k, 1] > 0]
        rec["io_ahead_us_every8groups"] = [[k] + [round(float(prog[k, q] - iop[k, q]) * 0.01, 1) for q in range(1, 9) if iop[k, q] > 0 and prog[k, q] > 0] for k in gi[::8]]
        mt = tl[:ns, 26:36].astype(np.int64)
        segc = np.diff(mt[:, ok], axis=1) / 4096.0
        rec["clk_per_step_by_segment_every32"] = [[k] + [round(float(x), 1) for x in segc[k]] for k in range(0, len(segc), 32)]
        rec["checkpoint_us"] = [[k] + [round(float(x - t0) * 0.01, 1) for x in prog[k, ok]] for k in range(0, len(seg), 64)]
        # slow-path counters per strip: feed checks that failed / their re-reads, publishes that
        # waited for the consumer / their polls (bodies per strip = nsteps / 16)
        sc = tl[:ns, 36:42].astype(np.int64)
        rec["slow_paths_mean_per_strip"] = {nm: round(float(sc[1:, i].mean()), 1) for i, nm in
                                            enumerate(("feed_slow", "feed_spins", "pub_slow", "pub_spins",
                                                       "feed_slow_past_4096", "feed_spins_past_4096"))}
        rec["feed_slow_by_wave_in_group"] = [round(float(sc[w::W, 0].mean()), 1) for w in range(W)]
        rec["feed_slow_past_4096_by_wave_in_group"] = [round(float(sc[w::W, 4].mean()), 1) for w in range(W)]
        rec["feed_spins_past_4096_by_wave_in_group"] = [round(float(sc[w::W, 5].mean()), 1) for w in range(W)]
    print(json.dumps(rec))
    b.close()


if __name__ == "__main__":
    main()
