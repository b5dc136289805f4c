#!/usr/bin/env python3
"""Band feed misses (experiment build with SA_EXP_BAND_MISS, development tool): how often a band's
feed prefetch (the ds_read at step BAND_PF_STEP of a body) found the next body's columns not yet
published, so that the band entered its slow path: per body index for the first 32 bodies, and over
all bodies; with the in-group and cross-group lags of the same run. Unlike the body stamps this adds
nothing to the fast path.   python3 tools/band_miss.py [n] [mode]"""
import os
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sequence-alignment-gpu_amd", "python"))
n = m = int(sys.argv[1]) if len(sys.argv) > 1 else 32768
mode = int(sys.argv[2]) if len(sys.argv) > 2 else 0
path = os.path.join(tempfile.mkdtemp(), "tl.bin")
os.environ["SA_TIMELINE"] = path
from sa_amd import synthetic
from sa_amd.batch import DeviceBatch

b = DeviceBatch(mode, synthetic.blast_matrix(), 5, [synthetic.random_sequence(6, n, 4)], [synthetic.random_sequence(7, m, 4)],
                rows_per_lane=1)
for _ in range(3):
    b.fill()
import torch
torch.cuda.synchronize()
tl = np.fromfile(path, dtype=np.uint64).reshape(-1, 48)
ns = (m + 63) // 64
bd = tl[ns:].astype(np.int64)
st = tl[:ns].astype(np.int64)
fed = bd[:, 1]
lag = np.diff(fed) * 10.0
W = 4
k = np.arange(1, len(fed))
ing = (k % W) != 0
mask = tl[ns:, 38]
bodies = (n + 64 + 31) // 32 * 2
hp = np.arange(len(fed)) % 1 == 0
hp[0] = False  # the pair's first band has no feed
bits = np.array([[(int(x) >> j) & 1 for j in range(32)] for x in mask[hp]])
print({"total_us": round(float(st[:, 2].max() - tl[:, 0][tl[:, 0] > 0].min()) * 0.01, 1),
       "lag_in_group_ns": round(float(lag[ing].mean()), 1), "lag_cross_ns": round(float(lag[~ing].mean()), 1),
       "miss_frac_body0_31": [round(float(x), 2) for x in bits.mean(axis=0)],
       "misses_per_band": round(float(bd[hp, 39].mean()), 1), "bodies_per_band": bodies,
       "polls_per_band": round(float(bd[hp, 40].mean()), 1),
       "first_feed_polls": round(float(bd[hp, 41].mean()), 1),
       "misses_by_slot": [round(float(bd[hp & (np.arange(len(fed)) % W == w), 39].mean()), 1) for w in range(W)]})
# XCD of each band (timeline word 3, high half: HW_REG_XCC_ID) and the cross-group lag split by
# whether the two groups share an XCD (one L2)
xcc = ((tl[ns:, 3] >> np.uint64(32)) & np.uint64(0xF)).astype(np.int64)
cross = np.nonzero(~ing)[0]  # lag[i]: band i -> i + 1
same = xcc[cross] == xcc[cross + 1]
print({"group_xcc_first16": xcc[::W][:16].tolist(),
       "cross_lag_same_xcd_ns": round(float(lag[cross][same].mean()), 1) if same.any() else None,
       "cross_lag_other_xcd_ns": round(float(lag[cross][~same].mean()), 1) if (~same).any() else None,
       "cross_same_count": int(same.sum()), "cross_count": len(cross)})
b.close()
