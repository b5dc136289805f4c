#!/usr/bin/env python3
"""Band start-up decomposition (experiment build with SA_EXP_BAND_STAMPS, development tool): for each
band, when its first feed arrived (fed), when it finished its first five bodies (the fifth publishes
the next band's first feed), and when the next band's first feed arrived. Prints means over the chain
in ns: fed -> body k done, and publish -> next fed (detection)."""
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
tl = np.fromfile(path, dtype=np.uint64).reshape(-1, 48).astype(np.int64)
ns = (m + 63) // 64
bd = tl[ns:]
fed = bd[:, 1]
body = bd[:, 6:11]
ok = (body > 0).all(axis=1)
lag = np.diff(fed) * 10.0
rel = (body - fed[:, None]) * 10.0
det = (fed[1:] - body[:-1, 4]) * 10.0
W = 4
k = np.arange(1, len(fed))
ing = (k % W) != 0
st = tl[:ns]
print({"total_us": round(float(st[:, 2].max() - tl[:, 0][tl[:, 0] > 0].min()) * 0.01, 1), "bands": len(fed), "stamped": int(ok.sum()),
       "fed_to_body_done_ns": [round(float(x), 1) for x in rel[ok].mean(axis=0)],
       "lag_in_group_ns": round(float(lag[ing].mean()), 1), "lag_cross_ns": round(float(lag[~ing].mean()), 1),
       "first_publish_to_next_fed_in_group_ns": round(float(det[ing & ok[:-1]].mean()), 1),
       "first_publish_to_next_fed_cross_ns": round(float(det[~ing & ok[:-1]].mean()), 1),
       # fed -> fifth body done by the band's slot in its group (slots 0 and 1 share a SIMD with the
       # I/O and drain waves), and the cross-group hand-off (slot 3 -> next group's slot 0)
       "body5_by_slot_ns": [round(float(rel[ok & (np.arange(len(fed)) % W == w), 4].mean()), 1) for w in range(W)],
       "lag_by_slot_ns": [round(float(lag[(k % W) == w].mean()), 1) for w in range(W)]})
# bodies 0..10 of in-group bands against their producer (the band above, same workgroup): body j's
# end (C), its next feed in hand (R), and the producer's body 5 + j end, which published that feed (P)
C, Rd = bd[:, 6:17], bd[:, 22:33]
P = bd[:, 11:22]
sel = np.nonzero(ing & (bd[1:, 6:22] > 0).all(axis=1) & (bd[:-1, 6:22] > 0).all(axis=1))[0] + 1
if len(sel):
    Cs, Rs, Ps = C[sel], Rd[sel], P[sel - 1]

    print({"in_group_bands": len(sel),
           "body_ns": [round(float(x), 1) for x in ((Cs[:, 1:] - Rs[:, :-1]) * 10.0).mean(axis=0)],
           "feed_wait_ns": [round(float(x), 1) for x in ((Rs - Cs) * 10.0).mean(axis=0)],
           "missed_frac": [round(float(x), 2) for x in (((Rs - Cs) * 10.0) > 60).mean(axis=0)],
           "end_minus_publish_ns": [round(float(x), 1) for x in ((Cs - Ps) * 10.0).mean(axis=0)],
           "ready_minus_publish_ns": [round(float(x), 1) for x in ((Rs - Ps) * 10.0).mean(axis=0)]})
b.close()
