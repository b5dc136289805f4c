#!/usr/bin/env python3
"""Debug aid (GPU): regenerates sa_api_check's requests (same LCG) and compares the plan's direction
matrices with the oracle's for the requested indices; prints the first wrong cell per strip."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sequence-alignment-gpu_amd", "python"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle  # noqa: E402
from sa_amd import synthetic  # noqa: E402
from sa_amd.batch import DeviceBatch  # noqa: E402

mode = 1 if sys.argv[1] == "local" else 0
count, maxlen = int(sys.argv[2]), int(sys.argv[3])
which = [int(x) for x in sys.argv[4].split(",")]
M64 = (1 << 64) - 1
seed = 12345


def nxt():
    global seed
    seed = (seed * 6364136223846793005 + 1442695040888963407) & M64
    return seed >> 33


texts, pats = [], []
for i in range(count):
    n = 1 + nxt() % maxlen
    m = 1 + nxt() % n
    t = np.array([nxt() % 4 for _ in range(n)], np.int8)
    p = np.empty(m, np.int8)
    for x in range(m):
        if (i & 1) == 0:
            r = nxt() % 8
            p[x] = t[x] if r else nxt() % 4
        else:
            p[x] = nxt() % 4
    texts.append(t)
    pats.append(p)
S = synthetic.blast_matrix()
b = DeviceBatch(mode, S, 5, texts, pats)
b.fill()
b.traceback()
res = b.all_alignments()
for i in which:
    n, m = len(texts[i]), len(pats[i])
    M = b.directions(i).reshape(m + 1, n + 1)
    E = np.empty((m + 1) * (n + 1), np.uint8)
    oracle.fill_only(mode, texts[i], pats[i], S, 5, E)
    E = E.reshape(m + 1, n + 1)
    bad = np.argwhere(M != E)
    print("pair", i, n, "x", m, "wrong cells", len(bad), "score", res[i]["score"],
          "oracle", oracle.align(mode, texts[i], pats[i], S, 5)["score"])
    seen = set()
    for r, c in bad:
        st = (r - 1) // 64
        if st in seen:
            continue
        seen.add(st)
        print("  strip", st, "first wrong row", r, "col", c, "got", M[r, c], "exp", E[r, c])
        if len(seen) > 6:
            break
bad_pairs = [i for i in range(count) if res[i] != oracle.align(mode, texts[i], pats[i], S, 5)]
print("pairs with wrong results:", bad_pairs)
