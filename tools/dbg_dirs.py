"""Development tool: where a fill's direction matrix differs from the oracle's (cell positions, codes).
python tools/dbg_dirs.py MODE R GAP N M"""
import sys, os
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "sequence-alignment-gpu_amd", "python"), os.path.join(ROOT, "oracle")]
import oracle
from sa_amd import synthetic
from sa_amd.batch import DeviceBatch
mode, R, gap, n, m = (int(x) for x in sys.argv[1:6])
S = synthetic.blast_matrix()
t = synthetic.random_sequence(500, n, 4)
p = synthetic.mutate(t, 600, 4, m)
b = DeviceBatch(mode, S, gap, [t], [p], rows_per_lane=R)
b.fill()
got = b.directions(0).reshape(m + 1, n + 1)
exp = np.empty((m + 1) * (n + 1), np.uint8)
oracle.fill_only(mode, t, p, S, gap, exp)
exp = exp.reshape(m + 1, n + 1)
bad = np.argwhere(got != exp)
print("bad", len(bad))
if len(bad):
    rows, cols = bad[:, 0], bad[:, 1]
    print("rows", rows.min(), rows.max(), "cols", cols.min(), cols.max())
    print("rows mod 64", np.bincount((rows - 1) % 64, minlength=64).tolist())
    print("strips", np.unique((rows - 1) // 64).tolist()[:40])
    print("cols mod 32", np.bincount((cols - 1 + (rows - 1) % 64) % 32, minlength=32).tolist())
    for r, c in bad[:20]:
        print(r, c, "got", got[r, c], "exp", exp[r, c])
