#!/usr/bin/env python3
"""Column-walk phase split (experiment build with SA_EXP_WALK_TIMING): a batch plan of 2048^2 DNA
global pairs, shader clocks per column in staging vs the walk proper, averaged over pairs."""
import os
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sequence-alignment-gpu_amd", "python"))
path = os.path.join(tempfile.mkdtemp(), "tm.bin")
os.environ["SA_TB_TIMING"] = path
from sa_amd import synthetic  # noqa: E402
from sa_amd.batch import DeviceBatch  # noqa: E402

npairs = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
L = 2048
ts = [synthetic.random_sequence(1000 + 2 * i, L, 4) for i in range(npairs)]
ps = [synthetic.random_sequence(1001 + 2 * i, L, 4) for i in range(npairs)]
b = DeviceBatch(0, synthetic.blast_matrix(), 5, ts, ps)
b.fill()
b.traceback()
b.traceback()
tm = np.fromfile(path, dtype=np.uint64).astype(np.int64)
walk_us = (tm[1:2 * npairs:2] - tm[0:2 * npairs:2]) * 0.01
st = tm[2 * npairs::2][:npairs] / L
wk = tm[2 * npairs + 1::2][:npairs] / L
print({"pairs": npairs, "walk_us_mean": round(float(walk_us.mean()), 1), "walk_us_max": round(float(walk_us.max()), 1),
       "stage_clk_per_col": round(float(st.mean()), 1), "walk_clk_per_col": round(float(wk.mean()), 1)})
b.close()
