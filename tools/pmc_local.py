#!/usr/bin/env python3
"""Driver for PMC passes (development): three fills of one plan (mode, n, m, pairs copies)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sequence-alignment-gpu_amd", "python"))
from sa_amd import synthetic  # noqa: E402
from sa_amd.batch import DeviceBatch  # noqa: E402

mode, n, m, pairs = (int(x) for x in sys.argv[1:5])
t = synthetic.random_sequence(6, n, 4)
p = synthetic.random_sequence(7, m, 4)
b = DeviceBatch(mode, synthetic.blast_matrix(), 5, [t] * pairs, [p] * pairs)
for _ in range(3):
    b.fill()
b.close()
