"""The dual fill (sa_fill.hip: score waves run the recurrence alone, direction waves on the other CUs
recompute every (strip, segment) and write the planes), forced on small chains in a subprocess (the
engine reads its knobs once per process): SA_DUAL=1 with 64- and 1024-step segments, cell by cell
against the oracle's DIRECTION matrix (alignSequenceCPU.cpp:203-284) and the full alignment
(:64-114). Large texts use the dual fill by default, so test_large_configs / test_full_size_properties
cover it at full size as well."""
from __future__ import annotations

import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SCRIPT = r'''
import sys, numpy as np
sys.path[:0] = [sys.argv[1] + "/sequence-alignment-gpu_amd/python", sys.argv[1] + "/oracle"]
import oracle
from sa_amd import engine, synthetic
from sa_amd.batch import DeviceBatch
S = synthetic.blast_matrix()
bad = []
# multi-strip, multi-group chains (R = 1 global), odd shapes, a pair whose strips end mid-group
for k, (n, m, gap) in enumerate([(3000, 2900, 5), (2100, 1000, 0), (700, 1100, 3), (4500, 260, -2)]):
    t = synthetic.random_sequence(800 + k, n, 4)
    p = synthetic.mutate(t, 900 + k, 4, m) if k % 2 == 0 else synthetic.random_sequence(950 + k, m, 4)
    b = DeviceBatch(0, S, gap, [t], [p], rows_per_lane=1)
    b.fill()
    got = b.directions(0)
    b.close()
    exp = np.empty((m + 1) * (n + 1), np.uint8)
    oracle.fill_only(0, t, p, S, gap, exp)
    if int((got != exp).sum()):
        bad.append(("dirs", n, m, gap, int((got != exp).sum())))
    r = engine.align_pair(0, t, p, S, gap, device=0)
    r.pop("fill_us")
    if r != oracle.align(0, t, p, S, gap):
        bad.append(("align", n, m, gap))
# several chained pairs in one plan (groups span pair boundaries)
ts = [synthetic.random_sequence(1000 + k, 1800 + 97 * k, 4) for k in range(5)]
ps = [synthetic.mutate(t, 1100 + k, 4, 300 + 211 * k) for k, t in enumerate(ts)]
got = engine.align_batch(0, ts, ps, S, 5, num_gpus=1)
for k in range(5):
    if got[k] != oracle.align(0, ts[k], ps[k], S, 5):
        bad.append(("batch", k))
print("DUAL_OK" if not bad else "DUAL_BAD %r" % (bad,))
'''


@pytest.mark.gpu
@pytest.mark.parametrize("seg", [64, 1024])
def test_dual_fill_vs_oracle(seg):
    env = dict(os.environ, SA_DUAL="1", SA_DUAL_SEG=str(seg), SA_HANDOFF_TIMEOUT_S="10")
    out = subprocess.run([sys.executable, "-c", SCRIPT, ROOT], env=env, capture_output=True, text=True, timeout=110)
    assert out.returncode == 0, out.stdout[-2000:] + out.stderr[-2000:]
    assert "DUAL_OK" in out.stdout, out.stdout[-2000:]
