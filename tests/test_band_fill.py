"""The band fill (sa_fill.hip process_band): 128-row score strips ("bands", two rows per lane, the
recurrence alone) run ahead on their own workgroups and feed the 64-row strips, which write the
direction planes, the global score and the local best cell. Checked in subprocesses (the engine reads
its knobs once per process) with SA_BAND=1 / 0 on small chains, cell by cell against the oracle's
DIRECTION matrix (alignSequenceCPU.cpp:116-201 local, :203-284 global) and the full alignment
(:10-114), for both modes and gaps 5 / 0 (and -2, global only: local kArr8 needs g >= 0, the plan
falls back to the one-wave fill there); at the default shapes (>= 16384 columns, several band and
strip groups); more groups than CUs (SA_MAX_CUS: persistent band and strip workers); a 23-letter
BLOSUM50 pair in both modes (the global band kernel without the code touch); protein chains reading copy 0
of their text profiles (kArr8A) with SA_ALIGN=1 / 0 / 2; with several chained pairs per plan (band groups spanning pairs); and a local then a
global 32768^2 call in one fresh process, against the reference's recorded outputs (large.json)."""
from __future__ import annotations

import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

HEAD = r'''
import sys, json, numpy as np
sys.path[:0] = [sys.argv[1] + "/sequence-alignment-gpu_amd/python", sys.argv[1] + "/oracle"]
import oracle
from sa_amd import engine, synthetic
from sa_amd.batch import DeviceBatch
S = synthetic.blast_matrix()
bad = []
def check(mode, n, m, gap, seed, related, S=S):
    A = S.shape[0]
    t = synthetic.random_sequence(seed, n, A)
    p = synthetic.mutate(t, seed + 1, A, m) if related else synthetic.random_sequence(seed + 2, m, A)
    b = DeviceBatch(mode, S, gap, [t], [p], rows_per_lane=1)
    b.fill()
    got = b.directions(0)
    b.close()
    exp = np.empty((m + 1) * (n + 1), np.uint8)
    oracle.fill_only(mode, t, p, S, gap, exp)  # (the reference's M, STOP included)
    nbad = int((got != exp).sum())
    if nbad:
        bad.append(("dirs", mode, n, m, gap, nbad))
    r = engine.align_pair(mode, t, p, S, gap, device=0)
    r.pop("fill_us")
    if r != oracle.align(mode, t, p, S, gap):
        bad.append(("align", mode, n, m, gap))
'''

SMALL = HEAD + r'''
cases = [(3000, 2900, 5), (2100, 1000, 0), (700, 1100, 3), (4500, 260, -2), (1500, 257, 5), (999, 513, 5)]
for k, (n, m, gap) in enumerate(cases):
    for mode in (0, 1):
        check(mode, n, m, gap, 800 + 10 * k, k % 2 == 0)
# protein (23 letters, BLOSUM50): the global band kernel without the code touch (the touching kernel
# serves alphabets of at most 4 letters) and the local band kernel, cell by cell
B50 = np.array(json.load(open(sys.argv[1] + "/tests/golden/matrices.json"))["blosum50"], np.int32).reshape(23, 23)
for mode in (0, 1):
    check(mode, 3000, 1100, 5, 900 + mode, mode == 0, S=B50)
# several chained pairs in one plan, even strip counts (each pair's first strip even): band groups
# and strip groups span pair boundaries
ts = [synthetic.random_sequence(1000 + k, 1800 + 97 * k, 4) for k in range(5)]
ps = [synthetic.mutate(t, 1100 + k, 4, 128 * (2 + 3 * k)) for k, t in enumerate(ts)]
for mode in (0, 1):
    got = engine.align_batch(mode, ts, ps, S, 5, num_gpus=1)
    for k in range(5):
        if got[k] != oracle.align(mode, ts[k], ps[k], S, 5):
            bad.append(("batch", mode, k))
print("BAND_OK" if not bad else "BAND_BAD %r" % (bad,))
'''

DEFAULT = HEAD + r'''
# the default path at >= 16384 columns: 18 strips, 8 bands, several groups of each
for mode, gap in ((0, 5), (0, -2), (1, 5), (1, 0)):
    check(mode, 16384, 1100, gap, 4000 + 7 * mode + gap, True)
print("BAND_OK" if not bad else "BAND_BAD %r" % (bad,))
'''

# more band and strip groups than the (capped) CUs: persistent workers loop over their queues
PERSIST = HEAD + r'''
for mode, gap in ((0, 5), (1, 5)):
    check(mode, 2048, 8192, gap, 5000 + mode, False)
print("BAND_OK" if not bad else "BAND_BAD %r" % (bad,))
'''

LARGE = r'''
import sys, json
sys.path[:0] = [sys.argv[1] + "/sequence-alignment-gpu_amd/python", sys.argv[1] + "/tests"]
from sa_amd import engine, synthetic
from conftest import matrix, same_result
cases = {c["name"]: c for c in json.load(open(sys.argv[1] + "/tests/golden/large.json"))}
bad = []
for name in ("cfg3_dna_local_32768_uniform", "headline_dna_global_32768_uniform"):
    c = cases[name]
    A = c["letters"]
    t = synthetic.random_sequence(c["text_seed"], c["n"], A)
    p = (synthetic.random_sequence(c["pattern_seed"], c["m"], A) if c["pattern_kind"] == "rand"
         else synthetic.mutate(t, c["pattern_seed"], A, c["m"]))
    S = matrix(c["matrix"], 4 if c["matrix"] == "blast" else 23)
    got = engine.align_pair(c["mode"], t, p, S, c["gap"], device=0)
    if not same_result(got, c["result"]):
        bad.append(name)
print("BAND_OK" if not bad else "BAND_BAD %r" % (bad,))
'''


# protein chains read copy 0 of their text profiles and shift the bytes in registers (kArr8A,
# sa_fill.h; SA_ALIGN=0: the four byte copies; 2: DNA as well): text lengths of every residue mod 4
# and mod 16 (the lane windows' byte shifts and the last body's padding), band and one-wave chains,
# both modes, cell by cell
ALIGN = HEAD + r'''
B50 = np.array(json.load(open(sys.argv[1] + "/tests/golden/matrices.json"))["blosum50"], np.int32).reshape(23, 23)
B62 = np.array(json.load(open(sys.argv[1] + "/tests/golden/matrices.json"))["blosum62"], np.int32).reshape(23, 23)
cases = [(3001, 1100, 5), (2998, 700, 0), (1283, 1500, 3), (4099, 257, 5), (515, 640, 5)]
for k, (n, m, gap) in enumerate(cases):
    for mode in (0, 1):
        check(mode, n, m, gap, 1200 + 10 * k, k % 2 == 1, S=B50 if k % 2 == 0 else B62)
for k, (n, m) in enumerate([(1, 300), (3, 65), (17, 200), (33, 129), (64, 700)]):  # short texts: padding reads
    for mode in (0, 1):
        check(mode, n, m, 5, 1400 + 10 * k, False, S=B50)
check(0, 2500, 900, 5, 1300, True)  # DNA (copy-0 reads only with SA_ALIGN=2)
check(1, 2047, 1300, 5, 1310, False)
print("BAND_OK" if not bad else "BAND_BAD %r" % (bad,))
'''


@pytest.mark.gpu
@pytest.mark.parametrize("align", ["1", "0", "2"])
@pytest.mark.parametrize("band", ["1", "0"])
def test_copy0_profile_reads_vs_oracle(align, band):
    _run(ALIGN, SA_ALIGN=align, SA_BAND=band)


def _run(script, **env):
    e = dict(os.environ, SA_HANDOFF_TIMEOUT_S="10", **env)
    out = subprocess.run([sys.executable, "-c", script, ROOT], env=e, capture_output=True, text=True, timeout=110)
    assert out.returncode == 0, out.stdout[-2000:] + out.stderr[-2000:]
    assert "BAND_OK" in out.stdout, out.stdout[-2000:]


@pytest.mark.gpu
@pytest.mark.parametrize("band", ["1", "0"])
def test_band_fill_vs_oracle(band):
    _run(SMALL, SA_BAND=band)


@pytest.mark.gpu
def test_band_fill_default_shapes_vs_oracle():
    _run(DEFAULT)


@pytest.mark.gpu
def test_band_fill_persistent_workers_vs_oracle():
    """SA_MAX_CUS=16 plans a 2048 x 8192 pair (16 band groups + 32 strip groups) on 16 CUs: 5 band and
    11 strip workgroups take their groups from the queues in chain order; every cell of the direction
    matrix and the alignment must still be the reference's (both modes)."""
    _run(PERSIST, SA_MAX_CUS="16")


@pytest.mark.gpu
@pytest.mark.parametrize("per_cu", ["1", "2"])
def test_one_wave_chain_fill_per_cu_vs_oracle(per_cu):
    """The same plans without bands (SA_BAND=0): 32 strip groups on 16 CUs with one chain workgroup
    per CU (the default for a few long pairs, a 96 KB LDS request) or two; cell by cell as above."""
    _run(PERSIST, SA_MAX_CUS="16", SA_BAND="0", SA_CHAIN_PER_CU=per_cu)


@pytest.mark.gpu
def test_local_then_global_32k_fresh_process():
    _run(LARGE)


def test_large_fixture_names():
    """(CPU) the fixtures the fresh-process test reads exist."""
    names = {c["name"] for c in json.load(open(os.path.join(ROOT, "tests", "golden", "large.json")))}
    assert {"cfg3_dna_local_32768_uniform", "headline_dna_global_32768_uniform"} <= names
