"""Table traceback (sa_walk.hip tb_*_kernel, sa_walk.h TbArgs): every strip's window of start columns
is walked in parallel into a table, the tables are chained per group and per pair, and each group's
strips are then walked in parallel from their now-known entry columns (local: then where the walk
ends, from H summed along the path). Checked in subprocesses (the engine reads its knobs once per
process) against the oracle's full alignment in both modes (traceBackNW / traceBackSW,
alignSequenceCPU.cpp:64-114 / :10-62):
  * SA_TB_STRICT=1 (no sequential walk afterwards): every pair below must be resolved by the tables
    alone, so a wrong or missing table result shows as a wrong alignment;
  * default: a pair whose path leaves the windows (a long insertion far off the diagonal; global
    unrelated pairs of unequal lengths, cases 3 and 4; a local alignment across a 1500-column gap)
    falls back to the sequential walk and is still exact;
  * SA_TB_ROUNDS=4 + SA_TB_STRICT=1: rounds re-centred at the failure point resolve those pairs too;
  * SA_TB_TABLES=0: the sequential walk alone on the same pairs."""
from __future__ import annotations

import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SCRIPT = r'''
import os, sys, json, numpy as np
sys.path[:0] = [sys.argv[1] + "/sequence-alignment-gpu_amd/python", sys.argv[1] + "/oracle"]
import oracle
from sa_amd import engine, synthetic
S = synthetic.blast_matrix()
B50 = np.array(json.load(open(sys.argv[1] + "/tests/golden/matrices.json"))["blosum50"], np.int32).reshape(23, 23)
which = sys.argv[2]
bad = []
def one(t, p, S, gap, tag, mode=0):
    r = engine.align_pair(mode, t, p, S, gap, device=0)
    r.pop("fill_us")
    if r != oracle.align(mode, t, p, S, gap):
        bad.append(tag + (mode,))
cases = [  # (n, m, gap, related, alphabet) -- m rows (8+ strips), n columns
    (4096, 4096, 5, False, 4), (4096, 4096, 5, True, 4), (1000, 5000, 5, True, 4), (3000, 20000, 5, False, 4),
    (20000, 3000, 5, False, 4), (9000, 8191, 0, True, 4), (5000, 4097, -2, False, 4), (600, 700, 5, False, 4),
    (3000, 2000, 5, False, 23), (2500, 2600, 5, True, 23), (2047, 4000, 5, False, 4), (2049, 4000, 5, True, 4)]
for k, (n, m, gap, rel, A) in enumerate(cases):
    t = synthetic.random_sequence(70 + k, n, 4 if A == 4 else 20)
    p = synthetic.mutate(t, 90 + k, 4 if A == 4 else 20, m) if rel else synthetic.random_sequence(110 + k, m, 4 if A == 4 else 20)
    for mode in (0, 1):
        if which == "strict" and mode == 0 and k in ((4,) if "SA_TB_ROUNDS" in os.environ else (3, 4)):
            # unrelated pairs of unequal lengths: the path strays from the line through (m, n), (0, 0);
            # rounds re-centred on it resolve case 3, while case 4 (17000 more columns than rows) has
            # LEFT runs longer than a window inside a group (it falls back in the other tests)
            continue
        one(t, p, S if A == 4 else B50, gap, ("case", k), mode)
if which == "fallback":
    # local: two copied segments of the text 1500 columns apart, one alignment across the gap (the
    # path leaves the slope-1 line through the best cell by 1500 columns)
    t = synthetic.random_sequence(210, 10000, 4)
    p = np.concatenate([t[500:4000], t[5500:9000]])
    one(t, p, S, 5, ("fallback_local", 0), 1)
    # the pattern matches the END of a much longer text: the path runs down the diagonal near column n
    # and then LEFT along row ~0, far from the line through (m, n) and (0, 0) (windows of 2048 columns)
    t = synthetic.random_sequence(200, 12000, 4)
    p = synthetic.mutate(t[-3000:], 201, 4, 3000)
    one(t, p, S, 5, ("fallback", 0))
    # several pairs in one plan: table pairs, a fallback pair and short pairs (sequential walk)
    ts = [synthetic.random_sequence(300 + k, 900 + 1700 * k, 4) for k in range(4)] + [t]
    ps = [synthetic.mutate(ts[k], 310 + k, 4, 200 + 1300 * k) for k in range(4)] + [p]
    for mode in (0, 1):
        got = engine.align_batch(mode, ts, ps, S, 5, num_gpus=1)
        for k in range(5):
            if got[k] != oracle.align(mode, ts[k], ps[k], S, 5):
                bad.append(("batch", k, mode))
print("TB_OK" if not bad else "TB_BAD %r" % (bad,))
'''


SWEEP = r'''
import os, sys, json, numpy as np
sys.path[:0] = [sys.argv[1] + "/sequence-alignment-gpu_amd/python", sys.argv[1] + "/oracle"]
import oracle
from sa_amd import engine, synthetic
S4 = synthetic.blast_matrix()
B50 = np.array(json.load(open(sys.argv[1] + "/tests/golden/matrices.json"))["blosum50"], np.int32).reshape(23, 23)
rng = np.random.default_rng(int(sys.argv[2]))
bad = []
for k in range(24):
    mode = int(rng.integers(0, 2))
    prot = bool(rng.integers(0, 4) == 0)
    A, S = (20, B50) if prot else (4, S4)
    m = int(rng.integers(512, 3000))
    n = int(rng.integers(300, 3200))
    gap = int(rng.choice([5, 5, 3, 0, -1, -2]))
    t = synthetic.random_sequence(5000 + k, n, A)
    p = synthetic.mutate(t, 5100 + k, A, m) if rng.integers(0, 2) else synthetic.random_sequence(5200 + k, m, A)
    r = engine.align_pair(mode, t, p, S, gap, device=0)
    r.pop("fill_us")
    if r != oracle.align(mode, t, p, S, gap):
        bad.append((k, mode, A, n, m, gap))
print("TB_OK" if not bad else "TB_BAD %r" % (bad,))
'''


def _run(which, **env):
    e = dict(os.environ, **env)
    out = subprocess.run([sys.executable, "-c", SCRIPT, ROOT, which], env=e, capture_output=True, text=True, timeout=110)
    assert out.returncode == 0, out.stdout[-2000:] + out.stderr[-2000:]
    assert "TB_OK" in out.stdout, out.stdout[-2000:]


@pytest.mark.gpu
def test_table_traceback_strict_vs_oracle():
    _run("strict", SA_TB_STRICT="1")


@pytest.mark.gpu
def test_table_traceback_rounds_strict_vs_oracle():
    """Four rounds of tables (SA_TB_ROUNDS=4; the default past 131072 rows): an unequal-length
    unrelated global pair the first round's windows miss (case 3) resolves from an anchor at the group
    where the path left them, still without the sequential walk."""
    _run("strict", SA_TB_STRICT="1", SA_TB_ROUNDS="4")


@pytest.mark.gpu
def test_table_traceback_fallback_vs_oracle():
    _run("fallback")


@pytest.mark.gpu
def test_sequential_walk_same_pairs_vs_oracle():
    _run("fallback", SA_TB_TABLES="0")


@pytest.mark.gpu
@pytest.mark.parametrize("rounds", ["1", "4"])
def test_table_traceback_random_sweep_vs_oracle(rounds):
    """24 random pairs (512..3000 rows, 300..3200 columns, both modes, DNA / BLOSUM50, gaps 5 / 3 / 0 /
    -1 / -2, related or not) with one or four rounds of tables: every result equals the oracle's
    (pairs the tables leave fall back)."""
    e = dict(os.environ, SA_TB_ROUNDS=rounds)
    out = subprocess.run([sys.executable, "-c", SWEEP, ROOT, "7" + rounds], env=e, capture_output=True, text=True, timeout=110)
    assert out.returncode == 0, out.stdout[-2000:] + out.stderr[-2000:]
    assert "TB_OK" in out.stdout, out.stdout[-2000:]


LONG_LOCAL = r'''
import os, sys, json, hashlib, numpy as np
sys.path[:0] = [sys.argv[1] + "/sequence-alignment-gpu_amd/python"]
from sa_amd import engine, synthetic
S = synthetic.blast_matrix()
# a related local pair past 131072 rows (the default multi-round table path): 6000 unrelated rows, a
# mutated copy of 140000 text letters, 6000 unrelated rows, so traceBackSW ends (STOP) thousands of
# rows above row 1 and the walk crosses the round boundary
t = synthetic.random_sequence(880, 150000, 4)
core = synthetic.mutate(t[4000:144000], 881, 4, 138000)
p = np.concatenate([synthetic.random_sequence(882, 6000, 4), core, synthetic.random_sequence(883, 6000, 4)])
r = engine.align_pair(1, t, p, S, 5, device=0)
r.pop("fill_us")
at, ap = r.pop("aligned_text"), r.pop("aligned_pattern")
alpha = "ATCG"
sc = 0
for a, b in zip(at, ap):
    sc += -5 if a == "-" or b == "-" else int(S[alpha.index(b), alpha.index(a)])
ft, fp = "".join(alpha[c] for c in t), "".join(alpha[c] for c in p)
tu, pu = at.replace("-", ""), ap.replace("-", "")
ok_t = ft.find(tu, max(0, r["start_text"] - 1)) in (r["start_text"], r["start_text"] + 1)
ok_p = fp.find(pu, max(0, r["start_pattern"] - 1)) in (r["start_pattern"], r["start_pattern"] + 1)
r["sha"] = hashlib.sha256((at + "|" + ap).encode()).hexdigest()
r["rescored"] = sc
r["substrings_at_starts"] = bool(ok_t and ok_p)
print("RESULT " + json.dumps(r))
'''


@pytest.mark.gpu
def test_long_local_table_rounds_vs_sequential_walk():
    """Local table traceback past 131072 rows (the default rounds path, which re-anchors on the path's
    slope and keeps the groups resolved before a failure): a related 150000 x 150000 local pair whose
    walk ends (STOP) about 6000 rows above row 1 (the alignment reaches into the unrelated prefix by chance matches). The oracle would take minutes here, so the default
    path is compared field by field with the sequential walk (SA_TB_TABLES=0) in a second process, and
    both alignments must re-score to the score and be substrings of the inputs at the reported starts
    (traceBackSW's start quirk: the first aligned index or one less, alignSequenceCPU.cpp:45-53)."""
    res = {}
    for tag, env in (("tables", {}), ("walk", {"SA_TB_TABLES": "0"})):
        out = subprocess.run([sys.executable, "-c", LONG_LOCAL, ROOT], env=dict(os.environ, **env),
                             capture_output=True, text=True, timeout=110)
        assert out.returncode == 0, out.stdout[-2000:] + out.stderr[-2000:]
        line = [x for x in out.stdout.splitlines() if x.startswith("RESULT ")]
        assert line, out.stdout[-2000:]
        res[tag] = __import__("json").loads(line[-1][7:])
    a, b = res["tables"], res["walk"]
    assert a == b, (a, b)
    assert a["rescored"] == a["score"] and a["substrings_at_starts"], a
    assert a["start_pattern"] > 1000 and a["num_bytes"] > 131072, a
