"""GPU parity: the HIP engine (through the C ABI, include/sa_hip.h) against the reference's own outputs
(tests/golden/*, produced by alignSequenceCPU of the reference) and against the oracle on seeded inputs.
Bit-exact: score, aligned text, aligned pattern, start indices."""
from __future__ import annotations

import hashlib
import itertools

import numpy as np
import pytest

import oracle
from conftest import encode, matrix, same_result
from sa_amd import synthetic

pytestmark = pytest.mark.gpu



def _inputs(case):
    A = case["A"]
    return encode(case["text"], A), encode(case["pattern"], A), matrix(case["matrix"], A)


def test_wave_primitives_selftest(eng):
    eng.selftest(0)


def test_known_answers(eng, golden):
    for case in golden["known_answers.json"]:
        t, p, S = _inputs(case)
        got = eng.align_pair(case["mode"], t, p, S, case["gap"])
        assert same_result(got, case["result"]), case["name"]
        if case["expect_score"] is not None:
            assert got["score"] == case["expect_score"]


def test_data_pairs_one_shot(eng, golden):
    d = golden["data_pairs.json"]
    seqs = d["sequences"]
    for case in d["cases"]:
        A = case["A"]
        got = eng.align_pair(case["mode"], encode(seqs[case["text"]], A), encode(seqs[case["pattern"]], A),
                             matrix(case["matrix"], A), case["gap"])
        assert same_result(got, case["result"]), (case["text"], case["pattern"], case["mode"])


def test_data_pairs_batched(eng, golden):
    """tests.cu:463-551 as ONE plan per (mode, alphabet): many pairs per fill launch."""
    from sa_amd.batch import DeviceBatch
    d = golden["data_pairs.json"]
    seqs = d["sequences"]
    key = lambda c: (c["mode"], c["A"], c["gap"], c["matrix"])
    cases = sorted(d["cases"], key=key)
    for (mode, A, gap, mat), grp in itertools.groupby(cases, key=key):
        grp = list(grp)
        b = DeviceBatch(mode, matrix(mat, A), gap, [encode(seqs[c["text"]], A) for c in grp],
                        [encode(seqs[c["pattern"]], A) for c in grp])
        res = b.run()
        for k, c in enumerate(grp):
            at, ap = b.alignment(k)
            got = dict(res[k], aligned_text=at, aligned_pattern=ap)
            assert same_result(got, c["result"]), (c["text"], c["pattern"], mode)
        b.close()


@pytest.mark.parametrize("rows_per_lane", [0, 1, 2, 4, 8, 16, 32])
def test_random_pairs(eng, golden, rows_per_lane):
    """Edge lengths (1..1000 around multiples of 64), ties, zero-score local alignments, asymmetric and
    wide-range matrices, pattern longer than text; every strip height of the engine."""
    for k, case in enumerate(golden["random_pairs.json"]):
        t, p, S = _inputs(case)
        got = eng.align_pair(case["mode"], t, p, S, case["gap"], rows_per_lane=rows_per_lane)
        assert same_result(got, case["result"]), (k, case["tag"], len(t), len(p))


@pytest.mark.parametrize("rows_per_lane", [0, 1, 2, 4, 8, 16, 32])
def test_gap_pairs(eng, rows_per_lane):
    """Gap penalties 0, -1, -2, -5, both modes, DNA and protein, single strips and multi-group chains
    (tests/golden/gap_pairs.json, from the reference: its CLI takes any int, utilities.cpp:188-199)."""
    from conftest import load
    for k, case in enumerate(load("gap_pairs.json")):
        t, p, S = _inputs(case)
        got = eng.align_pair(case["mode"], t, p, S, case["gap"], rows_per_lane=rows_per_lane)
        assert same_result(got, case["result"]), (k, case["tag"], case["gap"], len(t), len(p))


def test_gap_pairs_batched(eng):
    """The same cases as one plan per (mode, alphabet, gap, matrix): many pairs per fill launch."""
    from conftest import load
    from sa_amd.batch import DeviceBatch
    key = lambda c: (c["mode"], c["A"], c["gap"], c["matrix"])
    for (mode, A, gap, mat), grp in itertools.groupby(sorted(load("gap_pairs.json"), key=key), key=key):
        grp = list(grp)
        b = DeviceBatch(mode, matrix(mat, A), gap, [encode(c["text"], A) for c in grp],
                        [encode(c["pattern"], A) for c in grp])
        res = b.run()
        for k, c in enumerate(grp):
            at, ap = b.alignment(k)
            assert same_result(dict(res[k], aligned_text=at, aligned_pattern=ap), c["result"]), (c["tag"], gap, mode)
        b.close()


@pytest.mark.parametrize("rows_per_lane", [1, 2, 4, 32])
def test_seeded_vs_oracle(eng, rows_per_lane):
    """Multi-strip hand-offs (pattern >> 64*R rows) on seeded DNA and protein pairs."""
    rng = np.random.default_rng(1000 + rows_per_lane)
    blast = synthetic.blast_matrix()
    for k in range(12):
        A = 4 if k % 3 else 23
        S = blast if A == 4 else matrix("blosum62", 23)
        n = int(rng.integers(500, 3000))
        m = int(rng.integers(64, n + 1))
        t = synthetic.random_sequence(int(rng.integers(1 << 30)), n, A)
        p = synthetic.mutate(t, k, A, m) if k % 2 else synthetic.random_sequence(k + 99, m, A)
        mode = k % 2
        gap = int(rng.choice([1, 5, 11]))
        exp = oracle.align(mode, t, p, S, gap)
        got = eng.align_pair(mode, t, p, S, gap, rows_per_lane=rows_per_lane)
        got.pop("fill_us")
        assert got == exp, (k, n, m, mode)


def _large_inputs(case):
    A = case["letters"]
    t = synthetic.random_sequence(case["text_seed"], case["n"], A)
    p = (synthetic.random_sequence(case["pattern_seed"], case["m"], A) if case["pattern_kind"] == "rand"
         else synthetic.mutate(t, case["pattern_seed"], A, case["m"]))
    S = matrix(case["matrix"], 4 if case["matrix"] == "blast" else 23)
    return t, p, S


def test_large_configs(eng, golden):
    """BASELINE.json configs 2-5 at their full sizes vs the reference's recorded outputs."""
    for case in golden["large.json"]:
        t, p, S = _large_inputs(case)
        got = eng.align_pair(case["mode"], t, p, S, case["gap"])
        assert same_result(got, case["result"]), case["name"]


def _score_of(at: str, ap: str, S: np.ndarray, gap: int, A: int) -> int:
    alpha = "ATCG" if A == 4 else "ARNDCQEGHILKMFPSTWYVBZX"
    lut = {c: i for i, c in enumerate(alpha)}
    s = 0
    for x, y in zip(at, ap):
        if x == "-" or y == "-":
            s -= gap
        else:
            s += int(S[lut[y], lut[x]])  # S[pattern][text]
    return s


def test_full_size_properties(eng):
    """Size-independent checks at the headline size: the alignment re-scores to the reported score,
    ungapped strings are the inputs (global) or substrings at the reported starts (local)."""
    S = synthetic.blast_matrix()
    n = m = 32768
    t = synthetic.random_sequence(21, n, 4)
    p = synthetic.mutate(t, 22, 4, m)
    alpha = np.array(list("ATCG"))
    for mode in (0, 1):
        got = eng.align_pair(mode, t, p, S, 5)
        at, ap = got["aligned_text"], got["aligned_pattern"]
        assert _score_of(at, ap, S, 5, 4) == got["score"]
        tu, pu = at.replace("-", ""), ap.replace("-", "")
        if mode == 0:
            assert tu == "".join(alpha[t]) and pu == "".join(alpha[p])
        else:
            # local starts are "first aligned index" or one less (reference quirk, traceBackSW :45-53)
            full_t, full_p = "".join(alpha[t]), "".join(alpha[p])
            assert tu in full_t and pu in full_p
            assert full_t.find(tu, max(0, got["start_text"] - 1)) in (got["start_text"], got["start_text"] + 1)


def test_batch_plan_config5(eng, golden):
    """Config 5 shape: many 2048^2 pairs in one plan; the recorded pairs match the reference."""
    from sa_amd.batch import DeviceBatch
    S = synthetic.blast_matrix()
    N = 256
    texts = [synthetic.random_sequence(1000 + 2 * i, 2048, 4) for i in range(N)]
    pats = [synthetic.random_sequence(1001 + 2 * i, 2048, 4) for i in range(N)]
    b = DeviceBatch(0, S, 5, texts, pats)
    res = b.run()
    recorded = {c["name"]: c for c in golden["large.json"] if c["name"].startswith("cfg5_batch_pair_")}
    for i in range(8):
        at, ap = b.alignment(i)
        assert same_result(dict(res[i], aligned_text=at, aligned_pattern=ap), recorded[f"cfg5_batch_pair_{i}"]["result"])
    for i in (17, 101, 255):  # a few more against the oracle
        at, ap = b.alignment(i)
        exp = oracle.align(0, texts[i], pats[i], S, 5)
        assert dict(res[i], aligned_text=at, aligned_pattern=ap) == exp
    # repeated fills reuse the plan (epoch-tagged hand-offs) and give identical results
    res2 = b.run()
    assert res2 == res
    b.close()


@pytest.mark.parametrize("gap", [5, 0, -3])
@pytest.mark.parametrize("rows_per_lane", [1, 2, 4, 8, 16, 32])
@pytest.mark.parametrize("mode", [0, 1])
def test_fill_direction_matrix_vs_oracle(eng, mode, rows_per_lane, gap):
    """The fill alone, cell by cell: the engine's DIRECTION matrix (decoded from its bit-planes) equals
    the reference's (m+1)x(n+1) byte matrix M (alignSequenceCPU.cpp:116-284) on every cell. Local
    plans with one row per lane store no STOP bit in their planes (the raw decisions); the decoder
    puts STOP back wherever H is 0 (:188-190), so every plan returns the reference's own M."""
    from sa_amd.batch import DeviceBatch
    S = synthetic.blast_matrix()
    for k, (n, m) in enumerate([(1500, 1400), (700, 700), (130, 66)]):
        t = synthetic.random_sequence(500 + k, n, 4)
        p = synthetic.mutate(t, 600 + k, 4, m)
        b = DeviceBatch(mode, S, gap, [t], [p], rows_per_lane=rows_per_lane)
        b.fill()
        got = b.directions(0)
        exp = np.empty((m + 1) * (n + 1), np.uint8)
        oracle.fill_only(mode, t, p, S, gap, exp)
        bad = int((got != exp).sum())
        b.close()
        assert bad == 0, (n, m, bad)


@pytest.mark.parametrize("rows_per_lane", [16, 32])
def test_pair_packed_fill_vs_oracle(eng, rows_per_lane):
    """The pair-packed fill (two equal-shape global pairs per wave in u16 halves, fill_pair_kernel):
    every pair's DIRECTION matrix, score and alignment equal the oracle's, cell by cell."""
    from sa_amd.batch import DeviceBatch
    S = synthetic.blast_matrix()
    n, m = 1500, 64 * rows_per_lane - 37
    texts, pats = [], []
    for k in range(4):
        t = synthetic.random_sequence(900 + k, n, 4)
        texts.append(t)
        pats.append(synthetic.mutate(t, 950 + k, 4, m) if k % 2 else synthetic.random_sequence(970 + k, m, 4))
    b = DeviceBatch(0, S, 5, texts, pats, rows_per_lane=rows_per_lane)
    res = b.run()
    for k in range(4):
        got = b.directions(k)
        exp = np.empty((m + 1) * (n + 1), np.uint8)
        oracle.fill_only(0, texts[k], pats[k], S, 5, exp)
        assert int((got != exp).sum()) == 0, k
        at, ap = b.alignment(k)
        assert dict(res[k], aligned_text=at, aligned_pattern=ap) == oracle.align(0, texts[k], pats[k], S, 5)
    b.close()


@pytest.mark.parametrize("rows_per_lane,n,m", [(8, 1500, 1100), (16, 1500, 1100), (8, 2100, 1024), (8, 100, 1300),
                                                (8, 700, 4000), (8, 700, 4200), (16, 3000, 2047), (4, 1500, 1100),
                                                (4, 2047, 2048), (4, 333, 2049), (4, 70, 900)])
def test_pair_packed_chain_vs_oracle(eng, rows_per_lane, n, m):
    """Pair-packed CHAINS (fill_pair_chain_kernel): a couple of equal-shape global pairs per workgroup,
    one wave per strip of both, each strip's bottom row handed to the strip below in LDS. Every
    pair's DIRECTION matrix, score and alignment equal the oracle's, cell by cell: several strips,
    a partial last strip, fewer columns than rows, exactly 8 strips (the most a chain takes) and 9
    (which falls back to the one-wave chained fill)."""
    from sa_amd.batch import DeviceBatch
    S = synthetic.blast_matrix()
    texts, pats = [], []
    for k in range(4):
        t = synthetic.random_sequence(2900 + k, n, 4)
        texts.append(t)
        pats.append(synthetic.mutate(t, 2950 + k, 4, m) if k % 2 else synthetic.random_sequence(2970 + k, m, 4))
    b = DeviceBatch(0, S, 5, texts, pats, rows_per_lane=rows_per_lane)
    strips = -(-m // (64 * rows_per_lane))
    assert b.plan.info()["fill_kernel"] == ("pair_chain" if strips <= 8 else "strips")
    res = b.run()
    for k in range(4):
        got = b.directions(k)
        exp = np.empty((m + 1) * (n + 1), np.uint8)
        oracle.fill_only(0, texts[k], pats[k], S, 5, exp)
        assert int((got != exp).sum()) == 0, k
        at, ap = b.alignment(k)
        assert dict(res[k], aligned_text=at, aligned_pattern=ap) == oracle.align(0, texts[k], pats[k], S, 5)
    b.close()


def test_very_long_reference_cases(eng):
    """The reference's "very long" cases (tests/tests.cu:553-597, commented out there for run time):
    qbpln50 (70020 x 66700 protein, gap 7) and AbHV_ORF111 (211518 x 202437 DNA, gap 5), global, vs
    the reference's own alignSequenceCPU outputs (tests/golden/make_long.py); plus the properties:
    the alignment re-scores to the score and the ungapped strings are the inputs."""
    import gzip
    import json
    import os
    from conftest import GOLDEN
    with gzip.open(os.path.join(GOLDEN, "long.json.gz"), "rt") as f:
        cases = json.load(f)
    for case in cases:
        A = case["A"]
        t, p = encode(case["text"], A), encode(case["pattern"], A)
        S = matrix(case["matrix"], A)
        got = eng.align_pair(case["mode"], t, p, S, case["gap"])
        assert same_result(got, case["result"]), case["name"]
        at, ap = got["aligned_text"], got["aligned_pattern"]
        assert _score_of(at, ap, S, case["gap"], A) == got["score"], case["name"]
        assert at.replace("-", "") == case["text"] and ap.replace("-", "") == case["pattern"], case["name"]


@pytest.mark.parametrize("mode", [0, 1])
def test_chain_ring_laps_across_groups(eng, mode):
    """Strip chains whose hand-off rings wrap one to three times (text > 2048 columns), in plans where
    the W-strip groups start at every strip offset of a pair (the first strip of a group is fed by the
    I/O wave, the others by their neighbour wave): every pair bit-exact, every cell of two pairs."""
    from sa_amd.batch import DeviceBatch
    S = synthetic.blast_matrix()
    shapes = [(2100, 300), (4200, 650), (6300, 450), (2049, 130), (3000, 200)]
    texts = [synthetic.random_sequence(1300 + k, n, 4) for k, (n, _) in enumerate(shapes)]
    pats = [synthetic.mutate(t, 1400 + k, 4, m) for k, (t, (_, m)) in enumerate(zip(texts, shapes))]
    b = DeviceBatch(mode, S, 5, texts, pats, rows_per_lane=1)
    b.fill()
    b.traceback()
    got = b.all_alignments()
    for k in range(len(shapes)):
        assert got[k] == oracle.align(mode, texts[k], pats[k], S, 5), (mode, shapes[k])
    for k in (1, 4):
        n, m = shapes[k]
        exp = np.empty((m + 1) * (n + 1), np.uint8)
        oracle.fill_only(mode, texts[k], pats[k], S, 5, exp)  # (the reference's M, STOP included)
        assert int((b.directions(k) != exp).sum()) == 0, shapes[k]
    b.close()


@pytest.mark.parametrize("gap", [0, 1, 5])
def test_local_best_cell_near_last_column(eng, gap):
    """Local strips with text profiles run no masked tail when g > 0 (sa_fill.hip process_strip): the
    cells past column n are garbage whose H stays below the pair's best. Cases where the best cell is
    in or next to the last column (the garbage right of it is as large as it gets), in every row
    position of a strip and at body / chunk boundaries of n, with g = 0 (masked tail) beside them."""
    S = synthetic.blast_matrix()
    for k, (n, m) in enumerate([(1000, 1000), (1001, 999), (1024, 1088), (1040, 1023), (2063, 2050),
                                (65, 130), (17, 127), (4097, 191)]):
        t = synthetic.random_sequence(1500 + k, n, 4)
        # the pattern ends with the text's last letters: the best local cell sits at column n
        tail = t[-min(n, m):]
        p = np.concatenate([synthetic.random_sequence(1600 + k, m - len(tail), 4), tail]).astype(np.int8)
        for pp in (p, p[: m - 3]):
            exp = oracle.align(1, t, pp, S, gap)
            got = eng.align_pair(1, t, pp, S, gap, rows_per_lane=1)
            got.pop("fill_us")
            assert got == exp, (n, len(pp), gap)


@pytest.mark.parametrize("mode", [0, 1])
def test_low_complexity_and_extreme_shapes(eng, mode):
    """Inputs whose direction matrices are all ties or long single-direction runs: homopolymers,
    period-4 repeats against a shifted copy, a 20000-column text against a 70-row pattern (LEFT runs
    thousands of columns long), a 9000-row pattern against a 300-column text (UP runs), and a text
    and pattern with no letter in common (local score 0). Every strip height the planner picks plus
    R = 1 and 32, bit-exact vs the oracle."""
    S = synthetic.blast_matrix()
    A, C, G, T = 0, 2, 3, 1  # "ATCG" codes
    rep = np.array([A, C, G, T], np.int8)
    cases = [
        (np.full(5000, A, np.int8), np.full(3000, A, np.int8)),
        (np.tile(rep, 1500), np.tile(np.roll(rep, 1), 1100)),
        (synthetic.random_sequence(1700, 20000, 4), synthetic.random_sequence(1701, 70, 4)),
        (synthetic.random_sequence(1702, 300, 4), synthetic.random_sequence(1703, 9000, 4)),
        (np.tile(np.array([A, T], np.int8), 2100), np.tile(np.array([C, G], np.int8), 1900)),
    ]
    for k, (t, p) in enumerate(cases):
        exp = oracle.align(mode, t, p, S, 5)
        for R in (0, 1, 32):
            got = eng.align_pair(mode, t, p, S, 5, rows_per_lane=R)
            got.pop("fill_us")
            assert got == exp, (k, len(t), len(p), R)


@pytest.mark.parametrize("rows_per_lane", [0, 16, 32])
def test_low_complexity_batch(eng, rows_per_lane):
    """The same all-tie and long-run inputs through one plan of equal-shape pairs (the pair-packed
    fill for global at R = 16/32, the batch column walk at R = 32): every pair bit-exact."""
    from sa_amd.batch import DeviceBatch
    S = synthetic.blast_matrix()
    rep = np.array([0, 2, 3, 1], np.int8)
    n, m = 2000, 1800
    texts = [np.full(n, 0, np.int8), np.tile(rep, n // 4), np.tile(rep, n // 4),
             np.tile(np.array([0, 1], np.int8), n // 2)]
    pats = [np.full(m, 0, np.int8), np.tile(np.roll(rep, 1), m // 4), np.full(m, 3, np.int8),
            np.tile(np.array([2, 3], np.int8), m // 2)]
    for mode in (0, 1):
        b = DeviceBatch(mode, S, 5, texts, pats, rows_per_lane=rows_per_lane)
        b.fill()
        b.traceback()
        got = b.all_alignments()
        b.close()
        for k in range(len(texts)):
            assert got[k] == oracle.align(mode, texts[k], pats[k], S, 5), (mode, k)
