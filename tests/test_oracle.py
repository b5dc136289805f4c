"""CPU: the oracle (oracle/sa_oracle.c) against every golden record produced by the reference itself
(tests/golden/make_golden.py) and the reference's own known answers (tests/tests.cu:116-366)."""
from __future__ import annotations

import numpy as np
import pytest

import oracle
from conftest import encode, matrix, same_result
from sa_amd import synthetic


def _run(case, A_key="A"):
    A = case[A_key]
    return oracle.align(case["mode"], encode(case["text"], A), encode(case["pattern"], A), matrix(case["matrix"], A),
                        case["gap"])


def test_known_answers(golden):
    for case in golden["known_answers.json"]:
        got = _run(case)
        assert same_result(got, case["result"]), case["name"]
        if case["expect_score"] is not None:   # hard-coded expectation of tests.cu
            assert got["score"] == case["expect_score"], case["name"]
        if case["expect_strings"]:
            assert (got["aligned_text"], got["aligned_pattern"]) == tuple(case["expect_strings"]), case["name"]
        if case["expect_starts"]:
            assert (got["start_text"], got["start_pattern"]) == tuple(case["expect_starts"]), case["name"]


def test_data_pairs(golden):
    d = golden["data_pairs.json"]
    seqs = d["sequences"]
    for case in d["cases"]:
        A = case["A"]
        got = oracle.align(case["mode"], encode(seqs[case["text"]], A), encode(seqs[case["pattern"]], A),
                           matrix(case["matrix"], A), case["gap"])
        assert same_result(got, case["result"]), (case["text"], case["pattern"], case["mode"])


def test_random_pairs(golden):
    for k, case in enumerate(golden["random_pairs.json"]):
        assert same_result(_run(case), case["result"]), (k, case["tag"])


def test_gap_pairs():
    """Gap penalties 0, -1, -2, -5 (tests/golden/make_gaps.py, from the reference)."""
    from conftest import load
    for k, case in enumerate(load("gap_pairs.json")):
        assert same_result(_run(case), case["result"]), (k, case["tag"], case["gap"])


@pytest.mark.parametrize("name", ["cfg2_dna_global_8192_uniform", "cfg2_dna_global_8192_mutated",
                                  "cfg4_protein_global_4096_blosum50", "cfg4_protein_local_4096_blosum50",
                                  "cfg5_batch_pair_0"])
def test_large(golden, name):
    case = next(c for c in golden["large.json"] if c["name"] == name)
    A = case["letters"]
    t = synthetic.random_sequence(case["text_seed"], case["n"], A)
    p = (synthetic.random_sequence(case["pattern_seed"], case["m"], A) if case["pattern_kind"] == "rand"
         else synthetic.mutate(t, case["pattern_seed"], A, case["m"]))
    S = matrix(case["matrix"], 4 if case["matrix"] == "blast" else 23)
    got = oracle.align(case["mode"], t, p, S, case["gap"])
    assert same_result(got, case["result"])


def test_oracle_matches_reference_binary_on_fresh_inputs():
    """When the reference build is present (this container), pin the restatement on fresh inputs."""
    if not oracle.ref_available():
        pytest.skip("oracle/_ref not built")
    rng = np.random.default_rng(7)
    S = synthetic.blast_matrix()
    jobs = []
    for k in range(200):
        n = int(rng.integers(1, 400))
        m = int(rng.integers(1, n + 1))
        t = rng.integers(0, 4, n).astype(np.int8)
        p = synthetic.mutate(t, k, 4, m) if k % 2 else rng.integers(0, 4, m).astype(np.int8)
        jobs.append((k % 2, t, p, S, int(rng.integers(-6, 12))))
    for job, r in zip(jobs, oracle.ref_align_batch(jobs)):
        assert oracle.align(*job) == r


def test_oracle_local_raw_decisions():
    """(CPU) oracle mode 2 (the engine's rows_per_lane 1 local planes): every interior cell holds the
    reference's decision before its STOP override (alignSequenceCPU.cpp:181-189), so it equals mode 1
    wherever mode 1 is not STOP, and the border rows stay STOP."""
    import numpy as np
    from sa_amd import synthetic
    S = synthetic.blast_matrix()
    t = synthetic.random_sequence(11, 300, 4)
    p = synthetic.mutate(t, 12, 4, 280)
    n, m = len(t), len(p)
    loc = np.empty((m + 1) * (n + 1), np.uint8)
    raw = np.empty_like(loc)
    oracle.fill_only(1, t, p, S, 5, loc)
    oracle.fill_only(2, t, p, S, 5, raw)
    loc, raw = loc.reshape(m + 1, n + 1), raw.reshape(m + 1, n + 1)
    keep = loc != 3
    assert (raw[keep] == loc[keep]).all()
    assert (raw[1:, 1:] != 3).all() and (raw[0] == 3).all() and (raw[:, 0] == 3).all()
    assert (loc[1:, 1:] == 3).any()  # the case has STOP cells
