"""Empty texts and patterns, both modes, DNA and protein (tests/golden/edge_pairs.json, from the
reference's own alignSequenceCPU where the pair is inside its contract, text >= pattern; from the
oracle otherwise), and out-of-alphabet input bytes.

CPU: the oracle reproduces every record. GPU: one-shot at several strip heights, one plan mixing
empty and non-empty pairs, sa_align_batch over two shards; a plan whose arena holds a byte outside
0..A-1 reports SA_ERR_INVALID instead of a silently clamped alignment, and so does the one-shot
path (flagged on the device by its encode kernel; there is no host scan of the inputs).
"""
from __future__ import annotations

import numpy as np
import pytest

import oracle
from conftest import encode, load, matrix, same_result
from sa_amd import synthetic


def _cases():
    return load("edge_pairs.json")


def _inputs(c):
    return encode(c["text"], c["A"]), encode(c["pattern"], c["A"]), matrix(c["matrix"], c["A"])


def test_oracle_edge_pairs():
    for c in _cases():
        t, p, S = _inputs(c)
        assert same_result(oracle.align(c["mode"], t, p, S, c["gap"]), c["result"]), (c["mode"], len(t), len(p))


@pytest.mark.gpu
@pytest.mark.parametrize("rows_per_lane", [0, 1, 2, 32])
def test_edge_pairs_one_shot(eng, rows_per_lane):
    for c in _cases():
        t, p, S = _inputs(c)
        got = eng.align_pair(c["mode"], t, p, S, c["gap"], rows_per_lane=rows_per_lane)
        assert same_result(got, c["result"]), (c["mode"], c["A"], len(t), len(p))


@pytest.mark.gpu
def test_edge_pairs_mixed_plan_and_batch(eng):
    from sa_amd.batch import DeviceBatch
    for mode in (0, 1):
        for A in (4, 23):
            edge = [c for c in _cases() if c["mode"] == mode and c["A"] == A]
            S = matrix(edge[0]["matrix"], A)
            letters = 20 if A == 23 else 4
            # empty pairs interleaved with ordinary multi-strip ones
            extra = [(synthetic.random_sequence(900 + k, 150 + 97 * k, letters),
                      synthetic.random_sequence(950 + k, 140 + 61 * k, letters)) for k in range(len(edge))]
            texts, pats, exp = [], [], []
            for c, (t2, p2) in zip(edge, extra):
                t, p, _ = _inputs(c)
                texts += [t, t2]
                pats += [p, p2]
                exp += [c["result"], oracle.align(mode, t2, p2, S, c["gap"])]
            b = DeviceBatch(mode, S, edge[0]["gap"], texts, pats,
                            alphabet=None if A == 4 else b"ARNDCQEGHILKMFPSTWYVBZX-")
            b.fill()
            b.traceback()
            got = b.all_alignments()
            b.close()
            for k, (g, e) in enumerate(zip(got, exp)):
                assert same_result(g, e), (mode, A, k)
            got2 = eng.align_batch(mode, texts, pats, S, edge[0]["gap"], num_gpus=2,
                                   alphabet=None if A == 4 else b"ARNDCQEGHILKMFPSTWYVBZX-")
            for k, (g, e) in enumerate(zip(got2, exp)):
                assert same_result(g, e), ("align_batch", mode, A, k)


@pytest.mark.gpu
@pytest.mark.parametrize("where", ["text", "pattern"])
def test_out_of_alphabet_bytes_are_rejected(eng, where):
    from sa_amd.batch import DeviceBatch
    S = synthetic.blast_matrix()
    t = synthetic.random_sequence(5, 300, 4)
    p = synthetic.random_sequence(6, 200, 4)
    (t if where == "text" else p)[17] = 4  # one byte past the DNA alphabet
    with pytest.raises(eng.SaError):
        eng.align_pair(0, t, p, S, 5)  # the one-shot path's encode kernel flags it (ctrl.bad_input)
    b = DeviceBatch(0, S, 5, [synthetic.random_sequence(7, 100, 4), t], [synthetic.random_sequence(8, 90, 4), p])
    b.fill()
    b.traceback()
    with pytest.raises(eng.SaError) as ei:
        b.results()
    assert ei.value.code == 1  # SA_ERR_INVALID
    b.close()
