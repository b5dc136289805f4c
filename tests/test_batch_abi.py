"""The native multi-device batch entry point (include/sa_hip.h: sa_align_batch, sa_batch_deal; the C++
extension SequenceAlignment::alignSequenceGPUBatch).

CPU: the deal — round-robin for equal work (the same pair -> shard map as the torch path's
sa_amd.distributed.shard), longest-processing-time otherwise (balanced, deterministic, complete).
GPU: sa_align_batch against the reference's recorded batch (tests/golden/batch.json.gz) with one
device, and with several shards sharing device 0 (the threads / deal / reassembly path without
RCCL); the C++ batch call against per-request alignSequenceCPU through bin/sa_api_check.
"""
from __future__ import annotations

import json
import os
import subprocess

import numpy as np
import pytest

from conftest import PKG
from sa_amd import distributed, engine, synthetic
from test_batch_golden import fixture, inputs, record


@pytest.mark.parametrize("num,shards", [(1, 1), (7, 3), (4096, 8), (13, 2), (5, 8)])
def test_deal_equal_work_is_round_robin(num, shards):
    got = engine.batch_deal([2048 * 2048] * num, shards)
    for s in range(shards):
        assert [i for i, x in enumerate(got) if x == s] == distributed.shard(num, shards, s)


def test_deal_unequal_work_is_lpt_balanced():
    rng = np.random.default_rng(5)
    cells = (rng.integers(1, 40, 257) * 1000).tolist()
    for shards in (2, 3, 8):
        got = engine.batch_deal(cells, shards)
        assert got == engine.batch_deal(cells, shards)  # deterministic
        assert sorted(set(got)) == list(range(shards))
        load = [sum(c for c, s in zip(cells, got) if s == k) for k in range(shards)]
        # LPT bound: no shard exceeds the average by more than the largest single pair
        assert max(load) <= sum(cells) / shards + max(cells)
    # the largest pair goes first, to shard 0
    assert engine.batch_deal([1, 9, 3, 9, 2, 7], 2) == [1, 0, 1, 1, 1, 0]


def test_deal_rejects_bad_arguments():
    with pytest.raises(engine.SaError):
        engine.batch_deal([1, 2], 0)


@pytest.mark.gpu
@pytest.mark.parametrize("name,count,gpus", [("global", 512, 1), ("local", 300, 3), ("global", 101, 4)])
def test_align_batch_vs_reference(eng, name, count, gpus):
    doc = fixture()
    pairs = [inputs(name, i) for i in range(count)]
    got = engine.align_batch(doc[name]["mode"], [t for t, _ in pairs], [p for _, p in pairs],
                             synthetic.blast_matrix(), doc["gap"], num_gpus=gpus)
    bad = [i for i in range(count) if record(got[i]) != doc[name]["records"][i]]
    assert not bad, f"{len(bad)} of {count} pairs differ, first {bad[:5]}"


@pytest.mark.gpu
def test_align_batch_mixed_sizes_vs_oracle(eng):
    import oracle
    S = synthetic.blast_matrix()
    lens = [(0, 5), (7, 0), (0, 0), (300, 290), (1, 1), (2000, 1500), (65, 64), (129, 700)]
    ts = [synthetic.random_sequence(70 + k, n, 4) for k, (n, _) in enumerate(lens)]
    ps = [synthetic.mutate(t, 90 + k, 4, m) if len(t) and m else synthetic.random_sequence(90 + k, m, 4)
          for k, (t, (_, m)) in enumerate(zip(ts, lens))]
    for mode in (0, 1):
        got = engine.align_batch(mode, ts, ps, S, 5, num_gpus=2)
        for k in range(len(lens)):
            assert got[k] == oracle.align(mode, ts[k], ps[k], S, 5), (mode, lens[k])


@pytest.mark.gpu
def test_cpp_batch_api_vs_cpu(eng):
    """SequenceAlignment::alignSequenceGPUBatch vs alignSequenceCPU on the same Requests (C++14 caller)."""
    exe = os.path.join(PKG, "bin", "sa_api_check")
    for args in (["global", "64", "3000", "2"], ["local", "48", "2500", "3"]):
        out = subprocess.run([exe, *args], capture_output=True, text=True, timeout=300)
        assert out.returncode == 0, out.stdout + out.stderr
        res = json.loads(out.stdout.strip().splitlines()[-1])
        assert res["mismatches"] == 0 and res["requests"] == int(args[1]), res


@pytest.mark.gpu
def test_align_batch_repeated_calls_reuse_and_rebuild(eng):
    """sa_align_batch keeps each shard's arenas and plan across calls: the same shapes with new
    letters (plan reused: the results must follow the new inputs), then other shapes and another
    gap (plans rebuilt), then the first batch again, each against the oracle."""
    import oracle
    S = synthetic.blast_matrix()

    def batch(seed, n, m, k):
        ts = [synthetic.random_sequence(seed + 2 * i, n + 3 * i, 4) for i in range(k)]
        ps = [synthetic.mutate(t, seed + 2 * i + 1, 4, m + i) for i, t in enumerate(ts)]
        return ts, ps

    calls = [(batch(500, 400, 380, 6), 5), (batch(600, 400, 380, 6), 5), (batch(700, 900, 700, 5), 3),
             (batch(500, 400, 380, 6), 5)]
    for (ts, ps), gap in calls:
        for mode in (0, 1):
            got = engine.align_batch(mode, ts, ps, S, gap, num_gpus=2)
            for k in range(len(ts)):
                assert got[k] == oracle.align(mode, ts[k], ps[k], S, gap), (mode, gap, k)
