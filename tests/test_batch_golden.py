"""BASELINE.json config 5 checked at its real size: every one of the 4096 batch pairs (and a 1024-pair
local batch) against the reference's own results (tests/golden/batch.json.gz, made by make_batch.py
from oracle/_ref/ref_align), as the reference's batch test compares every pair
(tests/tests.cu:463-551).

CPU: the fixture agrees with large.json and with the oracle on sampled pairs.
GPU: the exact plan bench.py --workload batch times (4096 pairs, one plan, pair-packed fill) checked
pair by pair (score, length, starts, hash of both strings); the local batch likewise; and the
sharded path (pair i -> rank i mod 2, sa_amd.distributed.gather_results) with the HIP engine on
device 0 in both ranks of a world-size-2 gloo group.
"""
from __future__ import annotations

import gzip
import hashlib
import json
import os
import socket

import pytest

from conftest import GOLDEN, ROOT

import oracle
from sa_amd import synthetic

_DOC = None


def fixture() -> dict:
    global _DOC
    if _DOC is None:
        with gzip.open(os.path.join(GOLDEN, "batch.json.gz"), "rt") as f:
            _DOC = json.load(f)
    return _DOC


def inputs(name: str, i: int):
    d = fixture()[name]
    L, base = fixture()["L"], d["seed_base"]
    t = synthetic.random_sequence(base + 2 * i, L, 4)
    if d["pattern"] == "rand":
        p = synthetic.random_sequence(base + 2 * i + 1, L, 4)
    else:
        p = synthetic.mutate(t, base + 2 * i + 1, 4, L)
    return t, p


def record(r: dict) -> list:
    h = hashlib.sha256((r["aligned_text"] + "\n" + r["aligned_pattern"]).encode()).hexdigest()[:24]
    return [r["score"], r["num_bytes"], r["start_text"], r["start_pattern"], h]


def test_fixture_matches_large_json_and_oracle(golden):
    doc = fixture()
    assert doc["global"]["pairs"] == 4096 and len(doc["global"]["records"]) == 4096
    assert doc["local"]["pairs"] == 1024 and len(doc["local"]["records"]) == 1024
    recorded = {c["name"]: c["result"] for c in golden["large.json"] if c["name"].startswith("cfg5_batch_pair_")}
    for i in range(8):
        r, rec = recorded[f"cfg5_batch_pair_{i}"], doc["global"]["records"][i]
        assert rec[:4] == [r["score"], r["num_bytes"], r["start_text"], r["start_pattern"]], i
    S = synthetic.blast_matrix()
    for name, idx in (("global", (0, 1234, 4095)), ("local", (0, 777, 1023))):
        for i in idx:
            t, p = inputs(name, i)
            got = oracle.align(doc[name]["mode"], t, p, S, doc["gap"])
            assert record(got) == doc[name]["records"][i], (name, i)


def _check_batch(name: str, count: int, every: int = 1, rows_per_lane: int = 0):
    """Pairs 0, every, 2 * every, ... below count * every (every = N: rank 0's shard of an N-rank deal)."""
    from sa_amd.batch import DeviceBatch
    doc = fixture()
    idx = list(range(0, count * every, every))
    pairs = [inputs(name, i) for i in idx]
    b = DeviceBatch(doc[name]["mode"], synthetic.blast_matrix(), doc["gap"], [t for t, _ in pairs],
                    [p for _, p in pairs], rows_per_lane=rows_per_lane)
    b.fill()
    b.traceback()
    got = b.all_alignments()
    info = b.plan.info()
    b.close()
    bad = [i for k, i in enumerate(idx) if record(got[k]) != doc[name]["records"][i]]
    assert not bad, f"{len(bad)} of {count} {name} pairs differ, first {bad[:5]}"
    return info


@pytest.mark.gpu
def test_config5_every_pair(eng):
    """The 4096-pair plan bench.py times, every pair bit-exact vs the reference."""
    info = _check_batch("global", 4096)
    assert info["num_strips"] == 4096 and info["rows_per_lane"] == 32


@pytest.mark.gpu
@pytest.mark.parametrize("shards", [2, 4, 8])
def test_config5_shard_every_pair(eng, shards):
    """Rank 0's shard of config 5 on an N-rank deal (pairs i = 0 mod N: 2048 / 1024 / 512 pairs), the
    plan bench.py --shard-of N times: the planner sizes it to the GPU (pair-packed chains of shorter
    strips once one strip per pair leaves SIMDs idle), every pair bit-exact vs the reference."""
    info = _check_batch("global", 4096 // shards, every=shards)
    assert info["fill_kernel"] in ("pair", "pair_chain") and info["rows_per_lane"] >= 4


@pytest.mark.gpu
@pytest.mark.parametrize("rows_per_lane", [4, 8, 16])
def test_config5_shard_of_8_chain_heights(eng, rows_per_lane):
    """The 512-pair shard with the pair-packed chains of every strip height the planner can pick
    (8 / 4 / 2 strips per pair), every pair bit-exact vs the reference."""
    info = _check_batch("global", 512, every=8, rows_per_lane=rows_per_lane)
    assert info["fill_kernel"] == "pair_chain" and info["rows_per_lane"] == rows_per_lane


@pytest.mark.gpu
def test_local_batch_every_pair(eng):
    _check_batch("local", 1024)


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _gpu_worker(rank, world, port, name, count, q, device_rows=False):
    import sys
    sys.path.insert(0, os.path.join(ROOT, "sequence-alignment-gpu_amd", "python"))
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist

    from sa_amd import distributed
    from sa_amd.batch import DeviceBatch
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    doc = fixture()
    mine = distributed.shard(count, world, rank)
    pairs = [inputs(name, i) for i in mine]
    b = DeviceBatch(doc[name]["mode"], synthetic.blast_matrix(), doc["gap"], [t for t, _ in pairs],
                    [p for _, p in pairs], device=0)
    b.fill()
    b.traceback()
    if device_rows:
        # the bench's batch path: sa_result rows device to device (sa_plan_copy_results) into a
        # ceil(count / world)-row buffer, gathered by distributed.gather_device (gloo: via the host)
        width = (count + world - 1) // world
        buf = torch.full((width, 4), -1, dtype=torch.int64, device="cuda:0")
        b.plan.copy_results(buf.data_ptr())
        torch.cuda.synchronize()
        out = distributed.gather_device(buf.cpu(), count, world, rank)
        b.close()
        q.put(("rank0" if rank == 0 else "rank1", out, []))
        dist.destroy_process_group()
        return
    res = b.all_alignments()
    b.close()
    # strings stay on the rank that made them (only the scalar fields travel): check them here
    bad_local = [i for i, r in zip(mine, res) if record(r)[4] != doc[name]["records"][i][4]]
    out = distributed.gather_results([{k: r[k] for k in distributed.FIELDS} for r in res], count, world, rank, "cpu")
    if rank == 0:
        q.put(("rank0", out, bad_local))
    else:
        q.put(("rank1", None, bad_local))
    dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.parametrize("name,count,device_rows", [("global", 512, False), ("local", 256, False),
                                                     ("global", 511, True), ("local", 255, True)])
def test_sharded_batch_hip_engine_world2(eng, name, count, device_rows):
    """Sharded batch path with the HIP engine behind it: two gloo ranks, both on device 0. With
    device_rows, the results travel as bench.py's batch sends them (sa_plan_copy_results rows, then
    distributed.gather_device; odd counts leave rank 1 one row short)."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gpu_worker, args=(r, 2, port, name, count, q, device_rows)) for r in range(2)]
    for p in procs:
        p.start()
    msgs = dict((tag, (out, bad)) for tag, out, bad in (q.get(timeout=150) for _ in range(2)))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert msgs["rank0"][1] == [] and msgs["rank1"][1] == []
    got = msgs["rank0"][0]
    if device_rows:  # (count, 4) int64 rows in FIELDS order
        got = [dict(zip(("score", "num_bytes", "start_text", "start_pattern"), map(int, r))) for r in got]
    exp = fixture()[name]["records"]
    bad = [i for i in range(count) if [got[i][k] for k in ("score", "num_bytes", "start_text", "start_pattern")] != exp[i][:4]]
    assert not bad, f"{len(bad)} pairs differ after the gather, first {bad[:5]}"
