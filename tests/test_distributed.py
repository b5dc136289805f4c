"""CPU, world_size 2 over gloo: the batch path's sharding (pair i -> rank i mod world) and the
result gather to rank 0 (sa_amd.distributed) reassemble exactly the single-process results. The
per-pair computation here is the oracle (CPU test stand-in for the GPU engine; the GPU path of the
same gather is exercised by bench.py --workload batch on the box)."""
from __future__ import annotations

import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from conftest import ROOT


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _pairs(num):
    import sys
    sys.path.insert(0, os.path.join(ROOT, "sequence-alignment-gpu_amd", "python"))
    from sa_amd import synthetic
    out = []
    for i in range(num):
        t = synthetic.random_sequence(1000 + 2 * i, 96 + 7 * i, 4)
        p = synthetic.random_sequence(1001 + 2 * i, 80 + 5 * i, 4)
        out.append((t, p))
    return out


def _worker(rank, world, port, num, mode, q):
    import sys
    sys.path.insert(0, os.path.join(ROOT, "sequence-alignment-gpu_amd", "python"))
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import torch.distributed as dist

    import oracle
    from sa_amd import distributed, synthetic
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    pairs = _pairs(num)
    S = synthetic.blast_matrix()
    mine = distributed.shard(num, world, rank)
    res = []
    for i in mine:
        r = oracle.align(mode, pairs[i][0], pairs[i][1], S, 5)
        res.append({k: r[k] for k in distributed.FIELDS})
    out = distributed.gather_results(res, num, world, rank, "cpu")
    if rank == 0:
        q.put(out)
    dist.destroy_process_group()


@pytest.mark.parametrize("mode", [0, 1])
def test_sharded_batch_gather_world2(mode):
    num = 13  # uneven split on purpose
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, num, mode, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    import sys
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    from sa_amd import distributed, synthetic
    S = synthetic.blast_matrix()
    pairs = _pairs(num)
    for i in range(num):
        r = oracle.align(mode, pairs[i][0], pairs[i][1], S, 5)
        assert got[i] == {k: r[k] for k in distributed.FIELDS}, i
    # the deal is round-robin and covers every pair exactly once
    assert sorted(distributed.shard(num, 2, 0) + distributed.shard(num, 2, 1)) == list(range(num))


def _array_worker(rank, world, port, num, q):
    import sys
    sys.path.insert(0, os.path.join(ROOT, "sequence-alignment-gpu_amd", "python"))
    import numpy as np
    import torch.distributed as dist

    from sa_amd import distributed
    from sa_amd.engine import RESULT_DTYPE
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    mine = distributed.shard(num, world, rank)
    arr = np.zeros(len(mine), RESULT_DTYPE)
    arr["score"] = [10 * i - 7 for i in mine]
    arr["num_bytes"] = [i + 3 for i in mine]
    arr["start_text"] = [(1 << 64) - 1 if i % 3 == 0 else i for i in mine]
    arr["start_pattern"] = [i * 5 for i in mine]
    out = distributed.gather_array(arr, num, world, rank, "cpu")
    if rank == 0:
        q.put(out)
    dist.destroy_process_group()


def test_gather_array_world2():
    """The bench's vectorized result path: structured sa_result arrays -> rank 0, uint64 bits kept."""
    import numpy as np
    num = 11
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_array_worker, args=(r, 2, port, num, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert got.shape == (num, 4)
    for i in range(num):
        st = -1 if i % 3 == 0 else i  # (uint64)-1 as its int64 bit pattern
        assert got[i].tolist() == [10 * i - 7, i + 3, st, i * 5], i
    assert np.uint64(got[0, 2].view(np.uint64)) == np.uint64((1 << 64) - 1)


def _device_worker(rank, world, port, num, q, bad_pair=-1):
    import sys
    sys.path.insert(0, os.path.join(ROOT, "sequence-alignment-gpu_amd", "python"))
    import numpy as np
    import torch
    import torch.distributed as dist

    from sa_amd import distributed
    from sa_amd.engine import RESULT_DTYPE
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    mine = distributed.shard(num, world, rank)
    arr = np.zeros(len(mine), RESULT_DTYPE)
    arr["score"] = [10 * i - 7 for i in mine]
    arr["status"] = [5 if i == bad_pair else 0 for i in mine]  # SA_ERR_TIMEOUT on the injected pair
    arr["num_bytes"] = [i + 3 for i in mine]
    arr["start_text"] = [(1 << 64) - 1 if i % 3 == 0 else i for i in mine]
    arr["start_pattern"] = [i * 5 for i in mine]
    # what Plan.copy_results leaves in the bench's gather buffer: raw sa_result bytes, (width, 4) int64
    buf = torch.full(((num + world - 1) // world, 4), -1, dtype=torch.int64)
    buf[: len(mine)] = torch.from_numpy(arr.view(np.int64).reshape(len(mine), 4).copy())
    try:
        out = distributed.gather_device(buf, num, world, rank)
    except RuntimeError as e:
        out = f"raised: {e}"
    if rank == 0:
        q.put(out)
    dist.destroy_process_group()


def test_gather_device_world2():
    """The bench's device-resident result path: raw sa_result rows (Plan.copy_results) -> rank 0 in
    one gather; score is the low int32 of the first word, uint64 starts keep their bits."""
    num = 11
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_device_worker, args=(r, 2, port, num, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert got.shape == (num, 4)
    for i in range(num):
        st = -1 if i % 3 == 0 else i
        assert got[i].tolist() == [10 * i - 7, i + 3, st, i * 5], i


def test_gather_device_status_fails_loudly():
    """A pair whose sa_result.status is not SA_OK on rank 1 (here SA_ERR_TIMEOUT, what the expand kernel
    writes after a hand-off timeout) makes rank 0's gather raise instead of returning its score."""
    num = 11
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_device_worker, args=(r, 2, port, num, q, 7)) for r in range(2)]
    for p in procs:
        p.start()
    got = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert isinstance(got, str) and got.startswith("raised:"), got
    assert "rank 1 pair 7 has status 5" in got, got


def test_bench_launches_ranks_dry_run():
    """`bench.py --gpus 2` without WORLD_SIZE starts its own two ranks (torch.distributed.run) and the
    rank-0 line reports n_gpus 2 (--dry-run: gloo, no GPU work)."""
    import json
    import subprocess
    import sys
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "3", "--warmup", "1",
                          "--dry-run"], env=env, capture_output=True, text=True, timeout=180)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [json.loads(l) for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout
    assert lines[0]["n_gpus"] == 2 and lines[0]["ranks_seen"] == 2 and lines[0]["steps"] == 3


def test_bench_refuses_world_size_mismatch():
    """WORLD_SIZE (set by a launcher) must equal --gpus: a silent one-GPU line for --gpus 8 is refused."""
    import subprocess
    import sys
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "1", "--dry-run"], env=env,
                         capture_output=True, text=True, timeout=120)
    assert out.returncode != 0 and "WORLD_SIZE" in out.stderr


@pytest.mark.gpu
@pytest.mark.parametrize("workload,pair0", [("batch", 1408), ("dna8k", None)])
def test_bench_two_ranks_on_one_gpu(workload, pair0):
    """The N-rank bench path for real, on a one-GPU box: `bench.py --gpus 2` launches two ranks, both
    on device 0 with the gloo backend (SA_BENCH_ONE_DEVICE; RCCL needs a device per rank). The batch
    deals pairs i mod 2, pipelines each rank's steps two deep and gathers every step's results to rank
    0 on the traceback stream; the line reports both ranks' pairs (4096), and pair 0's score is the
    reference's (tests/golden/batch.json.gz). RCCL across devices is what this cannot cover."""
    import json
    import subprocess
    import sys
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env["SA_BENCH_ONE_DEVICE"] = "1"
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--workload", workload,
                          "--steps", "3", "--warmup", "1", "--no-cpu-baseline"], env=env, capture_output=True, text=True,
                         timeout=170)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [json.loads(l) for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout
    d = lines[0]
    assert d["n_gpus"] == 2 and d["steps"] == 3 and d["value"] > 0, d
    if workload == "batch":
        assert d["sample_result"]["pairs_per_gpu"] == 2048 and d["sample_result"]["pair0_score"] == pair0, d
        assert d["config"]["step_overlap"].startswith("two-deep"), d
