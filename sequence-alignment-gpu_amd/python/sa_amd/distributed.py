"""Batch sharding across GPUs (BASELINE.json config 5).

Independent pairs are dealt round-robin, pair i -> rank i mod world (equal-size pairs make this
balanced). The only data-path exchange is the per-pair result gather to rank 0 — score, length and
starts, 4 int64 per pair (128 KiB for 4096 pairs) — done with torch.distributed.gather, i.e. RCCL
over xGMI on the GPU backend ('nccl') and gloo in the CPU tests.
"""
from __future__ import annotations

FIELDS = ("score", "num_bytes", "start_text", "start_pattern")


def shard(num_pairs: int, world: int, rank: int) -> list[int]:
    return list(range(rank, num_pairs, world))


def _as_rows(results) -> "np.ndarray":
    """(k, 4) int64 rows of FIELDS from a list of result dicts or a numpy structured array
    (engine.RESULT_DTYPE); uint64 starts such as (uint64)-1 keep their bits."""
    import numpy as np
    if isinstance(results, np.ndarray):
        return np.stack([results[f].astype(np.uint64).view(np.int64) for f in FIELDS], axis=1) if len(results) \
            else np.zeros((0, len(FIELDS)), np.int64)
    to_i64 = lambda v: int(v) - (1 << 64) if int(v) >= (1 << 63) else int(v)
    return np.array([[to_i64(r[f]) for f in FIELDS] for r in results], dtype=np.int64).reshape(-1, len(FIELDS))


def gather_array(results, num_pairs: int, world: int, rank: int, device):
    """Gathers every rank's per-pair result rows to rank 0: an (num_pairs, 4) int64 array of FIELDS in
    global pair order on rank 0 (uint64 starts as their int64 bit patterns), None elsewhere."""
    import numpy as np
    import torch
    import torch.distributed as dist

    width = (num_pairs + world - 1) // world
    rows = _as_rows(results)
    buf = torch.full((width, len(FIELDS)), -1, dtype=torch.int64, device=device)
    if len(rows):
        buf[: len(rows)] = torch.from_numpy(rows).to(device)
    parts = [torch.empty_like(buf) for _ in range(world)] if rank == 0 else None
    dist.gather(buf, parts, dst=0)
    if rank != 0:
        return None
    out = np.empty((num_pairs, len(FIELDS)), np.int64)
    for r, part in enumerate(parts):
        idx = shard(num_pairs, world, r)
        out[idx] = part.cpu().numpy()[: len(idx)]
    return out


def gather_device(buf, num_pairs: int, world: int, rank: int):
    """Gathers every rank's sa_result rows, already in a (width, 4) int64 tensor on the rank's device
    (Plan.copy_results: bit copies of sa_result, so column 0 is score | status << 32), to rank 0 with
    one collective and no host round trip before it; rank 0 brings the gathered block to the host in
    one copy and raises RuntimeError if any pair's status is not SA_OK. Returns the (num_pairs, 4) int64 FIELDS array in global pair order on rank 0, None
    elsewhere (as gather_array)."""
    import numpy as np
    import torch
    import torch.distributed as dist

    if buf.is_cuda and dist.get_backend() == "gloo":
        buf = buf.cpu()  # (gloo gathers host tensors: the tests' one-GPU, several-rank runs)
    parts = [torch.empty_like(buf) for _ in range(world)] if rank == 0 else None
    dist.gather(buf, parts, dst=0)
    if rank != 0:
        return None
    allp = torch.stack(parts).cpu().numpy()
    out = np.empty((num_pairs, len(FIELDS)), np.int64)
    for r in range(world):
        idx = shard(num_pairs, world, r)
        rows = allp[r, : len(idx)]
        # sa_result.status (bits 32..63 of word 0): the expand kernel writes the fill's abort / bad-input
        # state into every pair, so a failed pair on any rank fails the gather here instead of reaching
        # rank 0 as a score
        status = (rows[:, 0] >> 32) & 0xFFFFFFFF
        if status.any():
            bad = int(np.flatnonzero(status)[0])
            raise RuntimeError(f"gather_device: rank {r} pair {idx[bad]} has status {int(status[bad])} "
                               f"({int(np.count_nonzero(status))} of {len(idx)} pairs of that rank failed)")
        score = rows[:, 0] & 0xFFFFFFFF
        out[idx, 0] = np.where(score >= 1 << 31, score - (1 << 32), score)
        out[idx, 1:] = rows[:, 1:]
    return out


def gather_results(results, num_pairs: int, world: int, rank: int, device) -> list[dict] | None:
    """Gathers every rank's per-pair results to rank 0 in global pair order; None on other ranks."""
    import torch
    import torch.distributed as dist

    width = (num_pairs + world - 1) // world
    buf = torch.full((width, len(FIELDS)), -1, dtype=torch.int64, device=device)
    rows = _as_rows(results)
    if len(rows):
        buf[: len(rows)] = torch.from_numpy(rows).to(device)
    parts = [torch.empty_like(buf) for _ in range(world)] if rank == 0 else None
    dist.gather(buf, parts, dst=0)
    if rank != 0:
        return None
    out: list[dict | None] = [None] * num_pairs
    for r, part in enumerate(parts):
        rows = part.cpu().tolist()
        for k, i in enumerate(shard(num_pairs, world, r)):
            rec = dict(zip(FIELDS, rows[k]))
            for f in ("start_text", "start_pattern"):
                rec[f] &= (1 << 64) - 1  # back to the uint64 the ABI returns (e.g. (uint64)-1)
            out[i] = rec
    return out  # type: ignore[return-value]
