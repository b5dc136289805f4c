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


def gather_results(results: list[dict], num_pairs: int, world: int, rank: int, device) -> list[dict] | None:
    """Gathers every rank's per-pair results to rank 0 in global pair order; None on other ranks."""
    import torch
    import torch.distributed as dist

    width = (num_pairs + world - 1) // world
    buf = torch.full((width, len(FIELDS)), -1, dtype=torch.int64, device=device)
    if results:
        to_i64 = lambda v: int(v) - (1 << 64) if int(v) >= (1 << 63) else int(v)  # uint64 starts, e.g. (uint64)-1
        vals = [[to_i64(r[f]) for f in FIELDS] for r in results]
        buf[: len(results)] = torch.tensor(vals, dtype=torch.int64, device=device)
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
