"""Batches of independent pairs on one device: device-resident arenas (torch is only the allocator and
stream provider) + one sa_plan (include/sa_hip.h) = one fill launch and one traceback launch for all
pairs. Used by bench.py (config 5, multi-GPU sharding) and the GPU parity tests."""
from __future__ import annotations

import numpy as np


class DeviceBatch:
    def __init__(self, mode: int, S: np.ndarray, gap: int, texts: list[np.ndarray], patterns: list[np.ndarray],
                 device: int = 0, rows_per_lane: int = 0, alphabet: bytes | None = None):
        import torch

        from . import engine
        assert len(texts) == len(patterns)
        self.torch = torch
        self.device = device
        tl = np.array([len(t) for t in texts], dtype=np.int64)
        pl = np.array([len(p) for p in patterns], dtype=np.int64)
        to = np.concatenate([[0], np.cumsum(tl)[:-1]]) if len(tl) else tl
        po = np.concatenate([[0], np.cumsum(pl)[:-1]]) if len(pl) else pl
        ht = np.concatenate(texts).astype(np.int8) if texts else np.zeros(1, np.int8)
        hp = np.concatenate(patterns).astype(np.int8) if patterns else np.zeros(1, np.int8)
        dev = torch.device("cuda", device)
        self.d_text = torch.from_numpy(np.concatenate([ht, np.zeros(16, np.int8)])).to(dev)
        self.d_pattern = torch.from_numpy(np.concatenate([hp, np.zeros(16, np.int8)])).to(dev)
        self.pairs = [(int(a), int(b), int(c), int(d)) for a, b, c, d in zip(to, tl, po, pl)]
        self.plan = engine.Plan(mode, S, gap, self.pairs, device=device, alphabet=alphabet,
                                rows_per_lane=rows_per_lane)
        torch.cuda.synchronize(dev)

    def stream(self) -> int:
        return self.torch.cuda.current_stream(self.device).cuda_stream

    def fill(self) -> None:
        self.plan.fill(self.d_text.data_ptr(), self.d_pattern.data_ptr(), self.stream())

    def traceback(self) -> None:
        self.plan.traceback(self.stream())

    def run(self) -> list[dict]:
        self.fill()
        self.traceback()
        return self.plan.results(self.stream())

    def results(self) -> list[dict]:
        return self.plan.results(self.stream())

    def all_alignments(self) -> list[dict]:
        return self.plan.all_alignments(self.stream())

    def alignment(self, i: int) -> tuple[str, str]:
        return self.plan.alignment(i, self.stream())

    def directions(self, i: int):
        return self.plan.directions(i, self.stream())

    def close(self) -> None:
        self.plan.close()
