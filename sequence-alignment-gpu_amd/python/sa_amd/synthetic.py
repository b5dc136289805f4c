"""Deterministic synthetic inputs for the benchmark configs.

* ``random_sequence(seed, n, A)``: i.i.d. letters ``(splitmix64_k >> 33) % A`` where splitmix64_k is
  the k-th output of a splitmix64 stream seeded with ``seed`` (k = 1, 2, ...). The same stream is
  implemented in C in ``oracle/ref_driver.cpp`` (``fillbench``) so both sides see identical inputs.
* ``mutate(seq, seed, A, length)``: a vectorised restatement of the reference's ``mutate.py:4-59``
  mutation model — per source letter 5 % deletion, else 2 % replacement by a random letter (the
  reference's "insertion" branch emits a random letter in place of the source letter,
  ``mutate.py:50-52``), else 5 % substitution by a different letter — then trimmed / padded with
  random letters to ``length``. Draws come from splitmix64 (4 per source letter), not Python's
  ``random``, so results are reproducible across hosts.
"""
from __future__ import annotations

import numpy as np

GOLDEN = np.uint64(0x9E3779B97F4A7C15)
_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)


def splitmix64(seed: int, count: int, offset: int = 0) -> np.ndarray:
    """Outputs k = offset+1 .. offset+count of a splitmix64 stream (uint64 array)."""
    with np.errstate(over="ignore"):
        k = np.arange(offset + 1, offset + count + 1, dtype=np.uint64)
        z = np.uint64(seed) + k * GOLDEN
        z = (z ^ (z >> np.uint64(30))) * _M1
        z = (z ^ (z >> np.uint64(27))) * _M2
        return z ^ (z >> np.uint64(31))


def random_sequence(seed: int, n: int, A: int = 4) -> np.ndarray:
    """Alphabet-index sequence (int8) of length n."""
    return ((splitmix64(seed, n) >> np.uint64(33)) % np.uint64(A)).astype(np.int8)


def _uniform(seed: int, count: int, offset: int = 0) -> np.ndarray:
    return (splitmix64(seed, count, offset) >> np.uint64(11)).astype(np.float64) * (1.0 / 9007199254740992.0)


def mutate(seq: np.ndarray, seed: int, A: int = 4, length: int | None = None,
           p_del: float = 0.05, p_ins: float = 0.02, p_sub: float = 0.05) -> np.ndarray:
    seq = np.asarray(seq, dtype=np.int64)
    n = len(seq)
    u = _uniform(seed, 4 * n).reshape(n, 4) if n else np.zeros((0, 4))
    dele = u[:, 0] < p_del
    ins = ~dele & (u[:, 1] < p_ins)
    sub = ~dele & ~ins & (u[:, 2] < p_sub)
    out = seq.copy()
    out[ins] = np.minimum((u[ins, 3] * A).astype(np.int64), A - 1)
    shift = 1 + np.minimum((u[sub, 3] * (A - 1)).astype(np.int64), A - 2)
    out[sub] = (seq[sub] + shift) % A
    out = out[~dele]
    if length is not None:
        if len(out) >= length:
            out = out[:length]
        else:
            pad = random_sequence(seed ^ 0x5EED, length - len(out), A).astype(np.int64)
            out = np.concatenate([out, pad])
    return out.astype(np.int8)


def blast_matrix() -> np.ndarray:
    """scoreMatrices/dna/blast.txt of the reference: +5 match / -4 mismatch (4x4, row-major)."""
    S = np.full((4, 4), -4, dtype=np.int32)
    np.fill_diagonal(S, 5)
    return S
