"""Shared test setup.

Markers: ``gpu`` — needs an MI355X (run on the GPU box with ``-m gpu``); everything else runs on CPU.
The oracle (oracle/) is imported here ONLY as the checker.
"""
from __future__ import annotations

import json
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
GOLDEN = os.path.join(ROOT, "tests", "golden")
PKG = os.path.join(ROOT, "sequence-alignment-gpu_amd")
for p in (os.path.join(ROOT, "oracle"), os.path.join(PKG, "python"), ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)

DNA = "ATCG"
PROT = "ARNDCQEGHILKMFPSTWYVBZX"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an AMD MI355X GPU (HIP engine parity and perf tests)")
    config.addinivalue_line("markers", "slow: long-running CPU test")
    # Build the in-tree libraries if they are missing or were built from other sources (build id, the
    # HIP library cross-compiles on CPU): a stale binary is never tested silently.
    if not os.path.exists(os.path.join(PKG, "lib", "libsa_hip.so")) or not os.path.exists(
            os.path.join(PKG, "bin", "alignSequence")) or _stale():
        subprocess.run(["make", "-s", "-C", PKG, "-j4"], check=True)
    if not os.path.exists(os.path.join(ROOT, "oracle", "_build", "libsa_oracle.so")):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "_build/libsa_oracle.so"], check=True)


def _stale() -> bool:
    """True when lib/libsa_hip.so holds another source hash than this tree's (buildid.py; read from
    the file, not loaded: loading it before torch would start a second HIP runtime)."""
    from sa_amd import buildid
    return buildid.library_id(os.path.join(PKG, "lib", "libsa_hip.so")) != buildid.source_hash()


def load(name: str):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


def encode(letters: str, A: int) -> np.ndarray:
    alpha = DNA if A == 4 else PROT
    lut = {c: i for i, c in enumerate(alpha)}
    return np.array([lut[c] for c in letters], dtype=np.int8)


_MATS = None


def matrix(spec, A: int) -> np.ndarray:
    global _MATS
    if _MATS is None:
        _MATS = load("matrices.json")
    vals = _MATS[spec] if isinstance(spec, str) else spec
    return np.array(vals, dtype=np.int32).reshape(A, A)


def same_result(got: dict, exp: dict) -> bool:
    """Exact comparison against a golden result record (full strings or SHA-256)."""
    import hashlib
    keys = ("score", "num_bytes", "start_text", "start_pattern")
    if any(got[k] != exp[k] for k in keys):
        return False
    if "aligned_text" in exp:
        return got["aligned_text"] == exp["aligned_text"] and got["aligned_pattern"] == exp["aligned_pattern"]
    return (hashlib.sha256(got["aligned_text"].encode()).hexdigest() == exp["sha_text"]
            and hashlib.sha256(got["aligned_pattern"].encode()).hexdigest() == exp["sha_pattern"])


@pytest.fixture(scope="session")
def golden():
    return {n: load(n) for n in ("known_answers.json", "data_pairs.json", "random_pairs.json", "large.json")}


@pytest.fixture(scope="session")
def eng():
    """The HIP engine (ctypes over libsa_hip.so) after its wave-primitive self-test on device 0."""
    from sa_amd import engine
    engine.selftest(0)
    return engine
