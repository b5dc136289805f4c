"""TEST INFRASTRUCTURE ONLY — Python access to the CPU oracle and to the reference's own CPU path.

* ``align`` / ``fill_only`` call the C restatement in ``oracle/sa_oracle.c`` (built into
  ``oracle/_build/libsa_oracle.so``), which follows ``alignSequenceCPU.cpp:10-333``.
* ``ref_align_batch`` runs ``oracle/_ref/ref_align`` — the reference's own
  ``alignSequenceCPU`` compiled by ``oracle/build_ref.sh`` — on binary records.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s cpu_baseline leg use this module,
and only as the checker / CPU baseline. The product path never imports it.
"""
from __future__ import annotations

import ctypes
import os
import struct
import subprocess
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "_build", "libsa_oracle.so")
REF_BIN = os.path.join(HERE, "_ref", "ref_align")

DNA_ALPHABET = b"ATCG-"                      # SequenceAlignment.hpp:56
PROTEIN_ALPHABET = b"ARNDCQEGHILKMFPSTWYVBZX-"  # SequenceAlignment.hpp:57-58

_lib = None


def build() -> None:
    subprocess.run(["make", "-s", "-C", HERE, "_build/libsa_oracle.so"], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        P = ctypes.c_void_p
        L.oracle_align.argtypes = [ctypes.c_int, P, ctypes.c_uint64, P, ctypes.c_uint64, P, ctypes.c_int32,
                                   ctypes.c_int32, ctypes.c_char_p, P, P, P, P, P, P]
        L.oracle_align.restype = ctypes.c_int
        L.oracle_fill_only.argtypes = [ctypes.c_int, P, ctypes.c_uint64, P, ctypes.c_uint64, P,
                                       ctypes.c_int32, ctypes.c_int32, P]
        L.oracle_fill_only.restype = ctypes.c_int32
        _lib = L
    return _lib


def alphabet_for(A: int) -> bytes:
    return DNA_ALPHABET if A == 4 else PROTEIN_ALPHABET


def align(mode: int, text: np.ndarray, pattern: np.ndarray, S: np.ndarray, gap: int,
          alphabet: bytes | None = None) -> dict:
    """Reference CPU semantics for one pair. mode 0 = global, 1 = local."""
    text = np.ascontiguousarray(text, dtype=np.int8)
    pattern = np.ascontiguousarray(pattern, dtype=np.int8)
    S = np.ascontiguousarray(S, dtype=np.int32)
    A = int(round(np.sqrt(S.size)))
    alphabet = alphabet or alphabet_for(A)
    n, m = len(text), len(pattern)
    cap = max(1, n + m)
    at = ctypes.create_string_buffer(cap)
    ap = ctypes.create_string_buffer(cap)
    score = ctypes.c_int32()
    nb, st, sp = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint64()
    rc = lib().oracle_align(mode, text.ctypes.data, n, pattern.ctypes.data, m, S.ctypes.data, A, gap,
                            alphabet, ctypes.byref(score), ctypes.byref(nb), ctypes.byref(st),
                            ctypes.byref(sp), at, ap)
    if rc:
        raise MemoryError("oracle: direction matrix allocation failed")
    L = nb.value
    return {"score": score.value, "num_bytes": L, "start_text": st.value, "start_pattern": sp.value,
            "aligned_text": at.raw[:L].decode(), "aligned_pattern": ap.raw[:L].decode()}


def fill_only(mode: int, text: np.ndarray, pattern: np.ndarray, S: np.ndarray, gap: int,
              M: np.ndarray | None = None) -> int:
    """Fill the (m+1)x(n+1) direction matrix only (tests/benchmarks.cu:153-154 convention). mode 2: local
    with the raw decision of every interior cell (no STOP override; the engine's rows_per_lane 1 planes)."""
    text = np.ascontiguousarray(text, dtype=np.int8)
    pattern = np.ascontiguousarray(pattern, dtype=np.int8)
    S = np.ascontiguousarray(S, dtype=np.int32)
    A = int(round(np.sqrt(S.size)))
    n, m = len(text), len(pattern)
    if M is None:
        M = np.empty((m + 1) * (n + 1), dtype=np.uint8)
    return lib().oracle_fill_only(mode, text.ctypes.data, n, pattern.ctypes.data, m, S.ctypes.data, A, gap,
                                  M.ctypes.data)


def ref_available() -> bool:
    return os.path.exists(REF_BIN)


def ref_align_batch(jobs: list[tuple]) -> list[dict]:
    """Run the reference's own alignSequenceCPU on jobs = [(mode, text, pattern, S, gap), ...]."""
    with tempfile.TemporaryDirectory() as d:
        inp, out = os.path.join(d, "in.bin"), os.path.join(d, "out.bin")
        with open(inp, "wb") as f:
            for mode, text, pattern, S, gap in jobs:
                S = np.ascontiguousarray(S, dtype=np.int32)
                A = int(round(np.sqrt(S.size)))
                f.write(struct.pack("<iiiiQQ", mode, A, gap, 0, len(text), len(pattern)))
                f.write(S.tobytes())
                f.write(np.asarray(text, dtype=np.int8).tobytes())
                f.write(np.asarray(pattern, dtype=np.int8).tobytes())
        subprocess.run([REF_BIN, "batch", inp, out], check=True)
        res = []
        with open(out, "rb") as f:
            for _ in jobs:
                score, _pad, L, st, sp = struct.unpack("<iiQQQ", f.read(32))
                at = f.read(L).decode()
                ap = f.read(L).decode()
                res.append({"score": score, "num_bytes": L, "start_text": st, "start_pattern": sp,
                            "aligned_text": at, "aligned_pattern": ap})
        return res
