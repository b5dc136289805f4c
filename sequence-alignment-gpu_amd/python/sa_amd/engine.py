"""ctypes binding of the C ABI in include/sa_hip.h (libsa_hip.so).

The product path: every call goes to the HIP engine. If the shared library is missing this
module raises at import time — there is no CPU fallback.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

PKG_ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))
LIB_PATH = os.environ.get("SA_HIP_LIB", os.path.join(PKG_ROOT, "lib", "libsa_hip.so"))

SA_GLOBAL, SA_LOCAL = 0, 1
STATUS = {0: "SA_OK", 1: "SA_ERR_INVALID", 2: "SA_ERR_NOMEM", 3: "SA_ERR_HIP", 4: "SA_ERR_UNSUPPORTED",
          5: "SA_ERR_TIMEOUT"}

# sa_plan_fill_kind (include/sa_hip.h SA_FILL_*)
FILL_KINDS = {0: "strips", 1: "band", 2: "pair", 3: "pair_chain"}

# Symbols declared in include/sa_hip.h (checked by tests/test_capi.py).
EXPORTS = ("sa_align_pair", "sa_plan_create", "sa_plan_destroy", "sa_plan_fill", "sa_plan_traceback",
           "sa_plan_fetch_results", "sa_plan_fetch_alignment", "sa_plan_info", "sa_plan_device_results", "sa_plan_copy_results",
           "sa_device_count", "sa_last_error", "sa_abi_version", "sa_selftest", "sa_plan_fetch_directions", "sa_release_workspace",
           "sa_plan_output_bytes", "sa_plan_fetch_all", "sa_align_batch", "sa_batch_deal", "sa_build_id",
           "sa_batch_last_stats", "sa_plan_fill_kind")


class SaParams(ctypes.Structure):
    _fields_ = [("mode", ctypes.c_int32), ("alphabet_size", ctypes.c_int32), ("gap_penalty", ctypes.c_int32),
                ("rows_per_lane", ctypes.c_int32), ("score_matrix", ctypes.c_void_p), ("alphabet", ctypes.c_char_p)]


class SaPair(ctypes.Structure):
    _fields_ = [("text_offset", ctypes.c_uint64), ("text_len", ctypes.c_uint64),
                ("pattern_offset", ctypes.c_uint64), ("pattern_len", ctypes.c_uint64)]


class SaResult(ctypes.Structure):
    _fields_ = [("score", ctypes.c_int32), ("status", ctypes.c_int32), ("num_alignment_bytes", ctypes.c_uint64),
                ("start_text", ctypes.c_uint64), ("start_pattern", ctypes.c_uint64)]


class SaError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"{STATUS.get(code, code)}: {msg}")
        self.code = code


def _load():
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"HIP engine not built: {LIB_PATH} is missing (run __graft_entry__.build())")
    # One HIP runtime per process: torch ships its own libamdhip64 (soname libamdhip64.so.7, but its
    # libraries NEED "libamdhip64.so"). Loaded first, torch's runtime also satisfies our NEEDED
    # libamdhip64.so.7; loaded after us it would start a second runtime that sees no GPU.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    L = ctypes.CDLL(LIB_PATH)
    P, I, U64 = ctypes.c_void_p, ctypes.c_int, ctypes.c_uint64
    L.sa_align_pair.argtypes = [ctypes.POINTER(SaParams), P, U64, P, U64, I, ctypes.POINTER(SaResult), P, P, U64,
                                ctypes.POINTER(ctypes.c_double)]
    L.sa_plan_create.argtypes = [ctypes.POINTER(SaParams), ctypes.POINTER(SaPair), ctypes.c_int64, I,
                                 ctypes.POINTER(P)]
    L.sa_plan_destroy.argtypes = [P]
    L.sa_plan_fill.argtypes = [P, P, P, P]
    L.sa_plan_traceback.argtypes = [P, P]
    L.sa_plan_fetch_results.argtypes = [P, P, P]
    L.sa_plan_fetch_alignment.argtypes = [P, ctypes.c_int64, P, P, U64, P]
    L.sa_plan_info.argtypes = [P, ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int32),
                               ctypes.POINTER(U64), ctypes.POINTER(U64)]
    L.sa_plan_fetch_directions.argtypes = [P, ctypes.c_int64, P, P]
    L.sa_plan_fill_kind.argtypes = [P]
    L.sa_plan_fill_kind.restype = I
    L.sa_plan_device_results.argtypes = [P]
    L.sa_plan_device_results.restype = P
    L.sa_plan_copy_results.argtypes = [P, P, P]
    L.sa_plan_copy_results.restype = I
    L.sa_device_count.argtypes = [ctypes.POINTER(I)]
    L.sa_last_error.restype = ctypes.c_char_p
    L.sa_selftest.argtypes = [I]
    L.sa_release_workspace.argtypes = [I]
    L.sa_plan_output_bytes.argtypes = [P]
    L.sa_plan_output_bytes.restype = U64
    L.sa_plan_fetch_all.argtypes = [P, ctypes.POINTER(SaResult), P, P, U64, P, P]
    L.sa_align_batch.argtypes = [ctypes.POINTER(SaParams), P, ctypes.c_int64, I, ctypes.POINTER(SaResult), P, P]
    L.sa_batch_deal.argtypes = [P, ctypes.c_int64, I, P]
    L.sa_build_id.restype = ctypes.c_char_p
    L.sa_batch_last_stats.argtypes = [ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ctypes.c_int32), P,
                                      ctypes.c_int32, ctypes.POINTER(ctypes.c_double)]
    for name in EXPORTS:
        getattr(L, name)
    check_build_id(L)
    return L


def check_build_id(L) -> None:
    """Refuse a library built from other sources than the ones next to it (buildid.py). SA_HIP_LIB
    (an explicitly chosen experiment build) and SA_ALLOW_STALE=1 skip the check."""
    from . import buildid
    if "SA_HIP_LIB" in os.environ or os.environ.get("SA_ALLOW_STALE") == "1":
        return
    built = L.sa_build_id().decode()
    want = buildid.source_hash()
    if built != want:
        raise ImportError(f"stale HIP engine: {LIB_PATH} was built from sources {built}, the tree holds {want} "
                          f"(rebuild: make -C {PKG_ROOT})")


lib = _load()


def _check(rc: int) -> None:
    if rc != 0:
        raise SaError(rc, lib.sa_last_error().decode(errors="replace"))


def _params(mode: int, S: np.ndarray, gap: int, alphabet: bytes | None, rows_per_lane: int):
    S = np.ascontiguousarray(S, dtype=np.int32).ravel()
    A = int(round(np.sqrt(S.size)))
    if A * A != S.size:
        raise ValueError("score matrix must be square")
    if alphabet is None:
        alphabet = b"ATCG-" if A == 4 else b"ARNDCQEGHILKMFPSTWYVBZX-"[: A] + b"-"
    p = SaParams(mode, A, gap, rows_per_lane, S.ctypes.data, alphabet)
    return p, S, alphabet


def selftest(device: int = 0) -> None:
    _check(lib.sa_selftest(device))


def align_pair(mode: int, text: np.ndarray, pattern: np.ndarray, S: np.ndarray, gap: int,
               alphabet: bytes | None = None, device: int = 0, rows_per_lane: int = 0) -> dict:
    """One pair from host memory through the HIP engine (synchronous)."""
    text = np.ascontiguousarray(text, dtype=np.int8)
    pattern = np.ascontiguousarray(pattern, dtype=np.int8)
    p, S_keep, alpha_keep = _params(mode, S, gap, alphabet, rows_per_lane)
    n, m = len(text), len(pattern)
    cap = max(1, n + m)
    at = ctypes.create_string_buffer(cap)
    ap = ctypes.create_string_buffer(cap)
    res = SaResult()
    fill_us = ctypes.c_double()
    _check(lib.sa_align_pair(ctypes.byref(p), text.ctypes.data, n, pattern.ctypes.data, m, device,
                             ctypes.byref(res), at, ap, cap, ctypes.byref(fill_us)))
    L = res.num_alignment_bytes
    return {"score": res.score, "num_bytes": L, "start_text": res.start_text, "start_pattern": res.start_pattern,
            "aligned_text": at.raw[:L].decode(), "aligned_pattern": ap.raw[:L].decode(), "fill_us": fill_us.value}


# numpy view of sa_result (include/sa_hip.h): int32 score, int32 status, uint64 x 3
RESULT_DTYPE = np.dtype([("score", "<i4"), ("status", "<i4"), ("num_bytes", "<u8"), ("start_text", "<u8"),
                         ("start_pattern", "<u8")])
assert RESULT_DTYPE.itemsize == ctypes.sizeof(SaResult)


class SaHostPair(ctypes.Structure):
    _fields_ = [("text", ctypes.c_void_p), ("text_len", ctypes.c_uint64), ("pattern", ctypes.c_void_p),
                ("pattern_len", ctypes.c_uint64)]


def batch_deal(cells: list[int], num_shards: int) -> list[int]:
    """sa_batch_deal: the pair -> shard assignment sa_align_batch uses (host only)."""
    c = np.ascontiguousarray(cells, dtype=np.uint64)
    out = np.zeros(max(1, len(c)), np.int32)
    _check(lib.sa_batch_deal(c.ctypes.data, len(c), num_shards, out.ctypes.data))
    return out[: len(c)].tolist()


def batch_last_stats() -> dict:
    """sa_batch_last_stats: the calling thread's last sa_align_batch (shards, RCCL or not, per-shard
    wall ms from upload to traceback end, gather wall ms)."""
    ns, rc = ctypes.c_int32(0), ctypes.c_int32(0)
    ms = np.zeros(64, np.float64)
    g = ctypes.c_double(0)
    _check(lib.sa_batch_last_stats(ctypes.byref(ns), ctypes.byref(rc), ms.ctypes.data, 64, ctypes.byref(g)))
    return {"num_shards": ns.value, "used_rccl": bool(rc.value), "shard_ms": ms[: ns.value].round(3).tolist(),
            "gather_ms": round(g.value, 3)}


def align_batch(mode: int, texts: list[np.ndarray], patterns: list[np.ndarray], S: np.ndarray, gap: int,
                num_gpus: int = 1, alphabet: bytes | None = None, strings: bool = True) -> list[dict]:
    """sa_align_batch: independent pairs from host memory over devices 0..num_gpus-1 (synchronous)."""
    p, S_keep, alpha_keep = _params(mode, S, gap, alphabet, 0)
    ts = [np.ascontiguousarray(t, dtype=np.int8) for t in texts]
    ps = [np.ascontiguousarray(x, dtype=np.int8) for x in patterns]
    n = len(ts)
    hp = (SaHostPair * max(1, n))(*[SaHostPair(t.ctypes.data, len(t), x.ctypes.data, len(x)) for t, x in zip(ts, ps)])
    bufs_t = [ctypes.create_string_buffer(max(1, len(t) + len(x))) for t, x in zip(ts, ps)] if strings else []
    bufs_p = [ctypes.create_string_buffer(max(1, len(t) + len(x))) for t, x in zip(ts, ps)] if strings else []
    at = (ctypes.c_void_p * max(1, n))(*[ctypes.addressof(b) for b in bufs_t]) if strings else None
    ap = (ctypes.c_void_p * max(1, n))(*[ctypes.addressof(b) for b in bufs_p]) if strings else None
    res = (SaResult * max(1, n))()
    _check(lib.sa_align_batch(ctypes.byref(p), hp, n, num_gpus, res, at, ap))
    out = []
    for i, r in enumerate(res[:n]):
        d = {"score": r.score, "num_bytes": r.num_alignment_bytes, "start_text": r.start_text,
             "start_pattern": r.start_pattern}
        if strings:
            L = r.num_alignment_bytes
            d["aligned_text"] = bufs_t[i].raw[:L].decode()
            d["aligned_pattern"] = bufs_p[i].raw[:L].decode()
        out.append(d)
    return out


class Plan:
    """Many pairs, device-resident arenas, explicit stream (for benches and the batch path)."""

    def __init__(self, mode: int, S: np.ndarray, gap: int, pairs: list[tuple[int, int, int, int]],
                 device: int = 0, alphabet: bytes | None = None, rows_per_lane: int = 0):
        self._p, self._S, self._alpha = _params(mode, S, gap, alphabet, rows_per_lane)
        arr = (SaPair * max(1, len(pairs)))(*[SaPair(*pr) for pr in pairs])
        self.num_pairs = len(pairs)
        self.pairs = pairs
        self.device = device
        h = ctypes.c_void_p()
        _check(lib.sa_plan_create(ctypes.byref(self._p), arr, len(pairs), device, ctypes.byref(h)))
        self.handle = h

    def close(self) -> None:
        if getattr(self, "handle", None):
            lib.sa_plan_destroy(self.handle)
            self.handle = None

    __del__ = close

    def info(self) -> dict:
        ns, r, db, mb = ctypes.c_int64(), ctypes.c_int32(), ctypes.c_uint64(), ctypes.c_uint64()
        _check(lib.sa_plan_info(self.handle, ctypes.byref(ns), ctypes.byref(r), ctypes.byref(db), ctypes.byref(mb)))
        kind = lib.sa_plan_fill_kind(self.handle)
        return {"num_strips": ns.value, "rows_per_lane": r.value, "device_bytes": db.value, "mask_bytes": mb.value,
                "fill_kernel": FILL_KINDS.get(kind, kind)}

    def fill(self, d_text: int, d_pattern: int, stream: int | None = None) -> None:
        _check(lib.sa_plan_fill(self.handle, d_text, d_pattern, stream))

    def traceback(self, stream: int | None = None) -> None:
        _check(lib.sa_plan_traceback(self.handle, stream))

    def results(self, stream: int | None = None) -> list[dict]:
        out = (SaResult * max(1, self.num_pairs))()
        _check(lib.sa_plan_fetch_results(self.handle, out, stream))
        return [{"score": r.score, "num_bytes": r.num_alignment_bytes, "start_text": r.start_text,
                 "start_pattern": r.start_pattern} for r in out[: self.num_pairs]]

    def results_array(self, stream: int | None = None) -> np.ndarray:
        """Every pair's sa_result as one numpy structured array (RESULT_DTYPE): no per-pair objects."""
        out = np.empty(max(1, self.num_pairs), RESULT_DTYPE)
        _check(lib.sa_plan_fetch_results(self.handle, out.ctypes.data, stream))
        return out[: self.num_pairs]

    def copy_results(self, d_dst: int, stream: int | None = None) -> None:
        """Asynchronous device-to-device copy of every pair's sa_result (32 bytes each) to d_dst."""
        _check(lib.sa_plan_copy_results(self.handle, d_dst, stream))

    def directions(self, index: int, stream: int | None = None) -> np.ndarray:
        """Decoded (m+1)x(n+1) DIRECTION matrix of pair `index` (reference layout, for verification)."""
        n, m = self.pairs[index][1], self.pairs[index][3]
        M = np.empty((m + 1) * (n + 1), dtype=np.uint8)
        _check(lib.sa_plan_fetch_directions(self.handle, index, M.ctypes.data, stream))
        return M

    def alignment(self, index: int, stream: int | None = None) -> tuple[str, str]:
        cap = max(1, self.pairs[index][1] + self.pairs[index][3])
        at = ctypes.create_string_buffer(cap)
        ap = ctypes.create_string_buffer(cap)
        _check(lib.sa_plan_fetch_alignment(self.handle, index, at, ap, cap, stream))
        r = self.results(stream)[index]
        return at.raw[: r["num_bytes"]].decode(), ap.raw[: r["num_bytes"]].decode()

    def all_alignments(self, stream: int | None = None) -> list[dict]:
        """Every pair's result with its aligned strings, fetched in one pass (sa_plan_fetch_all)."""
        nb = int(lib.sa_plan_output_bytes(self.handle))
        tb = np.empty(max(1, nb), np.uint8)
        pb = np.empty(max(1, nb), np.uint8)
        out = (SaResult * max(1, self.num_pairs))()
        offs = np.zeros(max(1, self.num_pairs), np.uint64)
        _check(lib.sa_plan_fetch_all(self.handle, out, tb.ctypes.data, pb.ctypes.data, max(1, nb),
                                     offs.ctypes.data, stream))
        res = []
        for r, o in zip(out[: self.num_pairs], offs.tolist()):
            L = r.num_alignment_bytes
            res.append({"score": r.score, "num_bytes": L, "start_text": r.start_text, "start_pattern": r.start_pattern,
                        "aligned_text": tb[o:o + L].tobytes().decode(), "aligned_pattern": pb[o:o + L].tobytes().decode()})
        return res
