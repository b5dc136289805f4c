#!/usr/bin/env python3
"""Generates tests/golden/batch.json.gz: EVERY pair of BASELINE.json config 5 (4096 independent
2048 x 2048 DNA global pairs, blast, gap 5, seeds 1000+2i / 1001+2i — the exact batch bench.py
times) plus a local-mode batch (1024 pairs of 2048 x 2048, pattern = mutate(text)), from the
REFERENCE ITSELF: oracle/_ref/ref_align (the reference's alignSequenceCPU, alignSequenceCPU.cpp:287)
run over 8 chunks in parallel processes. The C oracle restatement is cross-checked on every 16th
pair. The reference's own batch test compares every pair the same way (tests/tests.cu:463-551).

Per pair the record is [score, num_alignment_bytes, start_text, start_pattern, h], where h is the
first 24 hex digits of SHA-256(aligned_text + "\\n" + aligned_pattern). Inputs are regenerated from
the seeds by sa_amd.synthetic. Run in the build container:  python tests/golden/make_batch.py
"""
from __future__ import annotations

import gzip
import hashlib
import json
import os
import sys
from concurrent.futures import ProcessPoolExecutor

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.abspath(os.path.join(HERE, "..", ".."))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "sequence-alignment-gpu_amd", "python"))
import oracle  # noqa: E402
from sa_amd import synthetic  # noqa: E402

L = 2048
SETS = {
    # name: (mode, pairs, text seed base, pattern kind)
    "global": (0, 4096, 1000, "rand"),
    "local": (1, 1024, 20000, "mut"),
}


def pair_inputs(kind: str, base: int, i: int) -> tuple[np.ndarray, np.ndarray]:
    t = synthetic.random_sequence(base + 2 * i, L, 4)
    p = synthetic.random_sequence(base + 2 * i + 1, L, 4) if kind == "rand" else synthetic.mutate(t, base + 2 * i + 1, 4, L)
    return t, p


def digest(at: str, ap: str) -> str:
    return hashlib.sha256((at + "\n" + ap).encode()).hexdigest()[:24]


def run_chunk(args):
    mode, kind, base, lo, hi = args
    S = synthetic.blast_matrix()
    jobs = [(mode, *pair_inputs(kind, base, i), S, 5) for i in range(lo, hi)]
    out = []
    for (m, t, p, _, g), r in zip(jobs, oracle.ref_align_batch(jobs)):
        out.append([r["score"], r["num_bytes"], r["start_text"], r["start_pattern"],
                    digest(r["aligned_text"], r["aligned_pattern"])])
    for k in range(0, len(jobs), 16):  # cross-check the restatement on a sample
        m, t, p, S_, g = jobs[k]
        if oracle.align(m, t, p, S_, g) != oracle.ref_align_batch([jobs[k]])[0]:
            raise SystemExit(f"oracle restatement disagrees with the reference at pair {lo + k}")
    return out


def main() -> None:
    if not os.path.exists(oracle.REF_BIN):
        raise SystemExit("needs oracle/_ref/ref_align (oracle/build_ref.sh, with /root/reference mounted)")
    doc = {"L": L, "matrix": "blast", "gap": 5, "record": ["score", "num_bytes", "start_text", "start_pattern",
                                                          "sha256(text+'\\n'+pattern)[:24]"]}
    with ProcessPoolExecutor(8) as ex:
        for name, (mode, n, base, kind) in SETS.items():
            step = (n + 7) // 8
            chunks = [(mode, kind, base, lo, min(n, lo + step)) for lo in range(0, n, step)]
            recs = [r for part in ex.map(run_chunk, chunks) for r in part]
            doc[name] = {"mode": mode, "pairs": n, "seed_base": base, "pattern": kind, "records": recs}
            print(name, n, "pairs; first", recs[0])
    with gzip.open(os.path.join(HERE, "batch.json.gz"), "wt") as f:
        json.dump(doc, f, separators=(",", ":"))


if __name__ == "__main__":
    main()
