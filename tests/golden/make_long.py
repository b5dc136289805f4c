#!/usr/bin/env python3
"""Generates tests/golden/long.json.gz: the reference's two "very long" cases (tests/tests.cu:553-597,
commented out there for run time) with expected outputs from the REFERENCE ITSELF (oracle/_ref,
alignSequenceCPU.cpp:287, one byte per cell in host memory).

  qbpln50 vs mutated_qbpln50        protein --global gap 7   tests.cu:556-558   (70020 x 66700, ~4.7 GB)
  AbHV_ORF111 vs mutated_AbHV_ORF111  DNA --global gap 5     tests.cu:578-580   (~211k x ~202k, ~43 GB)

Run in the build container (where /root/reference is mounted):  python tests/golden/make_long.py
The Requests come from the reference's own parseArguments (ref_align parse, same argv as tests.cu),
so the text/pattern roles and the encoding are the reference's. The first case is also
cross-checked with the C restatement (oracle/sa_oracle.c); the second is too large to hold both
matrices in this container's memory, so only the reference runs it. Only inputs and outputs (data)
are written; the sequences are the reference's own test data files.
"""
from __future__ import annotations

import gzip
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import make_golden as mg  # noqa: E402

CASES = [
    ("qbpln50_protein_global", 556, ["--protein", "--gap-penalty", "7", "--global",
                                      "data/protein/qbpln50.txt", "data/protein/mutated_qbpln50.txt"], True),
    ("AbHV_ORF111_dna_global", 578, ["--dna", "--gap-penalty", "5", "--global",
                                      "data/dna/AbHV_ORF111.txt", "data/dna/mutated_AbHV_ORF111.txt"], False),
]


def main() -> None:
    if not mg.oracle.ref_available():
        raise SystemExit("build the reference first: oracle/build_ref.sh")
    mg.oracle.build()
    out = []
    for name, line, args, cross in CASES:
        req = mg.ref_parse(args)
        A = req["alphabetSize"][0]
        mode = 0 if req["alignment"][0] == 4 else 1
        t = np.array(req["text"], np.int8)
        p = np.array(req["pattern"], np.int8)
        S = np.array(req["matrix"], np.int32)
        t0 = time.time()
        ref = mg.oracle.ref_align_batch([(mode, t, p, S, req["gap"][0])])[0]
        print(f"{name}: {len(t)} x {len(p)} reference {time.time() - t0:.1f} s score {ref['score']}", flush=True)
        if cross and mg.oracle.align(mode, t, p, S, req["gap"][0]) != ref:
            raise SystemExit(f"oracle restatement disagrees with the reference on {name}")
        out.append({"name": name, "tests_cu_line": line, "args": args, "mode": mode, "A": A, "gap": req["gap"][0],
                    "matrix": req["matrix"], "text": mg.letters(t, A), "pattern": mg.letters(p, A),
                    "result": mg.result_record(ref, full_max=0)})
    with gzip.open(os.path.join(HERE, "long.json.gz"), "wt") as f:
        json.dump(out, f)


if __name__ == "__main__":
    main()
