#!/usr/bin/env python3
"""Generates tests/golden/edge_pairs.json: pairs with an empty text and/or pattern, both modes, DNA
(blast) and protein (BLOSUM50), from the REFERENCE ITSELF (oracle/_ref/ref_align = the reference's
alignSequenceCPU), cross-checked with the C oracle. The reference's behaviour there: global (0,k) /
(k,0) aligns k letters against gaps (score -k*g, starts 0); global (0,0) and every local case give an
empty alignment with starts (uint64)-1 (alignSequenceCPU.cpp:10-114 on a 1-row or 1-column M).
Run in the build container:  python tests/golden/make_edge.py
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.abspath(os.path.join(HERE, "..", ".."))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "sequence-alignment-gpu_amd", "python"))
sys.path.insert(0, HERE)
import oracle  # noqa: E402
from make_golden import letters, result_record, run_jobs  # noqa: E402
from sa_amd import synthetic  # noqa: E402


def main() -> None:
    mats = json.load(open(os.path.join(HERE, "matrices.json")))
    cases, jobs = [], []
    for A, mat in ((4, "blast"), (23, "blosum50")):
        for mode in (0, 1):
            for k, (n, m) in enumerate([(0, 1), (0, 7), (0, 64), (0, 65), (0, 200), (1, 0), (7, 0), (64, 0),
                                        (65, 0), (200, 0), (0, 0)]):
                t = synthetic.random_sequence(300 + k, n, 20 if A == 23 else 4)
                p = synthetic.random_sequence(400 + k, m, 20 if A == 23 else 4)
                cases.append({"mode": mode, "A": A, "matrix": mat, "gap": 5, "text": letters(t, A),
                              "pattern": letters(p, A)})
                jobs.append((mode, t, p, mats[mat], 5))
    # the reference allocates its output buffers as 2 * textNumBytes (alignSequenceCPU.cpp:306-307):
    # a pattern longer than the text (here: an empty text) is outside its contract (parseArguments
    # swaps to text >= pattern, utilities.cpp:225-230) and overflows them, so those cases come from
    # the oracle and are marked "by": "oracle", as in make_golden.py
    ref_idx = [i for i, c in enumerate(cases) if len(c["text"]) >= len(c["pattern"])]
    for i, r in zip(ref_idx, run_jobs([jobs[i] for i in ref_idx])):
        cases[i]["result"] = result_record(r)
        cases[i]["by"] = "reference"
    for i, c in enumerate(cases):
        if "result" not in c:
            m, t, p, S, g = jobs[i]
            c["result"] = result_record(oracle.align(m, t, p, np.array(S, np.int32), g))
            c["by"] = "oracle"
    json.dump(cases, open(os.path.join(HERE, "edge_pairs.json"), "w"), indent=0)
    print("edge cases:", len(cases))


if __name__ == "__main__":
    main()
