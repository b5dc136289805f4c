#!/usr/bin/env python3
"""Generates tests/golden/gap_pairs.json and the negative-gap CLI cases in tests/golden/cli/expected.json
from the REFERENCE ITSELF (oracle/_ref/ref_align = the reference's alignSequenceCPU and CLI).

Gap penalties <= 0: the reference CLI reads any int after --gap-penalty ("-3" is not an argumentMap
key, so std::stoi takes it, utilities.cpp:156,188-199) and its fill subtracts it as is
(alignSequenceCPU.cpp:175-176, 259-260). Cases: g in {0, -1, -2, -5}, both modes, DNA (blast, dnaMat)
and protein (BLOSUM50/62), small sizes around 64-row strip edges and multi-strip / multi-group sizes
(up to 1500 rows: several 4-strip groups of the R = 1 chain). The C oracle is cross-checked on every
record (run_jobs). Pattern-longer-than-text cases are outside the reference CLI's contract (2*text
output buffers) and come from the oracle ("by": "oracle"), as in make_golden.py.
Run in the build container:  python tests/golden/make_gaps.py
"""
import json
import os
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.abspath(os.path.join(HERE, "..", ".."))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "sequence-alignment-gpu_amd", "python"))
sys.path.insert(0, HERE)
import oracle  # noqa: E402
from make_golden import REF, letters, result_record, run_jobs  # noqa: E402
from sa_amd import synthetic  # noqa: E402

GAPS = (0, -1, -2, -5)


def main() -> None:
    if not oracle.ref_available():
        raise SystemExit("build the reference first: oracle/build_ref.sh")
    oracle.build()
    mats = json.load(open(os.path.join(HERE, "matrices.json")))
    rng = np.random.default_rng(20261017)
    cases, jobs = [], []

    def add(mode, t, p, mat, gap, tag, ref_ok=True):
        A = 4 if len(mats[mat]) == 16 else 23
        cases.append({"mode": mode, "A": A, "gap": gap, "matrix": mat, "text": letters(t, A),
                      "pattern": letters(p, A), "tag": tag, "by": "reference" if ref_ok else "oracle"})
        jobs.append((mode, t, p, mats[mat], gap, ref_ok))

    for mode in (0, 1):
        for gap in GAPS:
            for n, m in ((1, 1), (5, 3), (64, 64), (65, 63), (130, 129), (300, 256), (257, 200)):
                t = rng.integers(0, 4, n).astype(np.int8)
                p = rng.integers(0, 4, m).astype(np.int8)
                add(mode, t, p, "blast", gap, "edge_dna")
            for _ in range(4):
                n = int(rng.integers(100, 700)); m = int(rng.integers(1, n + 1))
                t = rng.integers(0, 4, n).astype(np.int8)
                add(mode, t, synthetic.mutate(t, int(rng.integers(1 << 30)), 4, m), "blast", gap, "mutated_dna")
            for _ in range(2):
                n = int(rng.integers(50, 400)); m = int(rng.integers(1, n + 1))
                add(mode, rng.integers(0, 4, n).astype(np.int8), rng.integers(0, 4, m).astype(np.int8), "dnaMat",
                    gap, "dnamat")
            for bl in ("blosum50", "blosum62"):
                for _ in range(3):
                    n = int(rng.integers(20, 500)); m = int(rng.integers(1, n + 1))
                    t = rng.integers(0, 20, n).astype(np.int8)
                    p = synthetic.mutate(t, int(rng.integers(1 << 30)), 20, m) if rng.random() < 0.5 \
                        else rng.integers(0, 23, m).astype(np.int8)
                    add(mode, t, p, bl, gap, "protein")
            # multi-strip, multi-group chains (R = 1: 64 rows per strip, 4 strips per group)
            for n, m in ((1500, 1500), (1200, 700), (2100, 1030)):
                t = rng.integers(0, 4, n).astype(np.int8)
                p = synthetic.mutate(t, int(rng.integers(1 << 30)), 4, m) if m != n \
                    else rng.integers(0, 4, m).astype(np.int8)
                add(mode, t, p, "blast", gap, "chain_dna")
            n, m = 900, 800
            t = rng.integers(0, 20, n).astype(np.int8)
            add(mode, t, synthetic.mutate(t, int(rng.integers(1 << 30)), 20, m), "blosum62", gap, "chain_protein")
            # pattern longer than text (oracle)
            m = int(rng.integers(70, 300)); n = int(rng.integers(1, m))
            add(mode, rng.integers(0, 4, n).astype(np.int8), rng.integers(0, 4, m).astype(np.int8), "blast", gap,
                "text_shorter", ref_ok=False)
    ref_jobs = [(m, t, p, S, g) for m, t, p, S, g, ok in jobs if ok]
    ref_res = iter(run_jobs(ref_jobs))
    for c, (m, t, p, S, g, ok) in zip(cases, jobs):
        r = next(ref_res) if ok else oracle.align(m, t, p, np.array(S, np.int32), g)
        c["result"] = result_record(r, full_max=10**6)
    json.dump(cases, open(os.path.join(HERE, "gap_pairs.json"), "w"))
    print("gap pairs:", len(cases))

    # CLI: the reference's stdout with a negative gap penalty, both modes
    cdir = os.path.join(HERE, "cli")
    exp_path = os.path.join(cdir, "expected.json")
    cli_out = json.load(open(exp_path))
    clis = {
        "config1_gap_minus2": ["-d", "-c", "--gap-penalty", "-2", "--global", "A", "B"],
        "config1_local_gap_minus2": ["-d", "-c", "--gap-penalty", "-2", "--local", "A", "B"],
        "dna_01_02_gap0": ["--gap-penalty", "0", "--global", f"{REF}/data/dna/dna_01.txt", f"{REF}/data/dna/dna_02.txt"],
    }
    for name, args in clis.items():
        args = [os.path.join(cdir, "a.txt") if x == "A" else os.path.join(cdir, "b.txt") if x == "B" else x for x in args]
        r = subprocess.run([oracle.REF_BIN, "cli", *args], cwd=REF, capture_output=True, text=True, check=True)
        shown = [x.replace(cdir + "/", "").replace(REF + "/", "") for x in args]
        cli_out[name] = {"args": shown, "stdout": r.stdout}
    json.dump(cli_out, open(exp_path, "w"), indent=1)
    print("cli cases:", len(cli_out))


if __name__ == "__main__":
    main()
