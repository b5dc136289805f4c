#!/usr/bin/env python3
"""Generates the committed parity fixtures in tests/golden/ from the REFERENCE ITSELF.

Run in the build container (where /root/reference is mounted):  python tests/golden/make_golden.py
Every expected output below comes from oracle/_ref/ref_align — the reference's own
alignSequenceCPU (alignSequenceCPU.cpp:287) / parseArguments (utilities.cpp:131) /
prettyAlignmentPrint (utilities.cpp:253), compiled by oracle/build_ref.sh. The C restatement in
oracle/sa_oracle.c is cross-checked against every record as it is generated. Only inputs and outputs
(data) are written; no reference source is copied.

Files
  matrices.json       score matrices of the reference (scoreMatrices/*, data)
  known_answers.json  tests/tests.cu:116-366 known-answer cases (+ the hard-coded expectations)
  data_pairs.json     tests/tests.cu:463-551 all-pairs cases over data/dna and data/protein
  random_pairs.json   seeded random / mutated / edge-length pairs, both modes, DNA and protein
  large.json          config-sized cases (8192^2, 32768^2, 4096^2 protein, 2048^2 batch pairs): score,
                      length, starts and SHA-256 of the aligned strings; inputs are regenerated from
                      the recorded seeds by sa_amd.synthetic
  cli/                config-1 CLI inputs and the reference's exact stdout
"""
from __future__ import annotations

import hashlib
import json
import os
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.abspath(os.path.join(HERE, "..", ".."))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "sequence-alignment-gpu_amd", "python"))
import oracle  # noqa: E402
from sa_amd import synthetic  # noqa: E402

REF = os.environ.get("SA_REFERENCE", "/root/reference")
DNA = "ATCG"
PROT = "ARNDCQEGHILKMFPSTWYVBZX"


def sha(s: str) -> str:
    return hashlib.sha256(s.encode()).hexdigest()


def letters(seq, A) -> str:
    alpha = DNA if A == 4 else PROT
    return "".join(alpha[int(c)] for c in seq)


def read_matrix(path: str, A: int) -> list[int]:
    toks = open(path).read().split()
    return [int(t) for t in toks[: A * A]]


def encode_file(path: str, alphabet: str) -> np.ndarray:
    """Restates validateAndTransform (utilities.cpp:31-63); checked against ref 'parse' below."""
    raw = open(path, "rb").read()
    out, ignore = [], False
    for b in raw:
        if not ignore and b == ord(">"):
            ignore = True
        elif ignore and b == ord("\n"):
            ignore = False
        elif ignore:
            continue
        up = b - 32 if b > 90 else b
        if up < 65 or up > 90:
            continue
        out.append(alphabet.index(chr(up)))
    return np.array(out, dtype=np.int8)


def ref_parse(args: list[str]) -> dict:
    r = subprocess.run([oracle.REF_BIN, "parse", *args], cwd=REF, capture_output=True, text=True, check=True)
    d = {}
    for line in r.stdout.splitlines():
        k, *v = line.split(" ")
        d[k] = [int(x) for x in v]
    return d


def result_record(r: dict, full_max: int = 300) -> dict:
    rec = {"score": r["score"], "num_bytes": r["num_bytes"], "start_text": r["start_text"],
           "start_pattern": r["start_pattern"], "sha_text": sha(r["aligned_text"]),
           "sha_pattern": sha(r["aligned_pattern"])}
    if r["num_bytes"] <= full_max:
        rec["aligned_text"] = r["aligned_text"]
        rec["aligned_pattern"] = r["aligned_pattern"]
    return rec


def run_jobs(jobs):
    """jobs: (mode, text, pattern, S(list), gap). Reference results, cross-checked with the C oracle."""
    ref = oracle.ref_align_batch([(m, t, p, np.array(S, np.int32), g) for m, t, p, S, g in jobs])
    for (m, t, p, S, g), r in zip(jobs, ref):
        o = oracle.align(m, t, p, np.array(S, np.int32), g)
        if o != r:
            raise SystemExit(f"oracle restatement disagrees with the reference: mode={m} n={len(t)} m={len(p)}")
    return ref


def main() -> None:
    if not oracle.ref_available():
        raise SystemExit("build the reference first: oracle/build_ref.sh")
    oracle.build()
    mats = {
        "blast": read_matrix(f"{REF}/scoreMatrices/dna/blast.txt", 4),
        "dnaMat": read_matrix(f"{REF}/scoreMatrices/dna/dnaMat.txt", 4),
    }
    for b in (30, 35, 40, 50, 62, 65, 80):
        mats[f"blosum{b}"] = read_matrix(f"{REF}/scoreMatrices/protein/blosum{b}.txt", 23)
    json.dump(mats, open(os.path.join(HERE, "matrices.json"), "w"))

    # ---------------- known answers: tests/tests.cu:116-366 ----------------
    # (name, args, expected score, expected strings or None, expected starts or None, tests.cu line)
    ka_cli = [
        ("DNA_01", ["--gap-penalty", "5", "--global", "data/dna/dna_01.txt", "data/dna/dna_02.txt"], -4, None, None, 119),
        ("DNA_05", ["--gap-penalty", "5", "--global", "data/dna/NC_018874.txt", "data/dna/GCA_003231495.txt"], -5991, None, None, 234),
        ("PROTEIN_02", ["--protein", "--gap-penalty", "5", "--global", "data/protein/P02232.fasta", "data/protein/P03989.fasta"], -597, None, None, 294),
        ("PROTEIN_03", ["--protein", "--cpu", "--gap-penalty", "5", "--global", "data/protein/P05013.fasta", "data/protein/P07327.fasta"], -423, None, None, 310),
        ("LOCAL_DNA_01", ["--gap-penalty", "5", "--local", "data/dna/GCA_003231495.txt", "data/dna/dna_01.txt"], 20, ("ACAC", "ACAC"), (248, 0), 330),
        ("LOCAL_PROTEIN_01", ["--protein", "--gap-penalty", "10", "--local", "data/protein/P08519.fasta", "data/protein/P10635.fasta"], 57, None, (4203, 94), 352),
        # GPU-vs-CPU sections (tests.cu:370-460): inputs only; the expectation is the CPU result.
        ("GPU_GLOBAL_PROTEIN_01", ["--protein", "--gpu", "--gap-penalty", "11", "--global", "data/protein/P10635.fasta", "data/protein/P02232.fasta"], None, None, None, 372),
        ("GPU_GLOBAL_PROTEIN_02", ["--protein", "--gpu", "--gap-penalty", "5", "--global", "data/protein/P27895.fasta", "data/protein/P27895.fasta"], None, None, None, 392),
        ("GPU_LOCAL_DNA_01", ["--gap-penalty", "5", "--local", "data/dna/GCA_003231495.txt", "data/dna/dna_01.txt"], None, None, None, 417),
        ("GPU_LOCAL_PROTEIN_01", ["--protein", "--gap-penalty", "5", "--local", "data/protein/P33450.fasta", "data/protein/P07327.fasta"], None, None, None, 439),
    ]
    ka_str = [
        ("DNA_02", "GCCT", "GGTC", 4, -4, None, 135),
        ("DNA_03", "TTCGCCT", "CTCGGTC", 4, 2, None, 163),
        ("DNA_04", "CATAAAACTCTCGGTCGGGCTTAGTACCAGGACCGGCGCACCAGAGTGTCAATCACGACCCTTCACACTTTGTGC",
         "ATGAAGTTGTTCGCCTTACTTTTAATTCTACTCTCTCCTCGAGATTCGTCCGCTGAAAAATCTCTCAGCG", 4, 22,
         ("CATAAAACTCTCGGTCGGGCTTAGTACCAGGAC--CGGCGCACCA-GAG-TGTCAATCACGACCCTTCACACTTTGT--GC-",
          "-ATGAAG-T-T-GTTCGC-CTTACTTTTAATTCTACT-CTCTCCTCGAGAT-TCG-TC-CG-C--TGAAAAATCTCTCAGCG"), 191),
        ("PROTEIN_01",
         "MVLSPADKTNVKAAWGKVGAHAGEYGAEALERMFLSFPTTKTYFPHFDLSHGSAQVKGHGKKVADALTNAVAHVDDMPNALSALSDLHAHKLRVDPVNFKLLSHCLLVTLAAHLPAEFTPAVHASLDKFLASVSTVLTSKYR",
         "MVLSGEDKSNIKAAWGKIGGHGAEYGAEALERMFASFPTTKTYFPHFDVSHGSAQVKGHGKKVADALASAAGHLDDLPGALSALSDLHAHKLRVDPVNFKLLSHCLLVTLASHHPADFTPAVHASLDKFLASVSTVLTSKYR",
         23, 821,
         ("MVLSPADKTNVKAAWGKVGAHAGEYGAEALERMFLSFPTTKTYFPHFDLSHGSAQVKGHGKKVADALTNAVAHVDDMPNALSALSDLHAHKLRVDPVNFKLLSHCLLVTLAAHLPAEFTPAVHASLDKFLASVSTVLTSKYR",
          "MVLSGEDKSNIKAAWGKIGGHGAEYGAEALERMFASFPTTKTYFPHFDVSHGSAQVKGHGKKVADALASAAGHLDDLPGALSALSDLHAHKLRVDPVNFKLLSHCLLVTLASHHPADFTPAVHASLDKFLASVSTVLTSKYR"), 251),
    ]
    known = []
    jobs = []
    for name, args, exp, strs, starts, line in ka_cli:
        req = ref_parse(args)
        A = req["alphabetSize"][0]
        mode = 0 if req["alignment"][0] == 4 else 1  # programArgs: GLOBAL=4, LOCAL=5
        known.append({"name": name, "tests_cu_line": line, "mode": mode, "A": A, "gap": req["gap"][0],
                      "matrix": req["matrix"], "text": letters(req["text"], A), "pattern": letters(req["pattern"], A),
                      "expect_score": exp, "expect_strings": strs, "expect_starts": starts})
        jobs.append((mode, np.array(req["text"], np.int8), np.array(req["pattern"], np.int8), req["matrix"], req["gap"][0]))
    for name, t, p, A, exp, strs, line in ka_str:
        alpha = DNA if A == 4 else PROT
        mat = mats["blast"] if A == 4 else mats["blosum50"]
        # these cases build the Request directly (no swap), tests.cu:137-154
        known.append({"name": name, "tests_cu_line": line, "mode": 0, "A": A, "gap": 5, "matrix": mat,
                      "text": t, "pattern": p, "expect_score": exp, "expect_strings": strs, "expect_starts": None})
        jobs.append((0, np.array([alpha.index(c) for c in t], np.int8), np.array([alpha.index(c) for c in p], np.int8), mat, 5))
    for k, r in zip(known, run_jobs(jobs)):
        if k["expect_score"] is not None:
            assert r["score"] == k["expect_score"], (k["name"], r["score"])
        if k["expect_strings"]:
            assert (r["aligned_text"], r["aligned_pattern"]) == tuple(k["expect_strings"]), k["name"]
        if k["expect_starts"]:
            assert (r["start_text"], r["start_pattern"]) == tuple(k["expect_starts"]), k["name"]
        k["result"] = result_record(r, full_max=10**6)
    json.dump(known, open(os.path.join(HERE, "known_answers.json"), "w"), indent=1)
    print("known answers:", len(known))

    # ---------------- all-pairs data tests: tests/tests.cu:463-551 ----------------
    seqs, cases, jobs = {}, [], []
    for kind, alpha, A, gap, flag in (("dna", DNA, 4, 11, "--dna"), ("protein", PROT, 23, 5, "--protein")):
        d = f"{REF}/data/{kind}"
        names = sorted(os.listdir(d))
        enc = {nm: encode_file(os.path.join(d, nm), alpha) for nm in names}
        for nm in names:
            seqs[f"{kind}/{nm}"] = letters(enc[nm], A)
        mat = mats["blast"] if A == 4 else mats["blosum50"]
        for i in range(len(names)):
            for j in range(i + 1, len(names)):
                t, p = enc[names[i]], enc[names[j]]
                if len(t) < len(p):
                    t, p = p, t
                    tn, pn = names[j], names[i]
                else:
                    tn, pn = names[i], names[j]
                if len(t) > 20000:  # tests.cu:486-487
                    continue
                for mode in (0, 1):
                    cases.append({"text": f"{kind}/{tn}", "pattern": f"{kind}/{pn}", "mode": mode, "A": A, "gap": gap,
                                  "matrix": "blast" if A == 4 else "blosum50"})
                    jobs.append((mode, t, p, mat, gap))
        # spot-check the encoding restatement against the reference parser
        for nm in names[:6]:
            req = ref_parse([flag, os.path.join(d, nm), os.path.join(d, nm)])
            assert list(req["text"]) == [int(x) for x in enc[nm]], nm
    for c, r in zip(cases, run_jobs(jobs)):
        c["result"] = result_record(r)
    used = {c["text"] for c in cases} | {c["pattern"] for c in cases}
    seqs = {k: v for k, v in seqs.items() if k in used}
    json.dump({"sequences": seqs, "cases": cases}, open(os.path.join(HERE, "data_pairs.json"), "w"))
    print("data pairs:", len(cases))

    # ---------------- random / edge pairs ----------------
    rng = np.random.default_rng(20261015)
    edge = [1, 2, 3, 4, 7, 31, 32, 33, 63, 64, 65, 66, 127, 128, 129, 255, 256, 257, 511, 512, 513, 1000]
    rcases, jobs = [], []

    def add(mode, t, p, mat_name, mat, gap, tag, ref_ok=True):
        A = 4 if len(mat) == 16 else 23
        rcases.append({"mode": mode, "A": A, "gap": gap, "matrix": mat_name if mat_name else mat,
                       "text": letters(t, A), "pattern": letters(p, A), "tag": tag, "by": "reference" if ref_ok else "oracle"})
        jobs.append((mode, t, p, mat, gap, ref_ok))

    for mode in (0, 1):
        for L1 in edge:
            for L2 in (1, 5, 64, 65, 130, 300):
                n, m = max(L1, L2), min(L1, L2)
                t = rng.integers(0, 4, n).astype(np.int8)
                p = rng.integers(0, 4, m).astype(np.int8)
                add(mode, t, p, "blast", mats["blast"], int(rng.choice([1, 5, 11])), "edge_dna")
        for _ in range(60):
            n = int(rng.integers(1, 700)); m = int(rng.integers(1, n + 1))
            t = rng.integers(0, 4, n).astype(np.int8)
            p = synthetic.mutate(t, int(rng.integers(1 << 30)), 4, m)
            add(mode, t, p, "blast", mats["blast"], int(rng.choice([1, 2, 5, 11])), "mutated_dna")
        for _ in range(30):
            n = int(rng.integers(1, 400)); m = int(rng.integers(1, n + 1))
            t = rng.integers(0, 4, n).astype(np.int8); p = rng.integers(0, 4, m).astype(np.int8)
            add(mode, t, p, "dnaMat", mats["dnaMat"], int(rng.choice([1, 2, 3])), "dnamat")
        for bl in ("blosum50", "blosum62", "blosum30", "blosum80"):
            for _ in range(12):
                n = int(rng.integers(1, 500)); m = int(rng.integers(1, n + 1))
                t = rng.integers(0, 20, n).astype(np.int8)
                p = synthetic.mutate(t, int(rng.integers(1 << 30)), 20, m) if rng.random() < 0.5 else rng.integers(0, 23, m).astype(np.int8)
                add(mode, t, p, bl, mats[bl], int(rng.choice([1, 5, 10, 11])), "protein")
        # asymmetric and wide-range matrices (orientation S[pattern*A+text]; values beyond int8)
        for _ in range(12):
            A = int(rng.choice([4, 23]))
            S = rng.integers(-300, 300, (A, A)).astype(np.int32).ravel().tolist()
            n = int(rng.integers(1, 300)); m = int(rng.integers(1, n + 1))
            add(mode, rng.integers(0, A, n).astype(np.int8), rng.integers(0, A, m).astype(np.int8), None, S,
                int(rng.integers(1, 200)), "asym_wide")
        for _ in range(12):
            A = int(rng.choice([4, 23]))
            S = rng.integers(-9, 12, (A, A)).astype(np.int32).ravel().tolist()
            n = int(rng.integers(1, 300)); m = int(rng.integers(1, n + 1))
            add(mode, rng.integers(0, A, n).astype(np.int8), rng.integers(0, A, m).astype(np.int8), None, S,
                int(rng.integers(1, 8)), "asym_small")
        # degenerate / tie-heavy inputs
        for n, m in ((300, 200), (129, 64), (64, 64), (1, 1), (70, 3)):
            add(mode, np.zeros(n, np.int8), np.ones(m, np.int8), "blast", mats["blast"], 5, "poly_mismatch")
            add(mode, np.zeros(n, np.int8), np.zeros(m, np.int8), "blast", mats["blast"], 5, "poly_match")
            add(mode, np.tile(np.array([0, 1], np.int8), n)[:n], np.tile(np.array([1, 0], np.int8), m)[:m], "dnaMat",
                mats["dnaMat"], 1, "alternating_ties")
        # pattern longer than text: beyond the reference CLI's contract (its buffers are 2*text);
        # expectations from the C oracle restatement, the same algorithm with n+m output buffers.
        for _ in range(20):
            m = int(rng.integers(2, 300)); n = int(rng.integers(1, m))
            add(mode, rng.integers(0, 4, n).astype(np.int8), rng.integers(0, 4, m).astype(np.int8), "blast",
                mats["blast"], int(rng.choice([1, 5])), "text_shorter", ref_ok=False)
    ref_jobs = [(m, t, p, S, g) for m, t, p, S, g, ok in jobs if ok]
    ref_res = iter(run_jobs(ref_jobs))
    for c, (m, t, p, S, g, ok) in zip(rcases, jobs):
        r = next(ref_res) if ok else oracle.align(m, t, p, np.array(S, np.int32), g)
        c["result"] = result_record(r, full_max=10**6)
    json.dump(rcases, open(os.path.join(HERE, "random_pairs.json"), "w"))
    print("random pairs:", len(rcases))

    # ---------------- config-sized cases (BASELINE.json configs 2-5) ----------------
    big = []
    specs = [
        ("cfg2_dna_global_8192_uniform", 0, 8192, 8192, ("rand", 3), ("rand", 4), "blast", 5, 4),
        ("cfg2_dna_global_8192_mutated", 0, 8192, 8192, ("rand", 3), ("mut", 5), "blast", 5, 4),
        ("cfg3_dna_local_32768_uniform", 1, 32768, 32768, ("rand", 6), ("rand", 7), "blast", 5, 4),
        ("cfg3_dna_local_32768_mutated", 1, 32768, 32768, ("rand", 6), ("mut", 8), "blast", 5, 4),
        ("headline_dna_global_32768_uniform", 0, 32768, 32768, ("rand", 6), ("rand", 7), "blast", 5, 4),
        ("cfg4_protein_global_4096_blosum50", 0, 4096, 4096, ("rand", 9), ("rand", 10), "blosum50", 5, 20),
        ("cfg4_protein_global_4096_blosum62", 0, 4096, 4096, ("rand", 9), ("rand", 10), "blosum62", 5, 20),
        ("cfg4_protein_global_4096_rand22", 0, 4096, 4096, ("rand", 11), ("rand", 12), "blosum50", 5, 22),
        ("cfg4_protein_local_4096_blosum50", 1, 4096, 4096, ("rand", 9), ("mut", 13), "blosum50", 5, 20),
    ]
    for i in range(8):
        specs.append((f"cfg5_batch_pair_{i}", 0, 2048, 2048, ("rand", 1000 + 2 * i), ("rand", 1001 + 2 * i), "blast", 5, 4))
    big_jobs = []
    for name, mode, n, m, ts, ps, mat, gap, A in specs:
        t = synthetic.random_sequence(ts[1], n, A)
        p = synthetic.random_sequence(ps[1], m, A) if ps[0] == "rand" else synthetic.mutate(t, ps[1], A, m)
        big.append({"name": name, "mode": mode, "n": n, "m": m, "text_seed": ts[1], "pattern_kind": ps[0],
                    "pattern_seed": ps[1], "matrix": mat, "gap": gap, "letters": A})
        big_jobs.append((mode, t, p, mats[mat], gap))
    # the 32k cases are checked against the reference only (the C oracle would double the time)
    ref = oracle.ref_align_batch([(m, t, p, np.array(S, np.int32), g) for m, t, p, S, g in big_jobs])
    for b, r in zip(big, ref):
        b["result"] = result_record(r, full_max=0)
        print(b["name"], b["result"]["score"], b["result"]["num_bytes"])
    json.dump(big, open(os.path.join(HERE, "large.json"), "w"), indent=1)

    # ---------------- CLI, config 1 (BASELINE.json configs[0]) ----------------
    cdir = os.path.join(HERE, "cli")
    os.makedirs(cdir, exist_ok=True)
    a = letters(synthetic.random_sequence(1, 1024, 4), 4)
    b = letters(synthetic.random_sequence(2, 1024, 4), 4)
    open(os.path.join(cdir, "a.txt"), "w").write(">config1 text, splitmix64 seed 1\n" + "\n".join(a[i:i + 70] for i in range(0, 1024, 70)) + "\n")
    open(os.path.join(cdir, "b.txt"), "w").write(">config1 pattern, splitmix64 seed 2\n" + "\n".join(b[i:i + 70] for i in range(0, 1024, 70)) + "\n")
    clis = {
        "config1": ["-d", "-c", "--global", "A", "B"],
        "config1_local": ["-d", "-c", "--local", "A", "B"],
        "config1_gap11": ["--gap-penalty", "11", "--global", "A", "B"],
        "protein_p02232_p03989": ["-p", "--local", f"{REF}/data/protein/P02232.fasta", f"{REF}/data/protein/P03989.fasta"],
        "dna_01_02": ["--gap-penalty", "5", "--global", f"{REF}/data/dna/dna_01.txt", f"{REF}/data/dna/dna_02.txt"],
    }
    cli_out = {}
    for name, args in clis.items():
        args = [os.path.join(cdir, "a.txt") if x == "A" else os.path.join(cdir, "b.txt") if x == "B" else x for x in args]
        r = subprocess.run([oracle.REF_BIN, "cli", *args], cwd=REF, capture_output=True, text=True, check=True)
        shown = [x.replace(cdir + "/", "").replace(REF + "/", "") for x in args]
        cli_out[name] = {"args": shown, "stdout": r.stdout}
    json.dump(cli_out, open(os.path.join(cdir, "expected.json"), "w"), indent=1)
    # the data files the CLI cases read (fixtures: data the reference's own tests hold)
    for rel in ("data/protein/P02232.fasta", "data/protein/P03989.fasta", "data/dna/dna_01.txt", "data/dna/dna_02.txt"):
        os.makedirs(os.path.join(cdir, os.path.dirname(rel)), exist_ok=True)
        open(os.path.join(cdir, rel), "wb").write(open(os.path.join(REF, rel), "rb").read())
    print("cli cases:", len(cli_out))


if __name__ == "__main__":
    main()
