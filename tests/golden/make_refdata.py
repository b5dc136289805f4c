#!/usr/bin/env python3
"""Copies the reference's own test data (data files its tests/tests.cu reads, relative to the reference
root) into tests/golden/refdata/, so that tests.cu — compiled against this repository's
include/SequenceAlignment.hpp by oracle/build_ref_callers.sh — runs from a scratch working directory
here and on the GPU box. Only the sequences tests.cu actually aligns are kept: its batch cases skip
every pair whose longer sequence exceeds 20000 letters (tests/tests.cu:484-486, :529-531), so files
longer than that contribute no checked pair. Data only; no reference source.
Run in the build container:  python tests/golden/make_refdata.py
"""
import os
import shutil
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REF = os.environ.get("SA_REFERENCE", "/root/reference")
OUT = os.path.join(HERE, "refdata")
sys.path.insert(0, HERE)
from make_golden import encode_file  # noqa: E402  (validateAndTransform restated)

LIMIT = 20000


def main() -> None:
    for sub, alphabet in (("dna", "ATCG"), ("protein", "ARNDCQEGHILKMFPSTWYVBZX")):
        src = os.path.join(REF, "data", sub)
        dst = os.path.join(OUT, "data", sub)
        os.makedirs(dst, exist_ok=True)
        for f in sorted(os.listdir(src)):
            if len(encode_file(os.path.join(src, f), alphabet)) <= LIMIT:
                shutil.copyfile(os.path.join(src, f), os.path.join(dst, f))
    os.makedirs(os.path.join(OUT, "tests"), exist_ok=True)
    shutil.copyfile(os.path.join(REF, "tests", "corruptScoreMatrix.txt"), os.path.join(OUT, "tests", "corruptScoreMatrix.txt"))
    print("refdata:", sorted(os.listdir(os.path.join(OUT, "data", "dna"))), sorted(os.listdir(os.path.join(OUT, "data", "protein"))))


if __name__ == "__main__":
    main()
