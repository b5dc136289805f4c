"""The reference's own C++ callers on this repository's API (the drop-in boundary).

oracle/build_ref_callers.sh compiles the reference's tests/tests.cu (Catch2) unchanged against
include/SequenceAlignment.hpp and links libsequence_alignment.so + libsa_hip.so
(-> oracle/_ref/ref_tests_api). It runs from a scratch working directory holding the reference's
test data (tests/golden/refdata, make_refdata.py) and its score matrices (tools/score_matrices.py),
since tests.cu opens them by relative path (tests/tests.cu:47, :56, :103, :465, :510).

CPU: the six CPU TEST_CASEs (tests/tests.cu:35-366, 32 assertions: parsing, known-answer
alignments); the -DBENCHMARK harness contract compiles to the fill-only entry point.
GPU: the GPU TEST_CASEs (tests/tests.cu:370-551: known answers and every data-file pair, our
alignSequenceGPU vs alignSequenceCPU) and the benchmark contract run.
"""
from __future__ import annotations

import os
import re
import shutil
import subprocess
import sys

import pytest

from conftest import GOLDEN, PKG, ROOT

BIN = os.path.join(ROOT, "oracle", "_ref", "ref_tests_api")
CPU_CASES = ["indexOfLetter", "parseScoreMatrixFile", "readSequenceBytes", "parseArguments",
             "alignSequenceCPU - Global", "alignSequenceCPU - Local"]
GPU_CASES = ["alignSequenceGPU - Global", "alignSequenceGPU - Local", "Batch DNA alignment",
             "Batch Protein alignment"]


@pytest.fixture(scope="module")
def ref_cwd(tmp_path_factory):
    if not os.path.exists(BIN):
        if os.path.isdir(os.environ.get("SA_REFERENCE", "/root/reference")):
            subprocess.run([os.path.join(ROOT, "oracle", "build_ref_callers.sh")], check=True)
        else:
            pytest.skip("oracle/_ref/ref_tests_api not built (needs the reference mounted at build time)")
    d = tmp_path_factory.mktemp("refcwd")
    shutil.copytree(os.path.join(GOLDEN, "refdata", "data"), d / "data")
    shutil.copytree(os.path.join(GOLDEN, "refdata", "tests"), d / "tests")
    subprocess.run([sys.executable, os.path.join(ROOT, "tools", "score_matrices.py"), str(d)], check=True)
    return d


def _run(cwd, cases) -> dict:
    out = subprocess.run([BIN, ",".join(cases)], cwd=cwd, capture_output=True, text=True, timeout=600)
    tail = out.stdout[-3000:] + out.stderr[-2000:]
    m = re.search(r"All tests passed \((\d+) assertions? in (\d+) test cases?\)", out.stdout)
    assert out.returncode == 0 and m, tail
    return {"assertions": int(m.group(1)), "cases": int(m.group(2))}


def test_reference_cpu_test_cases(ref_cwd):
    r = _run(ref_cwd, CPU_CASES)
    assert r == {"assertions": 32, "cases": 6}


def test_benchmark_macro_maps_to_fill_only_entry_point():
    exe = os.path.join(PKG, "bin", "sa_benchmark_contract")
    out = subprocess.run(["nm", "-C", exe], capture_output=True, text=True, check=True).stdout
    assert "SequenceAlignment::alignSequenceGPUFillMicros(" in out
    assert "SequenceAlignment::alignSequenceGPU(" not in out


@pytest.mark.gpu
def test_reference_gpu_test_cases(ref_cwd):
    r = _run(ref_cwd, GPU_CASES)
    # 4 GPU known-answer sections + the two all-pairs batch cases over the data files
    assert r["cases"] == 4 and r["assertions"] > 500, r


@pytest.mark.gpu
def test_benchmark_macro_contract_runs():
    out = subprocess.run([os.path.join(PKG, "bin", "sa_benchmark_contract"), "4097", "4097"], capture_output=True,
                         text=True, timeout=120)
    assert out.returncode == 0, out.stdout + out.stderr
    assert '"response_untouched": true' in out.stdout
