"""The alignSequence CLI drop-in (mainDriver.cu / utilities.cpp) against the reference's exact stdout
(tests/golden/cli/expected.json, produced by the reference binary). `-c` runs on CPU here; `-g` is the
same command through the MI355X engine (gpu marker)."""
from __future__ import annotations

import json
import os
import subprocess

import pytest

from conftest import GOLDEN, PKG, load

CLI = os.path.join(PKG, "bin", "alignSequence")
CDIR = os.path.join(GOLDEN, "cli")


@pytest.fixture(scope="module")
def workdir(tmp_path_factory):
    """A cwd holding scoreMatrices/ (the CLI loads its default matrices by relative path)."""
    d = tmp_path_factory.mktemp("cli")
    mats = load("matrices.json")
    for sub, name, A in (("dna", "blast", 4), ("dna", "dnaMat", 4), ("protein", "blosum50", 23),
                         ("protein", "blosum62", 23)):
        os.makedirs(d / "scoreMatrices" / sub, exist_ok=True)
        v = mats[name]
        (d / "scoreMatrices" / sub / f"{name}.txt").write_text(
            "\n".join(" ".join(str(x) for x in v[r * A:(r + 1) * A]) for r in range(A)) + "\n")
    return str(d)


def _args(case, device):
    out = []
    for a in case["args"]:
        if a in ("-c", "--cpu"):
            continue
        out.append(a if a.startswith("-") or a.lstrip("-").isdigit() else os.path.join(CDIR, a))
    return [device] + out


CASES = json.load(open(os.path.join(CDIR, "expected.json")))


@pytest.mark.parametrize("name", sorted(CASES))
def test_cli_cpu_device_matches_reference_stdout(workdir, name):
    r = subprocess.run([CLI, *_args(CASES[name], "-c")], cwd=workdir, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    assert r.stdout == CASES[name]["stdout"]


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(CASES))
def test_cli_gpu_device_matches_reference_stdout(workdir, name):
    r = subprocess.run([CLI, *_args(CASES[name], "-g")], cwd=workdir, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout == CASES[name]["stdout"]


def test_cli_usage_and_errors(workdir, tmp_path):
    r = subprocess.run([CLI], cwd=workdir, capture_output=True, text=True)
    assert r.returncode == 1 and r.stderr.startswith("Usage: ./alignSequence")
    r = subprocess.run([CLI, "-p", "-c"], cwd=workdir, capture_output=True, text=True)
    assert r.returncode == 1 and r.stderr.startswith("error: text sequence or pattern sequence not read\nUsage:")
    bad = tmp_path / "corrupt.txt"
    bad.write_text("1 2 3\n4 x 6\n")
    r = subprocess.run([CLI, "--score-matrix", str(bad), os.path.join(CDIR, "data/dna/dna_01.txt"),
                        os.path.join(CDIR, "data/dna/dna_02.txt")], cwd=workdir, capture_output=True, text=True)
    assert r.returncode == 1 and r.stderr == "error: matrix scores not read. Only integer scores accepted (int)\n"
    r = subprocess.run([CLI, "--gap-penalty", "x", "a", "b"], cwd=workdir, capture_output=True, text=True)
    assert r.returncode == 1 and r.stderr == "error: gap penalty not read. Only integer scores accepted (int)\n"
