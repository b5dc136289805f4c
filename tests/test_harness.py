"""sa_benchmarks, the reference's benchmark harness modes (tests/benchmarks.cu:102-363): every mode
prints its human-readable block and, with --json, one JSON line per size and device. CPU runs here;
the GPU legs (gpu marker) run the same modes through the MI355X engine."""
from __future__ import annotations

import json
import os
import subprocess
import sys

import pytest

from conftest import PKG

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(PKG, "bin", "sa_benchmarks")
sys.path.insert(0, os.path.join(ROOT, "tools"))


@pytest.fixture(scope="module")
def workdir(tmp_path_factory):
    import score_matrices
    d = tmp_path_factory.mktemp("harness")
    score_matrices.write(str(d))
    return str(d)


def _run(workdir, *args, timeout=120):
    r = subprocess.run([BIN, *args, "--json"], cwd=workdir, capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, r.stderr
    assert "could not parse" not in r.stderr
    return r.stdout, [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")]


@pytest.mark.parametrize("kind", ["global", "local"])
def test_throughput_cpu(workdir, kind):
    out, lines = _run(workdir, "throughput", kind, "--no-gpu", "--cpu", "--repeats", "1", "--sizes", "256x512,512x256")
    assert f"{kind.capitalize()} alignment benchmark:" in out and "MCUPS:" in out
    assert [(l["rows"], l["cols"], l["device"]) for l in lines] == [(256, 512, "cpu"), (512, 256, "cpu")]
    assert all(l["mcups"] > 0 for l in lines)


def test_latency_and_batch_cpu(workdir):
    _, lines = _run(workdir, "latency", "global", "--no-gpu", "--cpu", "--repeats", "1", "--sizes", "300x200")
    assert len(lines) == 1 and lines[0]["mode"] == "latency" and lines[0]["us"] > 0
    _, lines = _run(workdir, "batch", "3", "local", "--no-gpu", "--cpu", "--sizes", "256x256")
    assert len(lines) == 1 and lines[0]["mode"] == "batch" and lines[0]["type"] == "Local"


def test_usage_errors(workdir):
    for args in ([], ["nonsense"], ["batch"], ["throughput", "--bogus"]):
        r = subprocess.run([BIN, *args], cwd=workdir, capture_output=True, text=True)
        assert r.returncode == 2 and "usage" in r.stderr


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["global", "local"])
def test_harness_gpu_modes(workdir, kind):
    _, lines = _run(workdir, "throughput", kind, "--cpu", "--repeats", "2", "--sizes", "1024x1024,2048x4096")
    assert {(l["rows"], l["device"]) for l in lines} == {(1024, "cpu"), (1024, "gpu"), (2048, "cpu"), (2048, "gpu")}
    _, lines = _run(workdir, "latency", kind, "--repeats", "1", "--sizes", "4096x4096")
    assert lines[0]["device"] == "gpu" and lines[0]["us"] > 0
    _, lines = _run(workdir, "batch", "2", kind, "--sizes", "2048x2048")
    assert lines[0]["mode"] == "batch"
    _, lines = _run(workdir, "maxlength", kind, "--sizes", "30000x30000")
    assert lines[0]["mcups"] > 1000
