"""CPU: the C-ABI library loads and exports every symbol include/sa_hip.h declares; the C++ library
exports the SequenceAlignment API; synthetic inputs are deterministic. No compute calls (no GPU here)."""
from __future__ import annotations

import ctypes
import os
import re
import subprocess

import numpy as np

from conftest import PKG, ROOT
from sa_amd import synthetic


def _declared(header: str) -> list[str]:
    src = open(os.path.join(ROOT, "include", header)).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(sa_[a-z_]+)\s*\(", src)))


def test_c_abi_exports_every_declared_symbol():
    lib = ctypes.CDLL(os.path.join(PKG, "lib", "libsa_hip.so"))
    names = _declared("sa_hip.h")
    assert len(names) >= 12
    for name in names:
        assert hasattr(lib, name), name
    assert lib.sa_abi_version() == 1


def test_python_binding_covers_the_abi():
    from sa_amd import engine
    assert set(engine.EXPORTS) == set(_declared("sa_hip.h"))


def test_cpp_api_symbols():
    out = subprocess.run(["nm", "-D", "-C", os.path.join(PKG, "lib", "libsequence_alignment.so")],
                         capture_output=True, text=True, check=True).stdout
    for sym in ("SequenceAlignment::alignSequenceGPU(", "SequenceAlignment::alignSequenceCPU(",
                "SequenceAlignment::alignSequenceGPUFillMicros(", "SequenceAlignment::traceBackNW(",
                "SequenceAlignment::traceBackSW(", "parseArguments(", "prettyAlignmentPrint(",
                "validateAndTransform(", "parseScoreMatrixFile(", "readSequenceFile(", "indexOfLetter(",
                "fillMatrixNW(", "fillMatrixSW("):
        assert sym in out, sym


def test_engine_gfx950_code_object():
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-objdump", "--offloading", os.path.join(PKG, "lib", "libsa_hip.so")],
                         capture_output=True, text=True)
    txt = out.stdout + out.stderr
    assert "gfx950" in txt


def test_synthetic_is_deterministic():
    a = synthetic.random_sequence(3, 1000, 4)
    b = synthetic.random_sequence(3, 1000, 4)
    assert (a == b).all() and a.min() >= 0 and a.max() <= 3
    assert abs(np.bincount(a, minlength=4) / 1000 - 0.25).max() < 0.06
    m = synthetic.mutate(a, 5, 4, 1000)
    assert len(m) == 1000 and (m == synthetic.mutate(a, 5, 4, 1000)).all()
    # roughly 88 % of the letters survive unchanged in order
    assert (m[:300] == a[:300]).mean() < 1.0


def test_build_id_matches_sources_and_detects_an_edit(tmp_path):
    """Build provenance: libsa_hip.so reports the hash of the sources it was built from
    (sa_build_id, python/sa_amd/buildid.py) and the hash changes with any byte of csrc/."""
    import shutil
    from sa_amd import buildid
    L = ctypes.CDLL(os.path.join(PKG, "lib", "libsa_hip.so"))
    L.sa_build_id.restype = ctypes.c_char_p
    assert L.sa_build_id().decode() == buildid.source_hash()
    assert buildid.library_id(os.path.join(PKG, "lib", "libsa_hip.so")) == buildid.source_hash()
    # a copy of the sources with one byte changed hashes differently
    pkg2, root2 = tmp_path / "repo" / "sequence-alignment-gpu_amd", tmp_path / "repo"
    shutil.copytree(os.path.join(PKG, "csrc"), pkg2 / "csrc")
    shutil.copytree(os.path.join(ROOT, "include"), root2 / "include")
    shutil.copy(os.path.join(PKG, "Makefile"), pkg2 / "Makefile")
    same = buildid.source_hash(str(pkg2), str(root2))
    assert same == buildid.source_hash()
    f = pkg2 / "csrc" / "sa_walk.h"
    b = bytearray(f.read_bytes())
    b[-2] ^= 0x01
    f.write_bytes(bytes(b))
    assert buildid.source_hash(str(pkg2), str(root2)) != same
