"""(CPU) The band fill's generated score steps (sa_fill_steps.inc band_steps_asm, tools/gen_fill_asm.py)
interpreted over 64 lanes the way process_band drives them (tools/sim_band.py): every band's published
bottom row equals a direct DP of the same rows, global (shifted domain, alignSequenceCPU.cpp:259-273)
and local (:175-190), gaps 5 / 0 (and -2 global). Checks the 8-register rotation, the DPP `old`
lanes and the publish shift without a GPU; the GPU tests check the kernel itself."""
from __future__ import annotations

import os
import subprocess
import sys

from conftest import ROOT


def test_band_steps_asm_interpreted_vs_dp():
    out = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "sim_band.py")], capture_output=True, text=True,
                         timeout=300)
    assert out.returncode == 0, out.stdout[-3000:] + out.stderr[-2000:]
    assert out.stdout.count(" ok") == 5, out.stdout
