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


def test_ring_runs_never_cross_a_lap():
    """(CPU) The hand-off rings' addressing rule (sa_fill.hip ring_slot / ring_tag, kRing = 2048): a
    body's feed or publish covers columns s0 + 1 .. s0 + U (U = 16, s0 a multiple of U), and the
    shipped code masks each body's base slot and then addresses the body's 16 entries as one run, so
    that run must never cross the ring's wrap and must carry one lap tag. A run of a whole QUAD of
    bodies (64 entries from one base) holds that only when the quad starts on a 64-step boundary: the
    steady / tail phase boundary is a multiple of 2U = 32 steps only, so per-quad addressing (round
    5's 'pqn' experiment) let a quad starting at slot 2016 write and read slots 2048..2079 unwrapped,
    past the ring, while the other side wrapped: that hand-off never arrived (SA_ERR_TIMEOUT)."""
    kRing, U = 2048, 16
    slot = lambda c: (c + 63) & (kRing - 1)
    lap = lambda c: ((c + 63) >> 11) & 1
    for s0 in range(0, 3 * kRing + 4 * U, U):
        run = [slot(s0 + 1 + q) for q in range(U)]
        assert run == list(range(run[0], run[0] + U)), s0
        assert len({lap(s0 + 1 + q) for q in range(U)}) == 1, s0
    # quads from 32-step phase boundaries do cross the wrap (why per-quad bases need 64-step phases)
    crossing = [s0 for s0 in range(0, 2 * kRing, 2 * U) if slot(s0 + 1) + 4 * U > kRing]
    assert crossing and all(s0 % (4 * U) == 2 * U for s0 in crossing)
    assert not [s0 for s0 in range(0, 2 * kRing, 4 * U) if slot(s0 + 1) + 4 * U > kRing]
