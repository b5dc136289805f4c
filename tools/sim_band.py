#!/usr/bin/env python3
"""CPU check of the band fill's generated score steps (development tool): interprets the inline asm
of band_steps_asm<LOCAL, HN, HP> from sa_fill_steps.inc (the VALU / DPP subset it uses) over 64
lanes, drives it the way process_band does (16-step bodies, text-profile bytes, the feed queue, the
publish shift), and compares every band's published bottom row with a direct DP of the same rows:
global in the shifted domain F = H + g(i + j) (alignSequenceCPU.cpp:259-273), local H
(:175-190). Catches register-rotation and hazard-order mistakes in tools/gen_fill_asm.py without a
GPU.   python3 tools/sim_band.py
"""
import os
import re
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
INC = os.path.join(ROOT, "sequence-alignment-gpu_amd", "csrc", "sa_fill_steps.inc")


def band_asm(local: bool, hn: bool, hp: bool) -> list:
    src = open(INC).read()
    key = f"band_steps_asm<{str(local).lower()}, {str(hn).lower()}, {str(hp).lower()}>(BandRegs &r)"
    i = src.index(key)
    body = src[src.index('asm volatile("', i) + len('asm volatile("'):]
    body = body[: body.index('"\n')]
    return [x.strip() for x in body.split("\\n\\t")]


def sext8(v):
    v = v & 0xFF
    return np.where(v >= 128, v - 256, v)


def run(lines, regs, g):
    """Executes the instruction list on regs (name -> int64 array of 64 lanes)."""
    for ins in lines:
        op = ins.split()[0]
        args = [a.strip() for a in ins[len(op):].split(",")]
        if op in ("s_nop", "ds_read_b32", "ds_write_b32", "s_waitcnt", "v_bitop3_b32", "v_cmp_gt_i32_e64", "s_and_b64"):
            continue
        if op == "v_add_u32_sdwa":
            d, a = args[0], args[1]
            b = re.match(r"sext\((%\[\w+\])\)", args[2]).group(1)
            k = int(re.search(r"src1_sel:BYTE_(\d)", ins).group(1))
            regs[d] = (regs[a] + sext8(regs[b] >> (8 * k))).astype(np.int64)
        elif op == "v_mov_b32_dpp":
            d, s = args[0], args[1].split()[0]
            src = regs[s].copy()
            old = regs.get(d, np.zeros(64, np.int64)).copy()
            bc = "bound_ctrl:1" in ins
            out = old.copy()
            if "wave_shl:1" in ins:
                out[:63] = src[1:]
                out[63] = 0 if bc else old[63]
            elif "wave_shr:1" in ins:
                out[1:] = src[:63]
                out[0] = 0 if bc else old[0]
            else:
                raise SystemExit("dpp " + ins)
            regs[d] = out
        elif op == "v_max3_i32":
            d, a, b, c = args[0], args[1], args[2], args[3]
            regs[d] = np.maximum(np.maximum(regs[a], regs[b]), regs[c])
        elif op == "v_sub_u32_e64":
            d, a = args[0], args[1]
            assert ins.endswith("clamp")
            regs[d] = np.maximum(regs[a] - g, 0)
        else:
            raise SystemExit("unsupported " + ins)


def dp(mode, t, p, S, g):
    """Global: shifted-domain F (boundaries 0); local: H. (m+1) x (n+1)."""
    m, n = len(p), len(t)
    F = np.zeros((m + 1, n + 1), np.int64)
    for i in range(1, m + 1):
        for j in range(1, n + 1):
            if mode == 0:
                F[i, j] = max(F[i - 1, j - 1] + S[p[i - 1], t[j - 1]] + 2 * g, F[i, j - 1], F[i - 1, j])
            else:
                F[i, j] = max(0, F[i - 1, j - 1] + S[p[i - 1], t[j - 1]], F[i, j - 1] - g, F[i - 1, j] - g)
    return F


def bands(mode, t, p, S, g):
    """Published bottom rows of bands 0 .. B-2 (process_band), columns 1..n."""
    m, n = len(p), len(t)
    off = 2 * g if mode == 0 else g
    U = 16
    nsteps = ((n + 64) + 2 * U - 1) // (2 * U) * (2 * U)
    lane = np.arange(64)
    B = (m + 127) // 128
    feed_row = None  # the band above's bottom row, columns 1..n
    out = []
    for b in range(B - 1):
        hp = b > 0
        lines = band_asm(mode == 1, True, hp)
        rows = [128 * b + 2 * lane, 128 * b + 2 * lane + 1]  # 0-based pattern index of the lane's rows
        Q = np.zeros(64, np.int64)
        diag = np.zeros(64, np.int64)
        F0 = np.zeros(64, np.int64)
        F1 = np.zeros(64, np.int64)
        pub = np.zeros(n + 1, np.int64)

        def feed(s):  # lanes 0..15: columns s+1 .. s+16 of the band above (0 past n / row 0)
            q = np.zeros(64, np.int64)
            if hp:
                c = s + 1 + lane[:U]
                ok = c <= n
                q[:U][ok] = feed_row[c[ok]]
            return q

        Q = feed(0)
        for s0 in range(0, nsteps, U):
            regs = {"%[p7]": Q, "%[p6]": diag, "%[p5]": F0, "%[p1]": F1}
            for nm in ("%[p0]", "%[p2]", "%[p3]", "%[p4]", "%[t0]"):
                regs[nm] = np.full(64, 12345, np.int64)  # garbage
            for r, pre in ((0, "ta"), (1, "tb")):
                for w in range(4):
                    word = np.zeros(64, np.int64)
                    for byte in range(4):
                        x = s0 + 4 * w + byte - lane  # text index of lane k at this step
                        ok = (x >= 0) & (x < n)
                        sc = np.zeros(64, np.int64)
                        sc[ok] = S[p[rows[r][ok]], t[x[ok]]] + off
                        word |= (sc & 0xFF) << (8 * byte)
                    regs[f"%[{pre}{w}]"] = word
            run(lines, regs, g)
            Q, diag, F0, F1 = regs["%[p7]"], regs["%[p6]"], regs["%[p5]"], regs["%[p1]"]
            # publish: lanes 48..63 of p0 = bottom row of columns s0-63 .. s0-48
            v = regs["%[p0]"]
            for l in range(48, 64):
                c = s0 - 63 + (l - 48)
                if 1 <= c <= n:
                    pub[c] = v[l]
            Q = feed(s0 + U)
        out.append(pub)
        feed_row = pub
    return out


def main():
    from_path = os.path.join(ROOT, "sequence-alignment-gpu_amd", "python")
    sys.path.insert(0, from_path)
    from sa_amd import synthetic
    S = synthetic.blast_matrix()
    bad = 0
    for mode, n, m, g in ((0, 150, 384, 5), (0, 97, 300, 0), (0, 120, 257, -2), (1, 150, 384, 5), (1, 90, 300, 0)):
        t = synthetic.random_sequence(11 + n, n, 4)
        p = synthetic.mutate(t, 12 + m, 4, m)
        F = dp(mode, t, p, S, g)
        got = bands(mode, t, p, S, g)
        for b, row in enumerate(got):
            r = 128 * (b + 1)
            d = int((row[1:] != F[r, 1:]).sum())
            if d:
                bad += 1
                print("mismatch mode", mode, "n", n, "m", m, "g", g, "band", b, "cells", d,
                      "first", int(np.argmax(row[1:] != F[r, 1:])) + 1)
        print("mode", mode, "n", n, "m", m, "g", g, "bands", len(got), "ok" if not bad else "BAD")
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
