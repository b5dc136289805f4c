#!/usr/bin/env python3
"""Generates sequence-alignment-gpu_amd/csrc/sa_split_steps.inc: the hand-scheduled steady bodies of
the SPLIT R = 1 fill (global mode, int8 text profiles), where every strip has two waves:

  score wave  the recurrence only (5 VALU per step, no direction bits), writing every step's F to an
              LDS "F ring" (one ds_write2_b32 per two steps);
  dir wave    reads the F ring and derives both direction bits of every cell (3 VALU per step plus
              the per-word merge), then stores the planes exactly as the one-wave kernel does.

Why: one wave issues at most one instruction per ~4.4 clocks whatever its kind, and a step of the
one-wave kernel was 7 VALU + 0.94 merge + per-body bookkeeping (about 10 instructions, 47 clk on the
chain). The strip's anti-diagonal chain is only the score wave's part; moving the direction work to a
sibling wave on another SIMD takes it off the critical path.

Score step k (four registers rotate through the roles Qn -> Q/up -> diag/F -> left, period 4, exactly
as tools/gen_fill_asm.py; see its docstring for the queue / publish trick):
    [k even >= 2: ds_write2_b32 F_{k-2}, F_{k-1}]   (F_{k-2} lives in the register Qn overwrites)
    Qn = wave_shl:1(Q)          (HN: lane 63 keeps F_{k-2}, the bottom row)
    D  = diag + sext(score byte)
    up = wave_shr:1(F_{k-1})    in place in Q (lane 0 keeps the feed)
    M  = max(F_{k-1}, up)
    F  = max(D, M)              (into the diag register)
Every DPP stays two instructions behind the VALU write of what it reads: up_k reads F_{k-1}, written by
step k-1's last op, with Qn_k and D_k (and the write) in between.

F ring (sa_split.inc): row r of a strip holds F of lane r at physical slot (step & 127) + 1, so a
body's 16 values are one run inside the row (slots up to 128); row -1 holds the strip's feed (lane 0's
`up`) at slot (step & 127), written by the score wave from Q. The write offsets below are relative to
the row base plus (s0 & 96) * 4 (the body pair's place in the ring).

Dir step i of a body (values from the F ring: O[i] = F_{s0+i-1} for i >= 1, U[i] = the lane above's
F_{s0+i-1} (lane 0: the feed of step s0+i), oc = F_{s0-1}, ex = F_{s0+15}):
    left = i ? O[i] : oc,  up = U[i],  F = i < 15 ? O[i+1] : ex
    M = max(left, up);  X byte = M - F (sign = DIAG: F = max(D, M) > M);  Y byte = left - up (raw TOP)
U[0] is wave_shr:1(oc) with lane 0 keeping the feed (the physical slot of F_{s0-1} may have wrapped).
The X / Y byte layout is the one-wave kernel's, so its merge (tools/gen_fill_asm.py) builds the words.
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from gen_fill_asm import merge  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.environ.get("SA_GEN_SPLIT_OUT") or os.path.join(ROOT, "sequence-alignment-gpu_amd", "csrc", "sa_split_steps.inc")
# timing ablation for experiment builds only (results wrong): no F-ring writes
NOWR = bool(os.environ.get("SA_GEN_SPLIT_NOWR"))
# timing ablations: WAR = write F_{k-1} twice (a register not overwritten right after the write);
# WR1 = every other write only
WAR = bool(os.environ.get("SA_GEN_SPLIT_WAR"))
WR1 = bool(os.environ.get("SA_GEN_SPLIT_WR1"))

U = 16
PF_STEP = int(os.environ.get("SA_GEN_SPLIT_PF_STEP", "12"))


def score_block(hn: bool, hp: bool, half: int, dc: bool) -> str:
    A, B, C, FA = "%[q]", "%[qn]", "%[dg]", "%[f]"
    D, M, T0, FRA = "%[d]", "%[m]", "%[t0]", "%[fra]"
    TW = [f"%[tw{i}]" for i in range(4)]
    PF, BAD, PFA, CTAG, PADDR, PTAG, MSB = "%[pf]", "%[bad]", "%[pfa]", "%[ctag]", "%[paddr]", "%[ptag]", "%[msb]"
    regs = [B, FA, C, A]  # entry: regs[3] = Q, regs[1] = F (left), regs[2] = diag, regs[0] dead

    def off(k):  # physical slot of step s0 + k relative to the pair base (s0 & 96)
        return 16 * half + k + 1

    out = ["s_nop 1"]
    if dc:
        # the dir wave's consumption word (F ring backpressure), waited for with the block's end
        out.append("ds_read_b32 %[dcv], %[dca]")
    for k in range(U):
        if hp and k == PF_STEP:
            out.append(f"ds_read_b32 {PF}, {PFA}")
        if k >= 2 and k % 2 == 0 and not NOWR and not (WR1 and k % 4 == 2):
            a0 = regs[(k - 3) % 4] if WAR else regs[k % 4]
            out.append(f"ds_write2_b32 {FRA}, {a0}, {regs[(k - 3) % 4]} offset0:{off(k - 2)} offset1:{off(k - 1)}")
        qd, qr, dg, fp = regs[k % 4], regs[(k - 1) % 4], regs[(k - 2) % 4], regs[(k - 3) % 4]
        if hn:
            out.append(f"v_mov_b32_dpp {qd}, {qr} wave_shl:1 row_mask:0xf bank_mask:0xf")
        else:
            out.append(f"v_mov_b32_dpp {qd}, {qr} wave_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:1")
        out.append(f"v_add_u32_sdwa {D}, {dg}, sext({TW[k >> 2]}) dst_sel:DWORD dst_unused:UNUSED_PAD "
                   f"src0_sel:DWORD src1_sel:BYTE_{k & 3}")
        out.append(f"v_mov_b32_dpp {qr}, {fp} wave_shr:1 row_mask:0xf bank_mask:0xf")
        out.append(f"v_max_i32_e32 {M}, {fp}, {qr}")
        out.append(f"v_max_i32_e32 {dg}, {D}, {M}")
    # F_14 (regs[0]) and F_15 (regs[1]); before the publish, which overwrites regs[0]
    if not NOWR:
        out.append(f"ds_write2_b32 {FRA}, {regs[0]}, {regs[1]} offset0:{off(14)} offset1:{off(15)}")
    if hp or dc:
        # wait for the reads only: LDS operations complete in order, and the F-ring writes issued
        # after the last read need not be waited for (a full drain exposed a write's latency per body)
        last_read = PF_STEP if hp else -1
        after = 0 if NOWR else sum(1 for k in range(U) if k >= 2 and k % 2 == 0 and k > last_read
                                   and not (WR1 and k % 4 == 2)) + 1
        out.append(f"s_waitcnt lgkmcnt({after})")
    if hp:
        out.append(f"v_bitop3_b32 {PF}, {PF}, {CTAG}, {MSB} bitop3:0xd2")
        out.append(f"v_cmp_gt_i32_e64 {BAD}, 0, {PF}")
        out.append(f"s_and_b64 {BAD}, {BAD}, 0xffff")
    if hn:
        out.append(f"v_mov_b32_dpp {regs[0]}, {regs[3]} wave_shl:1 row_mask:0xf bank_mask:0xf")
        out.append(f"v_bitop3_b32 {T0}, {regs[0]}, {PTAG}, {MSB} bitop3:0xf2")
        out.append(f"ds_write_b32 {PADDR}, {T0}")
    return "\\n\\t".join(out)


def score_operands(hn: bool, hp: bool, dc: bool):
    outs = ['[q] "+v"(r.Q)', '[qn] "=&v"(r.Qn)', '[dg] "+v"(r.diag)', '[f] "+v"(r.F)',
            '[d] "=&v"(D)', '[m] "=&v"(M)', '[t0] "=&v"(t0)']
    ins = [f'[tw{i}] "v"(r.T[{i}])' for i in range(4)] + ['[fra] "v"(r.fra)']
    if hp:
        outs += ['[pf] "=&v"(r.pf)', '[bad] "=&s"(r.bad)']
        ins += ['[pfa] "v"(r.pfaddr)', '[ctag] "s"(r.ctag)']
    if dc:
        outs += ['[dcv] "=&v"(r.dcv)']
        ins += ['[dca] "v"(r.dcaddr)']
    if hn:
        ins += ['[paddr] "v"(r.pubaddr)', '[ptag] "s"(r.pubtag)']
    if hn or hp:
        ins += ['[msb] "v"(r.msb)']
    return outs, ins


def dir_block(half: int) -> str:
    out = ["s_nop 1", "v_mov_b32_dpp %[u0], %[oc] wave_shr:1 row_mask:0xf bank_mask:0xf"]
    for i in range(U):
        g, byte = 4 * half + (i & 3), 3 - (i >> 2)
        sd = f"dst_sel:BYTE_{byte} dst_unused:UNUSED_PRESERVE src0_sel:DWORD src1_sel:DWORD"
        left = "%[oc]" if i == 0 else f"%[o{i}]"
        up = f"%[u{i}]"
        f = f"%[o{i + 1}]" if i < 15 else "%[ex]"
        out.append(f"v_max_i32_e32 %[m], {left}, {up}")
        out.append(f"v_sub_u32_sdwa %[x{g}], %[m], {f} {sd}")
        out.append(f"v_sub_u32_sdwa %[y{g}], {left}, {up} {sd}")
    return "\\n\\t".join(out)


def main():
    lines = [
        "// GENERATED by tools/gen_split_asm.py -- do not edit. Hand-scheduled steady bodies of the SPLIT",
        "// R = 1 kArr8 global fill (see the generator's docstring: score wave / dir wave, F ring layout).",
        "// score_asm<HN, HP, HALF, DC>(r): 16 steps of the score wave; dir_asm<HALF>(r): the direction",
        "// differences of 16 steps from the F ring; dir_merge_asm(r): the chunk's two words.",
        "#pragma once",
        "",
    ]
    for hn in (False, True):
        for hp in (False, True):
            for half in (0, 1):
                for dc in (False, True):
                    outs, ins = score_operands(hn, hp, dc)
                    lines.append(f"template <> __device__ __forceinline__ void score_asm<{str(hn).lower()}, "
                                 f"{str(hp).lower()}, {half}, {str(dc).lower()}>(ScoreRegs &r)")
                    lines.append("{")
                    lines.append("    int D, M, t0;")
                    lines.append(f"    asm volatile(\"{score_block(hn, hp, half, dc)}\"")
                    lines.append("        : " + ", ".join(outs))
                    lines.append("        : " + ", ".join(ins) + (" : \"scc\");" if hp else ");"))
                    lines.append("    (void)D; (void)M; (void)t0;")
                    lines.append("}")
                    lines.append("")
    for half in (0, 1):
        outs = [f'[x{g}] "+v"(r.X[{g}])' for g in range(8)] + [f'[y{g}] "+v"(r.Y[{g}])' for g in range(8)]
        outs += ['[u0] "+v"(r.U[0])', '[m] "=&v"(M)']
        ins = ['[oc] "v"(r.oc)', '[ex] "v"(r.ex)'] + [f'[o{i}] "v"(r.O[{i}])' for i in range(1, 16)]
        ins += [f'[u{i}] "v"(r.U[{i}])' for i in range(1, 16)]
        lines.append(f"template <> __device__ __forceinline__ void dir_asm<{half}>(DirRegs &r)")
        lines.append("{")
        lines.append("    int M;")
        lines.append(f"    asm volatile(\"{dir_block(half)}\"")
        lines.append("        : " + ", ".join(outs))
        lines.append("        : " + ", ".join(ins) + ");")
        lines.append("    (void)M;")
        lines.append("}")
        lines.append("")
    outs = ['[a0] "=&v"(r.acc0)', '[a1] "=&v"(r.acc1)', '[tx] "=&v"(tx)']
    ins = [f'[x{g}] "v"(r.X[{g}])' for g in range(8)] + [f'[y{g}] "v"(r.Y[{g}])' for g in range(8)]
    ins += [f'[mk{g}] "v"(r.mk[{g}])' for g in range(8)]
    lines.append("__device__ __forceinline__ void dir_merge_asm(DirRegs &r)")
    lines.append("{")
    lines.append("    int tx;")
    lines.append(f"    asm volatile(\"{merge(False)}\"")
    lines.append("        : " + ", ".join(outs))
    lines.append("        : " + ", ".join(ins) + ");")
    lines.append("    (void)tx;")
    lines.append("}")
    lines.append("")
    open(OUT, "w").write("\n".join(lines))
    print("wrote", OUT)


if __name__ == "__main__":
    main()
