#!/usr/bin/env python3
"""Generates sequence-alignment-gpu_amd/csrc/sa_fill_steps.inc: hand-scheduled inline-asm step blocks
of the R = 1 fill's steady bodies (text profiles as int8 bytes, kArr8), global and local, with and
without a strip below (HN), for the first and the second half of a 32-slot plane word (HALF), plus the
per-word merge of the direction bits.

Why asm: on gfx950 a DPP instruction must be 2 wait states behind the VALU write of any VGPR it
reads, and an s_nop costs an issue slot (4 cycles) like a VALU op. Scheduled by the compiler the
step's two lane moves landed right behind their producers (one to two s_nops per step, plus a
register copy for the bottom-row register); here every DPP sits at least two instructions behind its
inputs with independent work in between, so a step is exactly its VALU ops and nothing else.

One step (four registers rotate through the roles Qn -> Q/up -> diag/F' -> left, period 4):
    b   Qn = Q shifted down one lane (wave_shl:1), written into the register of F two steps back
        (dead); with HN its lane 63 keeps that step's bottom-row value F (sa_fill.hip run_body)
    c   Q = F shifted up one lane (wave_shr:1), in place: lane 0 keeps the feed value = `up`
    d   D = diag + sext(score byte)          (SDWA byte select of the text-profile word)
    e   M = max(left, up)                    left = F of the previous step
    f   global: F' = max(D, M) | local: X = max(D, M, g), F' = X - g, key
        (F' goes to the diag register, dead after d)
    g   X[4h + (k & 3)] byte 3 - (k >> 2) = M - D     (SDWA, other bytes kept: sign = DIAG)
    h   Y[4h + (k & 3)] byte 3 - (k >> 2) = left - up  (sign = raw "up > left" / raw TOP)
with k the step in the body and h = HALF the body's word of the 32-slot chunk. A difference's low
byte has the sign of the difference when the difference lies in [-128, 127]: the plan uses these
bodies only when every difference is bounded so (sa_engine.hip, byte_diffs). The R = 1 plane word
is INTERLEAVED (sa_layout.h): slot k of a word has DIAG at bit 31 - 2k and the second plane at bit
30 - 2k, so register r = 4h + t0 (steps t0, t0 + 4, t0 + 8, t0 + 12 in bytes 3..0) lands with one
shift: (X[r] & 0x80808080) >> 2 t0, (Y[r] & 0x80808080) >> (2 t0 + 1). The merge costs 15 VALU per
word and the sign bits 1 VALU per bit: about 2.94 VALU per step for two bits instead of 4 (one
subtraction and one v_alignbit per bit). Local stores the same two bits (DIAG, raw TOP): a STOP cell
is one whose H is 0, and the row walk recomputes H along the path (sa_walk.hip), so the planes need
no third bit (round 4 spent an ffbh per step and 9 more merge VALU per word on it).
A global step is 7 VALU ops (plus the merge) with or without a strip below: the queue's
bottom-row values run one step later than the C++ bodies' (whose Qn takes F of the previous step
through a register copy), and the publish at the body's end shifts the queue once more with F of
the step before last in lane 63, which gives the same 16 values (1 VALU per body instead of 16).
(Publishing the first 8 of them after step 8's shift as well does not shorten the hand-off: a
consumer's feed read takes a whole body's 16 columns, whose last 8 come with the body's end.)

Local keys: key' = (F' << kb) - q, its running maximum bm over the block (one v_max3 per two
steps: keys alternate between two registers); the caller adds the body's key base
(kmask - (s0 & kmask)) once per body. Same order as the C++ recurrence
(alignSequenceCPU.cpp:175-192): larger H first, then the earlier column.
"""
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.environ.get("SA_GEN_FILL_OUT") or os.path.join(ROOT, "sequence-alignment-gpu_amd", "csrc", "sa_fill_steps.inc")


U = 16
# with a strip above, the next body's feed read is issued after this step (kPfLead = U - PF_STEP)
PF_STEP = int(os.environ.get("SA_GEN_PF_STEP", "14"))
# the band fill's score steps (band_steps_asm) read the next feed after this step (kPfLead = U - it);
# a 44-clock step leaves two steps too little time for the LDS read (the R = 1 score steps of round 3
# measured 1 % faster after step 10 than after 14, profiles/r03/dual_dev/pf_timeline.log)
BAND_PF_STEP = int(os.environ.get("SA_GEN_BAND_PF_STEP", "10"))
# timing ablations of the strips' feed (experiment builds only, results wrong): "noread" replaces the
# feed read by a value that passes the tag check, "nocheck" keeps the read and its wait but reports
# every lane good
EXP_FEED = os.environ.get("SA_GEN_EXP_FEED", "")


def block(local: bool, hn: bool, hp: bool, half: int) -> str:
    # named operands (the C++ wrapper below binds them)
    A, B, C, FA = "%[q]", "%[qn]", "%[dg]", "%[f]"
    D, M, T0 = "%[d]", "%[m]", "%[t0]"
    X = [f"%[x{g}]" for g in range(8)]
    Y = [f"%[y{g}]" for g in range(8)]
    Z = [f"%[z{g}]" for g in range(8)]
    TW = [f"%[tw{i}]" for i in range(4)]
    G, KB, BM, XR, KEY, KEY2 = "%[g]", "%[kb]", "%[bm]", "%[xr]", "%[key]", "%[key2]"
    PF, BAD, PFA, CTAG, PADDR, PTAG, MSB = "%[pf]", "%[bad]", "%[pfa]", "%[ctag]", "%[paddr]", "%[ptag]", "%[msb]"
    # four registers rotate through the roles with period 4 (U = 16 returns them to their operands):
    # at step k, regs[k % 4] takes the shifted queue (Qn; it held F of step k-2, dead), regs[k-1] is
    # Q (shifted down, then overwritten in place by up), regs[k-2] is diag (then takes F'), regs[k-3]
    # is F of the previous step (left). Lane 63 of each Qn thus takes the bottom-row value of step
    # k-2 instead of k-1; the publish restores the order with one more shift whose `old` is F of the
    # step before last (lanes 64-U..63 = steps s0-1 .. s0+U-2, as the C++ bodies publish).
    regs = [B, FA, C, A]  # at entry: regs[3] = Q, regs[1] = F (left), regs[2] = diag, regs[0] dead
    out = []
    out.append("s_nop 1")  # the compiler's last writes of Q / F stand right before
    for k in range(U):
        q = k
        g, byte = 4 * half + (q & 3), 3 - (q >> 2)
        sd = f"dst_sel:BYTE_{byte} dst_unused:UNUSED_PRESERVE src0_sel:DWORD src1_sel:DWORD"
        qd, qr, dg, fp = regs[k % 4], regs[(k - 1) % 4], regs[(k - 2) % 4], regs[(k - 3) % 4]
        if hp and q == PF_STEP:
            if EXP_FEED == "noread":
                out.append(f"v_not_b32 {PF}, {CTAG}")
            else:
                out.append(f"ds_read_b32 {PF}, {PFA}")
        if hn:
            out.append(f"v_mov_b32_dpp {qd}, {qr} wave_shl:1 row_mask:0xf bank_mask:0xf")
        else:
            out.append(f"v_mov_b32_dpp {qd}, {qr} wave_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:1")
        out.append(f"v_mov_b32_dpp {qr}, {fp} wave_shr:1 row_mask:0xf bank_mask:0xf")
        out.append(f"v_add_u32_sdwa {D}, {dg}, sext({TW[q >> 2]}) dst_sel:DWORD dst_unused:UNUSED_PAD "
                   f"src0_sel:DWORD src1_sel:BYTE_{q & 3}")
        out.append(f"v_max_i32_e32 {M}, {fp}, {qr}")
        out.append(f"v_sub_u32_sdwa {Y[g]}, {fp}, {qr} {sd}")
        if not local:
            out.append(f"v_max_i32_e32 {dg}, {D}, {M}")
            out.append(f"v_sub_u32_sdwa {X[g]}, {M}, {D} {sd}")
        else:
            # H = max(X, g) - g = max(X - g, 0) for g > 0 and X - g (never 0 clamped) for g <= 0
            out.append(f"v_max3_i32 {XR}, {D}, {M}, {G}")
            out.append(f"v_sub_u32_sdwa {X[g]}, {M}, {D} {sd}")
            out.append(f"v_subrev_u32_e32 {dg}, {G}, {XR}")
            kreg = KEY if k % 2 == 0 else KEY2
            out.append(f"v_lshl_add_u32 {kreg}, {dg}, {KB}, {-q}")
            # (no STOP bits: a cell is STOP exactly when its H is 0, and the traceback follows H along
            # the path from the best cell's score, sa_walk.hip local_check)
            if k % 2 == 1:
                out.append(f"v_max3_i32 {BM}, {BM}, {KEY}, {KEY2}")
    if hp and EXP_FEED == "nocheck":
        out.append("s_waitcnt lgkmcnt(0)")
        out.append(f"v_bitop3_b32 {PF}, {PF}, {CTAG}, {MSB} bitop3:0xd2")
        out.append(f"s_mov_b64 {BAD}, 0")
    elif hp:
        out.append("s_waitcnt lgkmcnt(0)")  # the feed read (issued 4 steps ago) is there
        # tag check: x = entry ^ expected tag (the value when it matches; bitop3 0xD2 = a ^ (~b & c)),
        # bad lanes = x < 0 among the body's U feed lanes; the publish below stands between the
        # compare and the caller's SALU test of the mask
        out.append(f"v_bitop3_b32 {PF}, {PF}, {CTAG}, {MSB} bitop3:0xd2")
        out.append(f"v_cmp_gt_i32_e64 {BAD}, 0, {PF}")
        out.append(f"s_and_b64 {BAD}, {BAD}, 0xffff")
    if hn:
        # publish: the queue shifted once more into the register of F of the step before last (dead),
        # whose lane 63 keeps that step's bottom-row value; lanes 64-U..63 with the body's lap tag. The
        # write stays in flight past the block (the compiler sees no LDS operation it would wait for)
        out.append(f"v_mov_b32_dpp {regs[0]}, {regs[3]} wave_shl:1 row_mask:0xf bank_mask:0xf")
        out.append(f"v_bitop3_b32 {T0}, {regs[0]}, {PTAG}, {MSB} bitop3:0xf2")  # a | (~b & c)
        out.append(f"ds_write_b32 {PADDR}, {T0}")
    return "\\n\\t".join(out)


def band_block(local: bool, hn: bool, hp: bool) -> str:
    """U = 16 steps of a band score strip: two rows per lane (rows 2k, 2k+1 of a 128-row band), the
    recurrence alone (no direction bits). Eight registers P0..P7 rotate with period 8: at step k the
    register of phase p is P[(k - p) % 8], and the phases are
        p = 0  F1 of step k-2 (dead): the queue shift Qn is written here (lane 63 keeps F1, HN)
        p = 1  Q (the feed queue); up = wave_shr:1(F1 of step k-1) in place (lane 0 keeps the feed)
        p = 2  up of step k-1 (= diag of row 0): D0 = diag0 + S0 in place, then F0 = max3(D0, F0', up)
        p = 3  F0 of step k-1 (left of row 0, diag of row 1)
        p = 6  D1 = F0 of step k-1 + S1, then F1 = max3(D1, F1', F0)
        p = 7  F1 of step k-1 (left of row 1; the DPP's source)
        p = 4, 5  free
    (local: H = X - g saturated at 0, one v_sub_u32 with clamp after each max3; X >= 0). The up-DPP
    stands three instructions behind the max3 (and the subtract) that wrote F1, the queue shift two;
    a body of 16 steps returns every value to its register. 6 VALU per step (8 local)."""
    P = [f"%[p{i}]" for i in range(8)]
    T0 = [f"%[ta{i}]" for i in range(4)]
    T1 = [f"%[tb{i}]" for i in range(4)]
    G, T = "%[g]", "%[t0]"
    PF, BAD, PFA, CTAG, PADDR, PTAG, MSB = "%[pf]", "%[bad]", "%[pfa]", "%[ctag]", "%[paddr]", "%[ptag]", "%[msb]"
    out = ["s_nop 1"]  # the compiler's last writes of Q / F1 may stand right before
    for k in range(U):
        ph = lambda p: P[(k - p) % 8]
        sel = f"dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_{k & 3}"
        out.append(f"v_add_u32_sdwa {ph(2)}, {ph(2)}, sext({T0[k >> 2]}) {sel}")
        out.append(f"v_add_u32_sdwa {ph(6)}, {ph(3)}, sext({T1[k >> 2]}) {sel}")
        if hp and k == BAND_PF_STEP:
            out.append(f"ds_read_b32 {PF}, {PFA}")
        bc = "" if hn else " bound_ctrl:1"
        out.append(f"v_mov_b32_dpp {ph(0)}, {ph(1)} wave_shl:1 row_mask:0xf bank_mask:0xf{bc}")
        out.append(f"v_mov_b32_dpp {ph(1)}, {ph(7)} wave_shr:1 row_mask:0xf bank_mask:0xf")
        out.append(f"v_max3_i32 {ph(2)}, {ph(2)}, {ph(3)}, {ph(1)}")
        if local:
            out.append(f"v_sub_u32_e64 {ph(2)}, {ph(2)}, {G} clamp")
        out.append(f"v_max3_i32 {ph(6)}, {ph(6)}, {ph(7)}, {ph(2)}")
        if local:
            out.append(f"v_sub_u32_e64 {ph(6)}, {ph(6)}, {G} clamp")
    if hp:
        out.append("s_waitcnt lgkmcnt(0)")
        out.append(f"v_bitop3_b32 {PF}, {PF}, {CTAG}, {MSB} bitop3:0xd2")
        out.append(f"v_cmp_gt_i32_e64 {BAD}, 0, {PF}")
        out.append(f"s_and_b64 {BAD}, {BAD}, 0xffff")
    if hn:
        # k = 16: phase 0 = P0 holds F1 of step 14, phase 1 = P7 the queue: one more shift gives lanes
        # 48..63 = F1 of steps s0-1 .. s0+14 (as the one-wave bodies publish)
        out.append(f"v_mov_b32_dpp {P[0]}, {P[7]} wave_shl:1 row_mask:0xf bank_mask:0xf")
        out.append(f"v_bitop3_b32 {T}, {P[0]}, {PTAG}, {MSB} bitop3:0xf2")
        out.append(f"ds_write_b32 {PADDR}, {T}")
    return "\\n\\t".join(out)


def band_operands(local: bool, hn: bool, hp: bool):
    # at entry / exit: Q = P7 (phase 1), diag0 = P6 (phase 2), F0 = P5 (phase 3), F1 = P1 (phase 7)
    outs = ['[p7] "+v"(r.Q)', '[p6] "+v"(r.diag)', '[p5] "+v"(r.F0)', '[p1] "+v"(r.F1)',
            '[p0] "=&v"(x0)', '[p2] "=&v"(x2)', '[p3] "=&v"(x3)', '[p4] "=&v"(x4)', '[t0] "=&v"(t0)']
    ins = [f'[ta{i}] "v"(r.TA[{i}])' for i in range(4)] + [f'[tb{i}] "v"(r.TB[{i}])' for i in range(4)]
    if local:
        ins += ['[g] "s"(r.g)']
    if hp:
        outs += ['[pf] "=&v"(r.pf)', '[bad] "=&s"(r.bad)']
        ins += ['[pfa] "v"(r.pfaddr)', '[ctag] "s"(r.ctag)']
    if hn:
        ins += ['[paddr] "v"(r.pubaddr)', '[ptag] "s"(r.pubtag)']
    if hn or hp:
        ins += ['[msb] "v"(r.msb)']
    return outs, ins


def merge(local: bool) -> str:
    """The chunk's sign bits into its two interleaved words a0 (slots 0..15), a1 (slots 16..31). Both
    modes store DIAG and the raw "up > left" (local: raw TOP) bits; local STOP is H == 0, which the
    traceback recomputes, so the local merge is the global one."""
    local = False
    out = []
    for h, acc in ((0, "%[a0]"), (1, "%[a1]")):
        # (register, shift, mask operand) terms of the word's DIAG|STOP accumulator and of its TOP one
        odd = [(f"%[x{4 * h + t0}]", 2 * t0, f"%[mk{2 * t0}]") for t0 in range(4)]
        if local:
            odd += [(f"%[z{4 * h + t0}]", 2 * t0, f"%[mz{t0}]") for t0 in range(4)]
        even = [(f"%[y{4 * h + t0}]", 2 * t0 + 1, f"%[mk{2 * t0 + 1}]") for t0 in range(4)]
        if not local:
            terms = [(odd + even, acc)]
        else:
            terms = [(odd, acc), (even, "%[tb]")]
        for lst, a in terms:
            first = True
            for reg, sh, mk in lst:
                if first and sh == 0:
                    out.append(f"v_and_b32_e32 {a}, 0x80808080, {reg}")
                elif first:
                    out.append(f"v_lshrrev_b32_e32 %[tx], {sh}, {reg}")
                    out.append(f"v_and_b32_e32 {a}, %[tx], {mk}")
                elif sh == 0:
                    out.append(f"v_and_or_b32 {a}, {reg}, {mk}, {a}")
                else:
                    out.append(f"v_lshrrev_b32_e32 %[tx], {sh}, {reg}")
                    out.append(f"v_and_or_b32 {a}, %[tx], {mk}, {a}")
                first = False
        if local:
            # plane 1 = (TOP & ~DIAG) | STOP = B & ~(A >> 1) at the even bits (A >> 1 = DIAG|STOP there)
            out.append(f"v_lshrrev_b32_e32 %[tx], 1, {acc}")
            out.append(f"v_bitop3_b32 {acc}, %[tb], %[tx], {acc} bitop3:0xba")  # c | (a & ~b)
    return "\\n\\t".join(out)


def operands(local: bool, hn: bool, hp: bool):
    outs = ['[q] "+v"(r.Q)', '[qn] "=&v"(r.Qn)', '[dg] "+v"(r.diag)', '[f] "+v"(r.F)',
            '[d] "=&v"(D)', '[m] "=&v"(M)', '[t0] "=&v"(t0)']
    outs += [f'[x{g}] "+v"(r.X[{g}])' for g in range(8)] + [f'[y{g}] "+v"(r.Y[{g}])' for g in range(8)]
    ins = [f'[tw{i}] "v"(r.T[{i}])' for i in range(4)]
    if local:
        outs += ['[bm] "+v"(r.bm)', '[xr] "=&v"(Xr)', '[key] "=&v"(key)', '[key2] "=&v"(key2)']
        ins += ['[g] "s"(r.g)', '[kb] "s"(r.kb)']
    if hp:
        # early-clobber: the mask is written before the publish reads its raw tag (an SGPR input the
        # compiler could otherwise assign to the same register)
        outs += ['[pf] "=&v"(r.pf)', '[bad] "=&s"(r.bad)']
        ins += ['[pfa] "v"(r.pfaddr)', '[ctag] "s"(r.ctag)']
    if hn:
        ins += ['[paddr] "v"(r.pubaddr)', '[ptag] "s"(r.pubtag)']
    if hn or hp:
        ins += ['[msb] "v"(r.msb)']
    return outs, ins


def main():
    lines = [
        "// GENERATED by tools/gen_fill_asm.py -- do not edit. Hand-scheduled steady steps of the R = 1",
        "// kArr8 fill (see the generator's docstring for the schedule and its hazard rules).",
        "// steps_asm<LOCAL, HN, HP, HALF>(r): the U = 16 steps of a body (slots 16 * HALF .. 16 * HALF + 15",
        "// of its chunk); Q / Qn / diag / F rotate through the roles with period 4 (back in place after",
        "// the body); with HP the next body's feed read (address r.pfaddr) is issued after step 12 and",
        "// waited for at the end (result r.pf). merge_asm<LOCAL>(r) builds the chunk's two words.",
        "// band_steps_asm<LOCAL, HN, HP>(r): the band fill's score-wave steps (two rows per lane, no",
        "// direction bits; see band_block in the generator).",
        "#pragma once",
        "",
    ]
    for local in (False, True):
        for hn in (False, True):
            for hp in (False, True):
                body = band_block(local, hn, hp)
                outs, ins = band_operands(local, hn, hp)
                lines.append(f"template <> __device__ __forceinline__ void band_steps_asm<{str(local).lower()}, "
                             f"{str(hn).lower()}, {str(hp).lower()}>(BandRegs &r)")
                lines.append("{")
                lines.append("    int x0, x2, x3, x4, t0;")
                lines.append(f"    asm volatile(\"{body}\"")
                lines.append("        : " + ", ".join(outs))
                lines.append("        : " + ", ".join(ins) + (" : \"scc\");" if hp else ");"))
                lines.append("    (void)x0; (void)x2; (void)x3; (void)x4; (void)t0;")
                lines.append("}")
                lines.append("")
    for local in (False, True):
        for hn in (False, True):
            for hp in (False, True):
                for half in (0, 1):
                    body = block(local, hn, hp, half)
                    outs, ins = operands(local, hn, hp)
                    lines.append(f"template <> __device__ __forceinline__ void steps_asm<{str(local).lower()}, "
                                 f"{str(hn).lower()}, {str(hp).lower()}, {half}>(StepRegs &r)")
                    lines.append("{")
                    lines.append("    int D, M, t0, Xr, key, key2;")
                    lines.append(f"    asm volatile(\"{body}\"")
                    lines.append("        : " + ", ".join(outs))
                    lines.append("        : " + ", ".join(ins) + (" : \"scc\");" if hp else ");"))
                    lines.append("    (void)D; (void)M; (void)t0; (void)Xr; (void)key; (void)key2;")
                    lines.append("}")
                    lines.append("")
        outs = ['[a0] "=&v"(r.acc0)', '[a1] "=&v"(r.acc1)', '[tx] "=&v"(tx)']
        ins = [f'[x{g}] "v"(r.X[{g}])' for g in range(8)] + [f'[y{g}] "v"(r.Y[{g}])' for g in range(8)]
        ins += [f'[mk{g}] "v"(r.mk[{g}])' for g in range(8)]
        lines.append(f"template <> __device__ __forceinline__ void merge_asm<{str(local).lower()}>(StepRegs &r)")
        lines.append("{")
        lines.append("    int tx, tb;")
        lines.append(f"    asm volatile(\"{merge(local)}\"")
        lines.append("        : " + ", ".join(outs))
        lines.append("        : " + ", ".join(ins) + ");")
        lines.append("    (void)tx; (void)tb;")
        lines.append("}")
        lines.append("")
    open(OUT, "w").write("\n".join(lines))
    print("wrote", OUT)


if __name__ == "__main__":
    main()
