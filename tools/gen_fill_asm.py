#!/usr/bin/env python3
"""Generates sequence-alignment-gpu_amd/csrc/sa_fill_steps.inc: hand-scheduled inline-asm step blocks
of the R = 1 fill's steady bodies (text profiles as int8 bytes, kArr8), global and local, with and
without a strip below (HN).

Why asm: on gfx950 a DPP instruction must be 2 wait states behind the VALU write of any VGPR it
reads, and an s_nop costs an issue slot (4 cycles) like a VALU op. Scheduled by the compiler the
step's two lane moves landed right behind their producers (one to two s_nops per step, plus a
register copy for the bottom-row register), 13-15 issue slots per step; here every DPP sits at least
two instructions behind its inputs with independent work in between, so a global step is exactly
its 9 VALU ops and nothing else.

One step (four registers rotate through the roles Qn -> Q/up -> diag/F' -> left, period 4):
    b   Qn = Q shifted down one lane (wave_shl:1), written into the register of F two steps back
        (dead); with HN its lane 63 keeps that step's bottom-row value F (sa_fill.hip run_body)
    c   Q = F shifted up one lane (wave_shr:1), in place: lane 0 keeps the feed value = `up`
    d   D = diag + sext(score byte)          (SDWA byte select of the text-profile word)
    e   M = max(left, up)                    left = F of the previous step
    f   t1 = left - up                       -> plane 1 (raw up > left / raw TOP)
    g   global: F' = max(D, M) | local: X = max(D, M, g), F' = X - g, t2 = F' - 1 (STOP), key
        (F' goes to the diag register, dead after d)
    h   t0 = M - D                           -> plane 0 (DIAG)
    i/j/k  push the sign bits into the plane words (v_alignbit acc, acc, t, 31)
A global step is its 9 VALU ops with or without a strip below: the queue's bottom-row values run
one step later than the C++ bodies' (whose Qn takes F of the previous step through a register
copy, 1 VALU per step), and the publish at the body's end shifts the queue once more with F of the
step before last in lane 63, which gives the same 16 values (1 VALU per body instead of 16).

Local keys: key' = (F' << kb) - q, its running maximum bm over the block (one v_max3 per two
steps: keys alternate between two registers); the caller adds the body's key base
(kmask - (s0 & kmask)) once per body. Same order as the C++ recurrence
(alignSequenceCPU.cpp:175-192): larger H first, then the earlier column.
"""
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "sequence-alignment-gpu_amd", "csrc", "sa_fill_steps.inc")

U = 16
# with a strip above, the next body's feed read is issued after this step (kPfLead = U - PF_STEP)
PF_STEP = int(os.environ.get("SA_GEN_PF_STEP", "12"))


def block(local: bool, hn: bool, hp: bool, qb: int = 0, qe: int = U) -> str:
    # operand numbers (see the C++ wrapper below)
    A, B, C = "%0", "%1", "%2"
    FA, FB = "%3", "%4"
    D, M, T0, T1 = "%5", "%6", "%7", "%8"
    ACC0, ACC1 = "%9", "%10"
    # outputs first (Q .. acc1 = %0..%10, local extras %11..%15, then the feed value and its
    # bad-lane mask), then inputs (T words, local g / kb, feed address and raw tag, publish address and
    # raw tag, the sign-bit constant). A raw tag is (c + 63) << 20 of the slot's column c: its bit 31 is
    # the lap parity, the complement of the tag (sa_fill.hip ring_tag); v_bitop3 applies it.
    h = 2 if hp else 0
    nout = (11 if not local else 17) + h
    PF = f"%{nout - 2}"
    BAD = f"%{nout - 1}"
    TW = [f"%{nout + i}" for i in range(4)]
    k = nout + 4
    ACC2 = BM = X = T2 = KEY = KEY2 = G = KB = None
    if local:
        ACC2, BM, X, T2, KEY, KEY2 = "%11", "%12", "%13", "%14", "%15", "%16"
        G, KB = f"%{k}", f"%{k + 1}"
        k += 2
    PFA, CTAG = f"%{k}", f"%{k + 1}"
    if hp:
        k += 2
    PADDR, PTAG = f"%{k}", f"%{k + 1}"
    if hn:
        k += 2
    MSB = f"%{k}"
    # four registers rotate through the roles with period 4 (U = 16 returns them to their operands):
    # at step k, regs[k % 4] takes the shifted queue (Qn; it held F of step k-2, dead), regs[k-1] is
    # Q (shifted down, then overwritten in place by up), regs[k-2] is diag (then takes F'), regs[k-3]
    # is F of the previous step (left). Lane 63 of each Qn thus takes the bottom-row value of step
    # k-2 instead of k-1; the publish restores the order with one more shift whose `old` is F of the
    # step before last (lanes 64-U..63 = steps s0-1 .. s0+U-2, as the C++ bodies publish).
    regs = [B, FA, C, A]  # at entry: regs[3] = Q, regs[1] = F (left), regs[2] = diag, regs[0] dead
    out = []
    out.append("s_nop 1")  # the compiler's last writes of Q / F stand right before
    for k, q in enumerate(range(qb, qe)):
        qd, qr, dg, fp = regs[k % 4], regs[(k - 1) % 4], regs[(k - 2) % 4], regs[(k - 3) % 4]
        if hp and q == PF_STEP:
            out.append(f"ds_read_b32 {PF}, {PFA}")
        if hn:
            out.append(f"v_mov_b32_dpp {qd}, {qr} wave_shl:1 row_mask:0xf bank_mask:0xf")
        else:
            out.append(f"v_mov_b32_dpp {qd}, {qr} wave_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:1")
        out.append(f"v_mov_b32_dpp {qr}, {fp} wave_shr:1 row_mask:0xf bank_mask:0xf")
        out.append(f"v_add_u32_sdwa {D}, {dg}, sext({TW[q >> 2]}) dst_sel:DWORD dst_unused:UNUSED_PAD "
                   f"src0_sel:DWORD src1_sel:BYTE_{q & 3}")
        out.append(f"v_max_i32_e32 {M}, {fp}, {qr}")
        out.append(f"v_sub_u32_e32 {T1}, {fp}, {qr}")
        if not local:
            out.append(f"v_max_i32_e32 {dg}, {D}, {M}")
            out.append(f"v_sub_u32_e32 {T0}, {M}, {D}")
            out.append(f"v_alignbit_b32 {ACC1}, {ACC1}, {T1}, 31")
            out.append(f"v_alignbit_b32 {ACC0}, {ACC0}, {T0}, 31")
        else:
            # H = max(X, g) - g = max(X - g, 0) for g > 0 and X - g (never 0 clamped) for g <= 0
            out.append(f"v_max3_i32 {X}, {D}, {M}, {G}")
            out.append(f"v_sub_u32_e32 {T0}, {M}, {D}")
            out.append(f"v_subrev_u32_e32 {dg}, {G}, {X}")
            out.append(f"v_alignbit_b32 {ACC1}, {ACC1}, {T1}, 31")
            out.append(f"v_add_u32_e32 {T2}, -1, {dg}")
            kreg = KEY if k % 2 == 0 else KEY2
            out.append(f"v_lshl_add_u32 {kreg}, {dg}, {KB}, {-q}")
            out.append(f"v_alignbit_b32 {ACC0}, {ACC0}, {T0}, 31")
            if k % 2 == 1:
                out.append(f"v_max3_i32 {BM}, {BM}, {KEY}, {KEY2}")
            out.append(f"v_alignbit_b32 {ACC2}, {ACC2}, {T2}, 31")
    nst = qe - qb
    assert nst % 4 == 0, "the register rotation needs whole periods"
    if hp:
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


def main():
    lines = [
        "// GENERATED by tools/gen_fill_asm.py -- do not edit. Hand-scheduled steady steps of the R = 1",
        "// kArr8 fill (see the generator's docstring for the schedule and its hazard rules).",
        "// steps_asm<LOCAL, HN, HP>(r): the U = 16 steps of a body; Q / Qn / diag / F rotate through the",
        "// roles with period 4 (back in place after the body); with HP the next body's feed read (address",
        "// r.pfaddr) is issued after step 12 and waited for at the end (result r.pf).",
        "#pragma once",
        "",
    ]
    for local in (False, True):
        for hn in (False, True):
            for hp in (False, True):
                body = block(local, hn, hp)
                lines.append(f"template <> __device__ __forceinline__ void steps_asm<{str(local).lower()}, "
                             f"{str(hn).lower()}, {str(hp).lower()}>(StepRegs &r)")
                lines.append("{")
                lines.append("    int D, M, t0, t1, X, t2, key, key2;")
                lines.append(f"    asm volatile(\"{body}\"")
                lines.append("        : \"+v\"(r.Q), \"=&v\"(r.Qn), \"+v\"(r.diag), \"+v\"(r.F), \"=&v\"(r.F2),")
                lines.append("          \"=&v\"(D), \"=&v\"(M), \"=&v\"(t0), \"=&v\"(t1), \"+v\"(r.acc0), \"+v\"(r.acc1)")
                if local:
                    lines.append("          , \"+v\"(r.acc2), \"+v\"(r.bm), \"=&v\"(X), \"=&v\"(t2), \"=&v\"(key), \"=&v\"(key2)")
                if hp:
                    # early-clobber: the mask is written before the publish reads its raw tag (an SGPR
                    # input the compiler could otherwise assign to the same register)
                    lines.append("          , \"=&v\"(r.pf), \"=&s\"(r.bad)")
                ins = "\"v\"(r.T[0]), \"v\"(r.T[1]), \"v\"(r.T[2]), \"v\"(r.T[3])"
                if local:
                    ins += ", \"s\"(r.g), \"s\"(r.kb)"
                if hp:
                    ins += ", \"v\"(r.pfaddr), \"s\"(r.ctag)"
                if hn:
                    ins += ", \"v\"(r.pubaddr), \"s\"(r.pubtag)"
                if hn or hp:
                    ins += ", \"v\"(r.msb)"
                lines.append(f"        : {ins}" + (" : \"scc\");" if hp else ");"))
                lines.append("    (void)D; (void)M; (void)t0; (void)t1; (void)X; (void)t2; (void)key; (void)key2;")
                lines.append("}")
                lines.append("")
    open(OUT, "w").write("\n".join(lines))
    print("wrote", OUT)


if __name__ == "__main__":
    main()
