#!/usr/bin/env python3
"""Generates sequence-alignment-gpu_amd/csrc/sa_fill_steps.inc: hand-scheduled inline-asm step blocks
of the R = 1 fill's steady bodies (text profiles as int8 bytes, kArr8), global and local, with and
without a strip below (HN).

Why asm: on gfx950 a DPP instruction must be 2 wait states behind the VALU write of any VGPR it
reads, and an s_nop costs an issue slot (4 cycles) like a VALU op. Scheduled by the compiler the
step's two lane moves landed right behind their producers (one to two s_nops per step, plus a
register copy for the bottom-row register), 13-15 issue slots per step; here every DPP sits at least
two instructions behind its inputs with independent work in between, so a global step is exactly
its 9 VALU ops (10 with a strip below) and nothing else.

One step (roles rotate A -> B -> C every step; F alternates between two registers):
    b   Qn = A shifted down one lane (wave_shl:1); with HN its old value, preloaded, is the previous
        step's bottom-row value F, which lane 63 keeps (sa_fill.hip run_body)
    c   A = F shifted up one lane (wave_shr:1), in place: lane 0 keeps the feed value = `up`
    d   D = diag + sext(score byte)          (SDWA byte select of the text-profile word)
    e   M = max(left, up)                    left = F of the previous step
    f   t1 = left - up                       -> plane 1 (raw up > left / raw TOP)
    g   global: F' = max(D, M) | local: X = max(D, M), F' = X -sat g, t2 = F' - 1 (STOP), key
    h   t0 = M - D                           -> plane 0 (DIAG)
    a'  (HN) C = F'                          preload of the next step's b (C held diag, now dead)
    i/j/k  push the sign bits into the plane words (v_alignbit acc, acc, t, 31)
The next step uses Q = B (old Qn), Qn = C, diag = A (this step's up).

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
    roles = [A, B, C]
    fregs = [FA, FB]
    out = []
    if hn:
        out.append(f"v_mov_b32 {B}, {FA}")  # preload of the first step's Qn (the previous step's F)
    out.append("s_nop 1")  # the compiler's last writes of Q / F / the preload stand right before
    for k, q in enumerate(range(qb, qe)):
        a, b, c = roles
        if hp and q == PF_STEP:
            out.append(f"ds_read_b32 {PF}, {PFA}")
        fp, fn = fregs[k % 2], fregs[(k + 1) % 2]
        last = q == qe - 1
        if hn:
            out.append(f"v_mov_b32_dpp {b}, {a} wave_shl:1 row_mask:0xf bank_mask:0xf")
        else:
            out.append(f"v_mov_b32_dpp {b}, {a} wave_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:1")
        out.append(f"v_mov_b32_dpp {a}, {fp} wave_shr:1 row_mask:0xf bank_mask:0xf")
        out.append(f"v_add_u32_sdwa {D}, {c}, sext({TW[q >> 2]}) dst_sel:DWORD dst_unused:UNUSED_PAD "
                   f"src0_sel:DWORD src1_sel:BYTE_{q & 3}")
        out.append(f"v_max_i32_e32 {M}, {fp}, {a}")
        out.append(f"v_sub_u32_e32 {T1}, {fp}, {a}")
        if not local:
            out.append(f"v_max_i32_e32 {fn}, {D}, {M}")
            out.append(f"v_sub_u32_e32 {T0}, {M}, {D}")
            if hn and not last:
                out.append(f"v_mov_b32_e32 {c}, {fn}")
            out.append(f"v_alignbit_b32 {ACC1}, {ACC1}, {T1}, 31")
            out.append(f"v_alignbit_b32 {ACC0}, {ACC0}, {T0}, 31")
        else:
            out.append(f"v_max_i32_e32 {X}, {D}, {M}")
            out.append(f"v_sub_u32_e32 {T0}, {M}, {D}")
            out.append(f"v_sub_u32_e64 {fn}, {X}, {G} clamp")
            out.append(f"v_alignbit_b32 {ACC1}, {ACC1}, {T1}, 31")
            out.append(f"v_add_u32_e32 {T2}, -1, {fn}")
            kreg = KEY if k % 2 == 0 else KEY2
            out.append(f"v_lshl_add_u32 {kreg}, {fn}, {KB}, {-q}")
            if hn and not last:
                out.append(f"v_mov_b32_e32 {c}, {fn}")
            out.append(f"v_alignbit_b32 {ACC0}, {ACC0}, {T0}, 31")
            if k % 2 == 1:
                out.append(f"v_max3_i32 {BM}, {BM}, {KEY}, {KEY2}")
            out.append(f"v_alignbit_b32 {ACC2}, {ACC2}, {T2}, 31")
        roles = [b, c, a]
    if hp:
        out.append("s_waitcnt lgkmcnt(0)")  # the feed read (issued 4 steps ago) is there
        # tag check: x = entry ^ expected tag (the value when it matches; bitop3 0xD2 = a ^ (~b & c)),
        # bad lanes = x < 0 among the body's U feed lanes; the publish below stands between the
        # compare and the caller's SALU test of the mask
        out.append(f"v_bitop3_b32 {PF}, {PF}, {CTAG}, {MSB} bitop3:0xd2")
        out.append(f"v_cmp_gt_i32_e64 {BAD}, 0, {PF}")
        out.append(f"s_and_b64 {BAD}, {BAD}, 0xffff")
    if hn:
        # publish: lanes 48..63 of the accumulated Q (now role B) with the body's lap tag; the write
        # stays in flight past the block (the compiler sees no LDS operation it would wait for)
        q_final = [A, B, C][U % 3]
        out.append(f"v_bitop3_b32 {T0}, {q_final}, {PTAG}, {MSB} bitop3:0xf2")  # a | (~b & c)
        out.append(f"ds_write_b32 {PADDR}, {T0}")
    return "\\n\\t".join(out)


def rot(n):
    return n % 3


def main():
    lines = [
        "// GENERATED by tools/gen_fill_asm.py -- do not edit. Hand-scheduled steady steps of the R = 1",
        "// kArr8 fill (see the generator's docstring for the schedule and its hazard rules).",
        "// steps_asm<LOCAL, HN, HP>(r): the U = 16 steps of a body; Q / Qn / diag rotate by one role per",
        "// step, F alternates between two registers; with HP the next body's feed read (address",
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
                lines.append(f"    r.rotate<{rot(U)}>();")
                lines.append("}")
                lines.append("")
    open(OUT, "w").write("\n".join(lines))
    print("wrote", OUT)


if __name__ == "__main__":
    main()
