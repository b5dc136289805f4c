#!/usr/bin/env python3
"""Generates tools/microbench/loopbench.inc: prototype steady loops of the fused R = 1 fill step
(development tool, timing only: the values computed are not checked).

Per step (global mode; lane 0 is the feeder row, lanes 1..63 the strip's rows):
    v_add_u32_dpp  D, F[s-2], S[s]  wave_shr:1     D = diag + S          (lane 0 keeps D: never written)
    v_max_i32_dpp  M, F[s-1], F[s-1] wave_shr:1    M = max(up, left)     (lane 0 keeps the preloaded feed)
    v_max_i32      F[s], D, M
    v_sub_u32_sdwa X[t&7] byte 3-(t>>3) = M - D         sign: DIAG
    v_sub_u32_sdwa Y[t&7] byte 3-(t>>3) = F[s-1] - M    sign: up > left
and per 32 steps the eight X / Y registers merge into the two plane words (bit 31 - t = step t).
Memory per 16-step body: 4 global_load_dwordx4 of int32 text profiles (two bodies ahead), 4 ds_read_b128
feed reads (next body), 4 ds_write_b128 publishes (after steps 2, 6, 10, 14), one plane store per 32
steps. Variants: 0 no synchronisation, 1 s_barrier every 8 steps, 2 progress word per body.
"""
import os

HERE = os.path.dirname(os.path.abspath(__file__))

F = [f"v{32 + i}" for i in range(4)]
M = [[f"v{36 + 16 * b + i}" for i in range(16)] for b in range(2)]
S = [[f"v{68 + 16 * b + i}" for i in range(16)] for b in range(3)]
X = [f"v{116 + i}" for i in range(8)]
Y = [f"v{124 + i}" for i in range(8)]
D = ["v132", "v133"]
ACC = ("v134", "v135")
TMP = "v136"
VFEED, VPUB, VSOFF, VMOFF, VPROG, VPRR, VLMASK, VPUBBASE, VRIN, VPADDR = (f"v{137 + i}" for i in range(10))
SB, MB = "s[40:41]", "s[42:43]"
SCNT, SP, SP2, SBODY, SNEED = "s44", "s45", "s46", "s47", "s48"
SMASK = [None] + [f"s{48 + g}" for g in range(1, 8)]  # s49..s55
VREGS_USED = 147
SREGS = list(range(40, 60))


def body(bank_s: int, bank_m: int, word_half: int, bi: int, variant: int, store_pending: bool = True, feat: int = 15) -> list[str]:
    """One 16-step body. word_half: 0 = steps 0..15 of the plane word, 1 = 16..31."""
    out = []
    e = out.append
    nb_s = (bank_s + 2) % 3  # S bank loaded two bodies ahead
    for q in range(16):
        t = 16 * word_half + q
        g, byte = t & 7, 3 - (t >> 3)
        Sr = S[bank_s][q]
        Mr = M[bank_m][4 * (q >> 2) + ((q + 3) & 3)]
        Fc, Fm1, Fm2, Dr = F[q & 3], F[(q - 1) & 3], F[(q - 2) & 3], D[q & 1]
        e(f"v_add_u32_dpp {Dr}, {Fm2}, {Sr} wave_shr:1 row_mask:0xf bank_mask:0xf")
        e(f"v_max_i32_dpp {Mr}, {Fm1}, {Fm1} wave_shr:1 row_mask:0xf bank_mask:0xf")
        e(f"v_max_i32_e32 {Fc}, {Dr}, {Mr}")
        e(f"v_sub_u32_sdwa {X[g]}, {Mr}, {Dr} dst_sel:BYTE_{byte} dst_unused:UNUSED_PRESERVE src0_sel:DWORD src1_sel:DWORD")
        e(f"v_sub_u32_sdwa {Y[g]}, {Fm1}, {Mr} dst_sel:BYTE_{byte} dst_unused:UNUSED_PRESERVE src0_sel:DWORD src1_sel:DWORD")
        if q == 0:
            # publish address of this body, feed address of the next (ring position P, one SGPR)
            e(f"v_bfi_b32 {VPUB}, {VLMASK}, {SP}, {VPUBBASE}")
            e(f"s_add_u32 {SP2}, {SP}, 64")
            e(f"s_and_b32 {SP2}, {SP2}, 0x1fff")
        if q < 4 and feat & 1:
            pass
        if q < 4 and feat & 1:
            e(f"global_load_dwordx4 v[{S[nb_s][4 * q][1:]}:{int(S[nb_s][4 * q][1:]) + 3}], {VSOFF}, {SB} offset:{128 + 16 * q}")
        if q == 4:
            if feat & 256:
                e("s_add_u32 s56, s56, 64")
                e("s_and_b32 s56, s56, 0x1fff")
                e("s_add_u32 s40, s57, s56")
            else:
                e("s_add_u32 s40, s40, 64")
                e("s_addc_u32 s41, s41, 0")
            e(f"v_add_u32_e32 {VFEED}, {SP2}, {VRIN}")
            if word_half == 0 and store_pending and feat & 4:
                # the previous word's store, issued after this body's loads: the end-of-body wait
                # for the next body's text profile does not wait for it
                e(f"global_store_dwordx2 {VMOFF}, v[{ACC[0][1:]}:{ACC[1][1:]}], {MB}")
                e("s_add_u32 s42, s42, 512")
                e("s_addc_u32 s43, s43, 0")
        if q in (2, 6, 10, 14) and (feat & 2 or feat & 32):
            if feat & 64:
                e("s_mov_b64 exec, s[58:59]")
            e(f"ds_write_b128 {VPUB}, v[{F[0][1:]}:{int(F[0][1:]) + 3}] offset:{16 * (q >> 2)}")
            if feat & 64:
                e("s_mov_b64 exec, -1")
        if q == 14 and variant == 2:
            e(f"v_mov_b32_e32 {VPROG}, {SBODY}")
            e(f"ds_write_b32 {VPADDR}, {VPROG} offset:4")
        if q == (4 if feat & 128 else 9) and (feat & 2 or feat & 16):
            if variant == 2:
                e(f"ds_read_b32 {VPRR}, {VPADDR}")
            for j in range(4):
                m0 = int(M[1 - bank_m][4 * j][1:])
                e(f"ds_read_b128 v[{m0}:{m0 + 3}], {VFEED} offset:{16 * j}")
        if variant == 1 and q in (7, 15):
            e("s_barrier")
    # end of body: next body's feed (LDS) and text profile (loaded one body earlier) must be there
    e(f"s_mov_b32 {SP}, {SP2}")
    vm = 5 if word_half == 0 else 4   # even bodies: this body's 4 loads and the store are younger
    if variant == 2:
        e(f"s_add_u32 {SBODY}, {SBODY}, 1")
        e(f"s_add_u32 {SNEED}, {SNEED}, 1")
        e(f"s_waitcnt vmcnt({vm}) lgkmcnt(3)")
        e(f"v_cmp_gt_i32_e32 vcc, {SNEED}, {VPRR}")
        e(f"s_cbranch_vccnz .Lslow{bi}_%=")
        e(f".Lback{bi}_%=:")
    else:
        e(f"s_waitcnt vmcnt({vm}) lgkmcnt(2)")
    if word_half == 1 and feat & 8:
        # merge the plane word (bit 31 - t = step t) and store it
        e(f"v_and_b32_e32 {ACC[0]}, 0x80808080, {X[0]}")
        e(f"v_and_b32_e32 {ACC[1]}, 0x80808080, {Y[0]}")
        for g in range(1, 8):
            e(f"v_lshrrev_b32_e32 {TMP}, {g}, {X[g]}")
            e(f"v_and_or_b32 {ACC[0]}, {TMP}, {SMASK[g]}, {ACC[0]}")
            e(f"v_lshrrev_b32_e32 {TMP}, {g}, {Y[g]}")
            e(f"v_and_or_b32 {ACC[1]}, {TMP}, {SMASK[g]}, {ACC[1]}")
    return out


def slow_paths(variant: int, nb: int) -> list[str]:
    """Progress not there yet: poll, then re-read the next body's feed (the early reads may be stale)."""
    out = []
    if variant != 2:
        return out
    for bi in range(nb):
        out.append(f".Lslow{bi}_%=:")
        out.append("s_sleep 0")
        out.append(f"ds_read_b32 {VPRR}, {VPADDR}")
        out.append("s_waitcnt lgkmcnt(0)")
        out.append(f"v_cmp_gt_i32_e32 vcc, {SNEED}, {VPRR}")
        out.append(f"s_cbranch_vccnz .Lslow{bi}_%=")
        nbm = 1 - (bi % 2)
        for j in range(4):
            m0 = int(M[nbm][4 * j][1:])
            out.append(f"ds_read_b128 v[{m0}:{m0 + 3}], {VFEED} offset:{16 * j}")
        out.append("s_waitcnt lgkmcnt(0)")
        out.append(f"s_branch .Lback{bi}_%=")
    return out


def loop(variant: int, feat: int = 15) -> str:
    lines = [f"s_mov_b32 {SCNT}, %[iters]"]
    lines += [f"s_mov_b32 {SMASK[g]}, 0x{(0x80808080 >> g):08x}" for g in range(1, 8)]
    lines += ["s_mov_b32 s56, 0", "s_mov_b32 s58, 0", "s_mov_b32 s59, 0x80000000",
              "s_mov_b64 s[40:41], %[sb]", "s_mov_b32 s57, s40", "s_mov_b64 s[42:43], %[mb]", f"s_mov_b32 {SP}, %[sp0]",
              f"s_mov_b32 {SNEED}, %[sneed]", f"s_mov_b32 {SBODY}, 0",
              f"v_mov_b32 {VSOFF}, %[vsoff]", f"v_mov_b32 {VMOFF}, %[vmoff]", f"v_mov_b32 {VLMASK}, %[vlmask]",
              f"v_mov_b32 {VPUBBASE}, %[vpubbase]", f"v_mov_b32 {VRIN}, %[vrin]", f"v_mov_b32 {VPADDR}, %[vpaddr]",
              f"v_add_u32_e32 {VFEED}, {SP}, {VRIN}"]
    lines += [f"v_mov_b32 v{r}, 0" for r in range(32, 134)]
    lines += [".Lloop_%=:"]
    for bi in range(6):
        lines += body(bi % 3, bi % 2, bi % 2, bi, variant, feat=feat)
    lines += [f"s_sub_u32 {SCNT}, {SCNT}, 1", f"s_cmp_lg_u32 {SCNT}, 0",
              "s_cbranch_scc1 .Lloop_%=", "s_branch .Ldone_%="]
    lines += slow_paths(variant, 6)
    lines += [".Ldone_%=:", "s_waitcnt vmcnt(0) lgkmcnt(0)"]
    return "\\n\\t".join(x for x in lines if x)


FEATS = {"NONE": 0, "LDS": 2, "LDSR": 16, "LDSW": 32, "LDSWX": 32 | 64, "LDSX": 2 | 64, "LDSEARLY": 2 | 128,
         "LDSEARLYX": 2 | 128 | 64, "LOADS": 1, "LOADSL2": 1 | 256, "ALL_L2": 1 | 2 | 4 | 8 | 256,
         "ALL_L2X": 1 | 2 | 4 | 8 | 256 | 64 | 128}


def main():
    clob = ", ".join(f'"v{i}"' for i in range(32, 32 + VREGS_USED - 32 + 1))
    sclob = ", ".join(f'"s{i}"' for i in SREGS)
    with open(os.path.join(HERE, "loopbench.inc"), "w") as f:
        f.write("// GENERATED by tools/microbench/gen_loopbench.py\n#pragma once\n")
        f.write(f"#define LB_VCLOB {clob}\n#define LB_SCLOB {sclob}\n")
        for v in range(3):
            f.write(f"#define LB_LOOP{v} \"{loop(v)}\"\n")
        for name, ft in FEATS.items():
            f.write(f"#define LB_{name} \"{loop(0, ft)}\"\n")
    print("ok")


if __name__ == "__main__":
    main()
