#!/usr/bin/env python3
"""Generates sequence-alignment-gpu_amd/csrc/sa_walk_rows.inc: the unrolled scalar row walk of one
64-row strip used by the row-walk traceback kernel (sa_walk.hip, walk_rw_kernel).

One asm statement walks rows 63..0 of a strip (lane k of the window VGPRs = strip row k). Per row:
    v_readlane  next row's window word (issued one row ahead: the VALU->SALU latency is ~20 clk)
    s_lshr_b64  x = {word, 0} >> u          SCC = a non-LEFT cell at or left of the current column
    s_cbranch_scc0  -> advance stub         (window exhausted: rotate W0..W7, retry the same row)
    s_ff1_i32_b32   p = first set bit       (p = 2 * LEFT run + 1 if the cell is DIAG)
    s_bitcmp1_b32   p, 0                    SCC = DIAG
    s_addc_u32      u = u + p + DIAG        (next row's search position)
    v_writelane     record p at lane k, issued in the next row's block right after its shift (so
                    its issue hides under the shift's latency instead of standing on the row chain;
                    p alternates between s94 and s95)
Local mode: a STOP cell has both of its bits set, so the search finds its even bit p; bit p ^ 1 of
the shifted word is set only then (s_xor + s_bitcmp1, branch to the exit).

Usage: python3 tools/gen_walk_asm.py > sequence-alignment-gpu_amd/csrc/sa_walk_rows.inc
"""
from __future__ import annotations

import sys


def cur_regs(k: int) -> tuple[str, str]:
    """(window word, 64-bit pair) scalar registers holding row k's word."""
    return ("s88", "s[88:89]") if k % 2 else ("s90", "s[90:91]")


def prec(k: int) -> str:
    """Scalar register holding row k's record p (alternating, so that row k's write can wait)."""
    return "s94" if k % 2 == 0 else "s95"


def gen(local: bool) -> list[str]:
    L: list[str] = []
    e = L.append
    e("s_mov_b32 s89, 0")
    e("s_mov_b32 s91, 0")
    e("v_readlane_b32 s88, %[w0], 63")
    for k in range(63, -1, -1):
        w, pair = cur_regs(k)
        nw, _ = cur_regs(k - 1) if k > 0 else (None, None)
        p = prec(k)
        e(f".Lrow{k}_%=:")
        e(f"s_lshr_b64 s[92:93], {pair}, %[u]")
        if k < 63:
            # the previous row's record, issued under the shift's latency (off the row chain)
            e(f"v_writelane_b32 %[rec], {prec(k + 1)}, {k + 1}")
        e(f"s_cbranch_scc0 .Ladv{k}_%=")
        e(f"s_ff1_i32_b32 {p}, s92")
        if k > 0:
            # the next row's word, under the search's latency
            e(f"v_readlane_b32 {nw}, %[w0], {k - 1}")
        e(f"s_bitcmp1_b32 {p}, 0")
        e(f"s_addc_u32 %[u], %[u], {p}")
        if local:
            # STOP test after the position update (off the row chain; the stub undoes the update:
            # p is even for a STOP)
            e(f"s_xor_b32 s86, {p}, 1")
            e("s_bitcmp1_b32 s92, s86")
            e(f"s_cbranch_scc1 .Lstopm{k}_%=")
    e(f"v_writelane_b32 %[rec], {prec(0)}, 0")
    e("s_mov_b32 %[st], -1")
    e(f"s_mov_b32 %[lp], {prec(0)}")
    e("s_branch .Lout_%=")
    # out-of-line stubs
    for k in range(63, -1, -1):
        w, pair = cur_regs(k)
        nw, _ = cur_regs(k - 1) if k > 0 else (None, None)
        p = prec(k)
        e(f".Ladv{k}_%=:")
        e("s_sub_u32 s97, 32, %[u]")
        e("s_add_u32 %[pa], %[pa], s97")
        e("s_mov_b32 %[u], 0")
        e(f".Ladvl{k}_%=:")
        e("s_add_u32 %[na], %[na], 1")
        e("s_cmp_gt_u32 %[na], 7")
        e(f"s_cbranch_scc1 .Lexh{k}_%=")
        for x in range(7):
            e(f"v_mov_b32 %[w{x}], %[w{x + 1}]")
        e("v_mov_b32 %[w7], 0")
        e(f"v_readlane_b32 {w}, %[w0], {k}")
        if k > 0:
            e(f"v_readlane_b32 {nw}, %[w0], {k - 1}")
        e(f"s_cmp_lg_u32 {w}, 0")
        e(f"s_cbranch_scc1 .Lfnd{k}_%=")
        e("s_add_u32 %[pa], %[pa], 32")
        e(f"s_branch .Ladvl{k}_%=")
        e(f".Lfnd{k}_%=:")
        e(f"s_ff1_i32_b32 {p}, {w}")
        if local:
            e(f"s_xor_b32 s86, {p}, 1")
            e(f"s_bitcmp1_b32 {w}, s86")
            e(f"s_cbranch_scc1 .Lstop{k}_%=")
        e(f"s_bitcmp1_b32 {p}, 0")
        e(f"s_addc_u32 %[u], %[u], {p}")
        e(f"s_add_u32 {p}, {p}, %[pa]")
        e("s_mov_b32 %[pa], 0")
        if k > 0:
            # the next row block writes this record (its deferred write)
            e(f"s_branch .Lrow{k - 1}_%=")
        else:
            e(f"v_writelane_b32 %[rec], {p}, {k}")
            e("s_mov_b32 %[st], -1")
            e(f"s_mov_b32 %[lp], {p}")
            e("s_branch .Lout_%=")
        e(f".Lexh{k}_%=:")
        e(f"s_mov_b32 %[st], {k}")
        e("s_branch .Lout_%=")
        if local:
            e(f".Lstopm{k}_%=:")
            e(f"s_sub_u32 %[u], %[u], {p}")
            e(f".Lstop{k}_%=:")
            e(f"s_mov_b32 %[st], {0x100 | k}")
            e(f"s_mov_b32 %[lp], {p}")
            e("s_branch .Lout_%=")
    e(".Lout_%=:")
    return L


def emit(name: str, lines: list[str]) -> str:
    body = "\n".join(f'    "{ln}\\n"' for ln in lines)
    return f"#define {name} \\\n" + " \\\n".join(f'    "{ln}\\n"' for ln in lines) + "\n"


def main() -> None:
    out = sys.stdout
    out.write("// Generated by tools/gen_walk_asm.py -- do not edit. The unrolled 64-row strip walk of the\n")
    out.write("// row-walk traceback (sa_walk.hip): SA_WALK_ROWS_GLOBAL / SA_WALK_ROWS_LOCAL are inline-asm\n")
    out.write("// templates; scratch scalar registers s84-s97 are declared clobbered by the statement.\n")
    out.write("#pragma once\n")
    out.write(emit("SA_WALK_ROWS_GLOBAL", gen(False)))
    out.write(emit("SA_WALK_ROWS_LOCAL", gen(True)))


if __name__ == "__main__":
    main()
