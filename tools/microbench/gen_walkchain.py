#!/usr/bin/env python3
"""Row-walk chain variants for tools/microbench/walkchain.hip (development tool): clk per row of the
unrolled 64-row block under different instruction sequences (see VARIANTS)."""
import os

OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "walkchain.inc")

# per row k (lane), with a = s88/s89 or s90/s91 alternating (the window read a row ahead)
def row(v, k):
    a, b = ("s[88:89]", "s90") if k % 2 else ("s[90:91]", "s88")
    p, pp = ("s95", "s94") if k % 2 else ("s94", "s95")
    out = []
    if v in ("A", "B", "C", "D"):
        out.append(f"s_lshr_b64 s[92:93], {a}, %[u]")
        if v in ("A", "B"):
            out.append(f"v_writelane_b32 %[rec], {pp}, {k}")
        if v in ("A", "C"):
            out.append(f"s_cbranch_scc0 .Lx_%=")
        out.append(f"s_ff1_i32_b32 {p}, s92")
        if v in ("A", "B", "C"):
            out.append(f"v_readlane_b32 {b}, %[w0], {(k + 1) % 64}")
        out.append(f"s_bitcmp1_b32 {p}, 0")
        out.append(f"s_addc_u32 %[u], %[u], {p}")
    elif v in ("E", "F", "G"):
        # 3-op chain: the shift's SCC (word non-zero) is the +1 of u += p + 1
        out.append(f"s_lshr_b64 s[92:93], {a}, %[u]")
        out.append(f"v_writelane_b32 %[rec], {pp}, {k}")
        if v == "E":
            out.append(f"s_cbranch_scc0 .Lx_%=")
        out.append(f"s_ff1_i32_b32 {p}, s92")
        out.append(f"v_readlane_b32 {b}, %[w0], {(k + 1) % 64}")
        out.append(f"s_addc_u32 %[u], %[u], {p}")
        if v == "G":
            out.append(f"s_nop 0")
    elif v == "H":
        # the chain alone, 3 ops
        out.append(f"s_lshr_b64 s[92:93], {a}, %[u]")
        out.append(f"s_ff1_i32_b32 {p}, s92")
        out.append(f"s_addc_u32 %[u], %[u], {p}")
    elif v == "I":
        # 2 ops: lshr + ff1 only (u += ff1 via s_add inside... not a walk; SALU latency floor)
        out.append(f"s_lshr_b64 s[92:93], {a}, %[u]")
        out.append(f"s_ff1_i32_b32 %[u], s92")
    return out

VARIANTS = ["A", "B", "C", "D", "E", "F", "G", "H", "I"]

lines = ["#pragma once"]
for v in VARIANTS:
    body = ["s_mov_b32 s89, s88", "s_mov_b32 s91, s90"]
    for k in range(64):
        body += row(v, k)
        # keep the 64-bit windows' high halves equal to the low ones (wrap of u) without extra ops:
        # the high half is fixed at entry; the readlane refreshes only the low one (same value per lane)
    body.append(".Lx_%=:")
    lines.append(f"#define WC_{v} \\")
    lines.append("    \"" + "\\n\\t".join(body) + "\"")
open(OUT, "w").write("\n".join(lines) + "\n")
print("wrote", OUT)
