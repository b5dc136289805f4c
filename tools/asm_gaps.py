#!/usr/bin/env python3
"""Development tool: instruction counts between consecutive hand-scheduled steady bodies (the
compiler-generated per-body work) of the R = 1 chained fill kernels, from device assembly:
    hipcc -O3 -std=c++17 --offload-arch=gfx950 --cuda-device-only -S csrc/fill_r1.hip -I../include -o fill_r1.s
    python tools/asm_gaps.py fill_r1.s"""
import re
import sys

S = open(sys.argv[1]).read().split("\n")
for name in ("_ZN2sa11fill_kernelILi1ELb0ELi3ELb1ELb0EEEvNS_8FillArgsE", "_ZN2sa11fill_kernelILi1ELb1ELi3ELb1ELb0EEEvNS_8FillArgsE"):
    st = [i for i, l in enumerate(S) if l.startswith(name + ":")][0]
    en = [i for i in range(st, len(S)) if S[i].startswith(".Lfunc_end")][0]
    L = S[st:en]
    blocks, i = [], 0
    while i < len(L):
        if ";;#ASMSTART" in L[i]:
            j = i
            while ";;#ASMEND" not in L[j]:
                j += 1
            txt = "\n".join(L[i:j])
            if "ds_read_b32" in txt and "ds_write_b32" in txt and j - i > 100:
                blocks.append((i, j))
            i = j
        i += 1
    out = []
    for k in range(len(blocks) - 1):
        a, b = blocks[k][1], blocks[k + 1][0]
        body = [l.strip() for l in L[a + 1:b] if l.strip() and not l.strip().startswith(";") and not l.startswith(".L") and "ASM" not in l]
        if len(body) > 120:
            out.append("loop")
            continue
        kinds = {"s": sum(x.startswith("s_") for x in body), "v": sum(x.startswith("v_") for x in body),
                 "m": sum(x.split()[0].startswith(("global", "ds_", "buffer", "scratch")) for x in body),
                 "spill": sum("v_readlane" in x or "v_writelane" in x for x in body)}
        out.append(f"{len(body)}(s{kinds['s']} v{kinds['v']} m{kinds['m']} sp{kinds['spill']})")
    print("local " if name.startswith("_ZN2sa11fill_kernelILi1ELb1") else "global", " ".join(out[:10]))
