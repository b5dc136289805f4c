#!/usr/bin/env python3
"""Simulation (CPU, development tool): would a speculative segmented traceback pay? The rows of one
pair are split into G segments of whole strips; every segment but the bottom one walks from a guessed
entry column (global: the line to (0, 0); local: the start's diagonal), and once the true entry is
known a fix-up walk runs until it meets the speculative path at a strip boundary. Prints the fix-up
rows per segment and the resulting critical path against the sequential walk.
    python tools/tb_segments.py N MODE G      (direction matrix from the C oracle, (N+1)^2 bytes)
Result: random DNA paths drift hundreds of columns from any guess and merge too late."""
import os, sys, numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, 'sequence-alignment-gpu_amd', 'python'))
from oracle import oracle
from sa_amd import synthetic
N=int(sys.argv[1]); mode=int(sys.argv[2]); G=int(sys.argv[3])
t=synthetic.random_sequence(6,N,4); p=synthetic.random_sequence(7,N,4)
S=synthetic.blast_matrix()
M=np.empty((N+1)*(N+1),np.uint8); oracle.fill_only(mode,t,p,S,5,M); M=M.reshape(N+1,N+1)
if mode==0: i0=j0=N
else:
    r=oracle.align(mode,t,p,S,5)
    # start from the max: recover by running traceback? use the oracle's start: end cell = start + consumed
    at=r['aligned_text']; ap=r['aligned_pattern']
    j0=r['start_text']+1+sum(c!='-' for c in at)-1; i0=r['start_pattern']+1+sum(c!='-' for c in ap)-1
print('start',i0,j0)
def walk(i,j,stop_row):
    """walk from entry (i,j) [i = bottom row of a strip] up to row stop_row (exclusive); return per-strip entry cols"""
    E={}
    while i>stop_row and j>0:
        if (i%64)==0 and i not in E: E[i]=j
        d=M[i,j]
        if d==1: i-=1;j-=1
        elif d==0: j-=1
        elif d==2: i-=1
        else: return E,(i,j),True
    return E,(i,j),False
# strips: rows 64b+1..64b+64; segment boundaries at rows multiple of 64
top=(i0-1)//64  # strip of start
nst=top+1
bounds=[int(round(nst*g/G)) for g in range(G+1)]  # strips [bounds[g], bounds[g+1])
trueE,_,_=walk(i0,j0,0)
crit=0
rows_seg=[]
for g in range(G-1,-1,-1):
    lo,hi=bounds[g],bounds[g+1]
    rb=64*hi if g<G-1 else i0   # entry row
    if g==G-1:
        rows_seg.append(('exact',rb-64*lo)); continue
    guess = round(j0*rb/i0) if mode==0 else j0-(i0-rb)
    spec,_,_=walk(rb,max(1,guess),64*lo)
    te=trueE.get(rb)
    if te is None: rows_seg.append(('dead',0)); continue
    # fix-up: walk from true entry until its E matches spec's at a strip boundary
    fx,_,_=walk(rb,te,64*lo)
    merged=None
    for r in range(rb,64*lo-1,-64):
        if r in fx and r in spec and fx[r]==spec[r]: merged=r;break
    rows_seg.append(('guess',guess,'true',te,'fixrows',rb-(merged if merged is not None else 64*lo)))
print(rows_seg)
L=(bounds[G]-bounds[G-1])*64
fix=sum(x[-1] for x in rows_seg[1:] if x[0]=='guess')
print('seq rows',i0,'parallel critical ~',L+fix,'speedup',i0/(L+fix))
