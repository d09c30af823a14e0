#!/usr/bin/env python3
"""Line model of the compact Thompson-noise reads of configs_4 at P = 8 (DESIGN.md section 4,
round 5): participants drawn as the bench draws them (P distinct of 32, 21 of them LR-TS), the
pairs ranked in (slot, auction) order as ag_ts_noise_index ranks them, the 768-lane workgroups'
grid-stride tiles; per (iteration, slot) the 128-B lines each workgroup's pairs touch (pair j,
coefficient c at ((j/64)*60 + c)*64 + j%64 floats: a 32-pair chunk of a row is one line), and
their union per XCD (workgroups dispatched round-robin over 8 XCDs; or mapped XCD-aware). Prints
line bytes over algorithmic bytes (240 B per pair).

    python tools/archive/noise_model.py
"""
import numpy as np
rng=np.random.default_rng(0)
B=1<<21; P=8; N=32
lrts=np.zeros(N,bool); lrts[11:]=True
# participants: P distinct of N per auction (uniform)
part=np.argsort(rng.random((B,N)),axis=1)[:,:P].T  # [P][B]
flag=lrts[part]                                     # [P][B]
j=np.cumsum(flag.ravel())-1; j=j.reshape(P,B)       # (s,i) order rank
G=256; BT=768; stride=G*BT
def model(xcd_aware):
    tot_wg=0; tot_xcd=0; alg=0
    for it in range((B+stride-1)//stride):
        for s in range(P):
            chunks_xcd=[set() for _ in range(8)]
            for b in range(G):
                r = (b%8)*(G//8)+b//8 if xcd_aware else b
                lo=it*stride+r*BT; hi=min(lo+BT,B)
                if lo>=B: continue
                f=flag[s,lo:hi]; jj=j[s,lo:hi][f]
                c=np.unique(jj>>5)
                tot_wg+=len(c); alg+=len(jj)
                chunks_xcd[b%8].update(c.tolist())
            tot_xcd+=sum(len(x) for x in chunks_xcd)
    return tot_wg*60*128/(alg*240), tot_xcd*60*128/(alg*240)
print("per-WG unique lines / algorithmic, per-XCD union / algorithmic:")
print("blockIdx order:", model(False))
print("XCD-aware     :", model(True))
