#!/usr/bin/env python3
"""Op-count estimate of a common-subexpression pass over the K=20/M=60 bit-sliced
encode: per 10-row tile, XOR3 ops of the four-Russians updates
vs the same after greedy sharing of XOR3 triples across output planes.
Argument W: restrict triples to windows of W consecutive inputs (0: no limit)."""
import sys, itertools, collections, random
sys.path.insert(0,'/root/repo')
from zfec_amd import capi
k,m=20,60
code=capi.Code(k,m); E=code.enc_matrix()
# GF mul
exp=[0]*510; log=[0]*256; x=1
for i in range(255):
    exp[i]=x; log[x]=i; x<<=1
    if x&0x100: x^=0x11d
for i in range(255,510): exp[i]=exp[i-255]
def mul(a,b): return 0 if a==0 or b==0 else exp[log[a]+log[b]]
def masks(c):
    return [sum(1<<a for a in range(8) if (mul(c,1<<a)>>b)&1) for b in range(8)]
W=int(sys.argv[1]) if len(sys.argv)>1 else 0
rows=list(range(k,m))
tot_cur=0; tot_new=0
for t in range(4):
    R=rows[t*10:(t+1)*10]
    planes=[]
    cur=0
    used=set()
    for i in R:
        for b in range(8):
            s=set()
            for j in range(k):
                mk=masks(E[i*k+j])[b]
                if mk&15: s.add((j,'L',mk&15))
                if mk>>4: s.add((j,'H',mk>>4))
            planes.append(s); used|=s
    # current cost: per plane per input 1 op (ignore init mov nuance)
    for s in planes:
        cur+= (len(s)+1)//2   # approx xor3 packing, one op per 2 terms
    # table cost: combos used per input side
    tab=0
    for j in range(k):
        for side in 'LH':
            ms={mk for (jj,sd,mk) in used if jj==j and sd==side}
            # closure built via top-bit decomposition
            have=set()
            def build(mm):
                global_cnt=0
                if mm&(mm-1)==0 or mm in have: return 0
                top=1<<(mm.bit_length()-1)
                c=build(mm^top)+1; have.add(mm); return c
            tab+=sum(build(mm) for mm in ms)
    # greedy triple CSE
    P=[set(s) for s in planes]; newsyms=0; nid=0
    while True:
        cnt=collections.Counter()
        for s in P:
            l=sorted(s,key=str)
            if len(l)<3: continue
            for tr in itertools.combinations(l,3):
                if W and len({(x[0]//W if x[0]!="N" else x[1]) for x in tr})>1: continue
                cnt[tr]+=1
        if not cnt: break
        tr,f=cnt.most_common(1)[0]
        if f<2: break
        nid+=1; sym=('N',tr[0][0]//W if W else nid, nid); newsyms+=1
        for s in P:
            if all(x in s for x in tr):
                for x in tr: s.discard(x)
                s.add(sym)
    after=sum((len(s)+1)//2 for s in P)+newsyms
    print(f"tile {t}: plane ops {cur} -> triple-CSE {after} (new {newsyms}); table ops {tab}")
    tot_cur+=cur+tab; tot_new+=after+tab
print(tot_cur, tot_new)
