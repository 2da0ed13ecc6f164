"""Diagnostic: how balanced is lane-mode B?  For 4-window waves of a corpus (cfg4 "s2orc" or cfg2 "ascii"),
the cost of the kernel's nested loops (per position 30 + 22 per candidate instructions, the wave stepping as
long as its longest chunk and each position as long as its most-candidate lane) against the perfectly
balanced cost (all work / 64 lanes), and what chunking could reach: the kernel's nearest-cut chunks,
work-weighted cuts and the optimal partition of each row at cut points (a per-lane work-sum model).
Mirrors tools/lane_model.py's chunking.  Usage: python tools/b_balance.py s2orc 150"""
import sys, os
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'dp-tokenization_amd'), os.path.join(ROOT, 'tests'), os.path.join(ROOT, 'tools')]
import lane_model as LM
from dptok import synth
from oracle import ref_port
t2i = synth.llama_shaped_vocab()
vocab = set(t2i.keys())
gen = sys.argv[1]; N=int(sys.argv[2])
if gen == 's2orc':
    text, offs = synth.generate_parallel("s2orc", N, procs=4, seed=4)
else:
    text, offs = synth.random_ascii_corpus(N, 256, seed=1)
bt = text.tobytes()
def windows(s):
    out=[]; pos=0
    while pos < len(s):
        if len(s)-pos <= 256: out.append(s[pos:]); break
        cut = s.rfind(' ', pos+1, pos+256)
        if cut <= pos: cut = pos+256
        out.append(s[pos:cut]); pos = cut
    return out
def lanes_of(text):
    atoms, wsf, cpos = LM.window(text)
    na=len(atoms)
    em=[0]*(na+1)
    for j in range(na):
        s=""
        for L in range(1,17):
            if j+L>na or (L>1 and wsf[j+L-1]): break
            s+=atoms[j+L-1]
            if s in vocab: em[j+L] |= 1<<(L-1)
    C=((na+15)>>4)|1
    lanes=[]
    for d in range(16):
        c0=min(d*C,na); c1=min(c0+C,na); mloc,lcut=0xFFFF,0
        for k in range(16,-1,-1):
            i=c0+1+k
            if i<=c1:
                hb=max(em[i].bit_length()-1,0)
                mloc=min(mloc,i-1-hb)
                if mloc>=i-1: lcut|=1<<k
        lanes.append(dict(c0=c0,c1=c1,mloc=mloc,lcut=lcut))
    for d in range(16):
        S=min([l["mloc"] for l in lanes[d+1:]]+[0xFFFF]); c0=lanes[d]["c0"]; lcut=lanes[d]["lcut"]
        cut=0 if S<c0 else (lcut if S-c0>=16 else lcut&((2<<(S-c0))-1))
        lanes[d]["fc"]=c0+((cut&-cut).bit_length()-1) if cut else na
        lanes[d]["lc"]=c0+cut.bit_length()-1 if cut else 0
    for d in range(16): lanes[d]["rs"]=min([l["fc"] for l in lanes[d:]])
    for d in range(16):
        c0=lanes[d]["c0"]; prev=max([l["lc"] for l in lanes[:d]]+[0])
        if c0-prev < lanes[d]["rs"]-c0: lanes[d]["rs"]=prev
    for d in range(16): lanes[d]["re"]=lanes[d+1]["rs"] if d<15 else na
    out=[]
    for l in lanes:
        out.append([bin(em[i]>>1).count('1') for i in range(l["rs"]+1,l["re"]+1)])
    return out
A,B=30,22
allw=[]
for i in range(N):
    s=bt[offs[i]:offs[i+1]].decode('utf-8','replace')
    allw += windows(s)
tot_real=0; tot_ideal=0; tot_rowideal=0; iters_real=0; iters_ideal=0
for w0 in range(0, len(allw)-3, 4):
    L=[]
    for w in allw[w0:w0+4]:
        try: L += lanes_of(w)
        except Exception as e: L += [[] for _ in range(16)]
    T=max(len(x) for x in L)
    cost=0
    for t in range(T):
        mc=max((x[t] for x in L if t < len(x)), default=0)
        cost += A + B*mc
    ideal=sum(A*len(x)+B*sum(x) for x in L)/64
    tot_real+=cost; tot_ideal+=ideal
    iters_real+=T; iters_ideal+=sum(len(x) for x in L)/64
print(gen, "windows", len(allw), "B cost real/ideal", tot_real/tot_ideal, "iterations real/ideal", iters_real/iters_ideal)

# ---- alternatives: optimal partition per row (min max chunk work), and flattened loops
def row_data(text):
    atoms, wsf, cpos = LM.window(text)
    na=len(atoms)
    em=[0]*(na+1)
    for j in range(na):
        s=""
        for L in range(1,17):
            if j+L>na or (L>1 and wsf[j+L-1]): break
            s+=atoms[j+L-1]
            if s in vocab: em[j+L] |= 1<<(L-1)
    # cuts: p in [0, na] with min_{i>p} lo_i >= p
    lo=[0]*(na+1)
    for i in range(1,na+1): lo[i]=i-1-max(em[i].bit_length()-1,0)
    cuts=[]; m=10**9
    for p in range(na,-1,-1):
        if m >= p: cuts.append(p)
        if p>=1: m=min(m,lo[p])
    cuts=sorted(set(cuts))
    cands=[0]+[bin(em[i]>>1).count('1') for i in range(1,na+1)]
    return na,cuts,cands
def opt_chunks(na,cuts,cands,K=16):
    # positions (p, q] between cuts; work per position A + B*cands; min max over <=K chunks: binary search
    w=[0]*(na+1)
    pre=[0]*(na+1)
    for i in range(1,na+1): pre[i]=pre[i-1]+A+B*cands[i]
    def feasible(L):
        k=0; cur=0; ci=0
        # greedy: from cut cur, go to the furthest cut c with pre[c]-pre[cur] <= L
        idx=0
        while cur < na:
            best=None
            for c in cuts:
                if c>cur and pre[c]-pre[cur] <= L: best=c
            if best is None: return None
            k+=1; cur=best
            if k>K: return None
        return k
    lo_,hi_=0,pre[na]
    while lo_<hi_:
        mid=(lo_+hi_)//2
        if feasible(mid) is not None: hi_=mid
        else: lo_=mid+1
    return lo_
tr=0; to=0; ti=0
for w0 in range(0, min(len(allw),1200)-3, 4):
    Lr=[]; opt=[]; ideal=0
    for w in allw[w0:w0+4]:
        try:
            L=lanes_of(w); Lr+=L
            na,cuts,cands=row_data(w); opt.append(opt_chunks(na,cuts,cands))
        except Exception: Lr+=[[] for _ in range(16)]; opt.append(0)
    T=max(len(x) for x in Lr)
    cost=0
    for t in range(T):
        mc=max((x[t] for x in Lr if t < len(x)), default=0)
        cost += A + B*mc
    # flattened per-lane work with current chunks: max over lanes of sum(A+B*c) -> each iteration costs A+B
    flat=max(sum(1+c for c in x) for x in Lr)*(A+B)
    tr+=cost; to+=max(opt); ti+=sum(A*len(x)+B*sum(x) for x in Lr)/64
    tflat=locals().get('tflat',0)+flat
print("current", tr/ti, "optimal-partition (work-sum per lane, perfect inner balance)", to/ti, "flattened current chunks", tflat/ti)

def weighted_chunks(na,cuts,cands,K=16):
    pre=[0]*(na+1)
    for i in range(1,na+1): pre[i]=pre[i-1]+A+B*cands[i]
    tot=pre[na]
    bounds=[0]
    for d in range(1,K):
        tgt=tot*d/K
        # nearest cut by work
        best=min(cuts, key=lambda c: abs(pre[c]-tgt))
        bounds.append(max(best,bounds[-1]))
    bounds.append(na)
    return max(pre[bounds[k+1]]-pre[bounds[k]] for k in range(K))
def nearest_pos_chunks(na,cuts,cands,K=16):
    pre=[0]*(na+1)
    for i in range(1,na+1): pre[i]=pre[i-1]+A+B*cands[i]
    C=((na+15)>>4)|1
    bounds=[0]
    for d in range(1,K):
        tgt=min(d*C,na)
        best=min(cuts, key=lambda c: (abs(c-tgt), -c))
        bounds.append(max(best,bounds[-1]))
    bounds.append(na)
    return max(pre[bounds[k+1]]-pre[bounds[k]] for k in range(K))
tw=0; tn=0; to2=0; ti2=0; trowideal=0
for w0 in range(0, min(len(allw),1200)-3, 4):
    ws_=[];wn=[];op=[];ii=0;ri=[]
    for w in allw[w0:w0+4]:
        try:
            na,cuts,cands=row_data(w)
        except Exception: continue
        ws_.append(weighted_chunks(na,cuts,cands)); wn.append(nearest_pos_chunks(na,cuts,cands)); op.append(opt_chunks(na,cuts,cands))
        work=sum(A+B*c for c in cands[1:]); ii+=work/64; ri.append(work/16)
    tw+=max(ws_); tn+=max(wn); to2+=max(op); ti2+=ii; trowideal+=max(ri)
print("per-lane work-sum model: nearest-pos", tn/ti2, "work-weighted", tw/ti2, "optimal", to2/ti2, "row-bound ideal", trowideal/ti2)
