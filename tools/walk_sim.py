"""The resolve walk's step counts (eg_sync_kernel's resolve_block), simulated on the CPU.

For every 512-bit chunk of the oracle-written stream of a 1080p-wide slice (256 rows, 8 frames): the walk
of the pass-0 parse (from the chunk's first bit) and the true parse (from the true exit of the chunk
before) as the kernel steps it (a run of 1-bit codes, then the table's codes when they end at or before
the other parse, else one code); the per-chunk step distribution, the maximum over a wave's 63 chunks
(what a SIMT wave pays), then the same with a boundary-mask table, and the per-block cost of walking
kWalkSimt steps per lane and queueing the rest for one wave.  Test / study infrastructure (uses oracle/).
    python tools/walk_sim.py [ramp|uniform]"""
import os, sys, numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO); sys.path.insert(0, os.path.join(REPO, 'oracle'))
import importlib; pkg=importlib.import_module('3ddctvideoencoding_amd'); import oracle
kind=sys.argv[1] if len(sys.argv)>1 else "ramp"
fr = pkg.synthetic.frames(1920, 1080, 8, kind=kind)[:, :256, :]
fr = np.ascontiguousarray(fr)
plan = oracle.Plan(8,8,8)
q = plan.encode_q(fr)
vals = q.reshape(-1,512)[:, pkg.diagonal_order(8,8,8)].ravel().astype(np.int64)
code = np.where(vals<=0, -2*vals, 2*vals-1)+1
n = np.floor(np.log2(code.astype(np.float64))).astype(np.int64)+1
L = 2*n-1
bits = np.unpackbits(np.frombuffer(oracle.eg_write(vals.astype(np.int32)), np.uint8))[:L.sum()]
N = bits.size
true = np.zeros(N+200, bool); true[np.concatenate([[0], np.cumsum(L)])] = True
bits = np.concatenate([bits, np.ones(200, np.uint8)])
z = np.zeros(N+200, np.int64)
for i in range(N+199, -1, -1):
    z[i] = 0 if bits[i] else (z[i+1]+1 if i+1 < N+200 else 1)
def nxt(p): return p + 2*z[p] + 1
def run1(p):  # ones starting at p, capped at 31
    k=0
    while k<31 and bits[p+k]: k+=1
    return k
def lut(p):  # codes complete in next 12 bits, bits taken
    q=p; k=0
    while True:
        w=2*z[q]+1
        if q+w-p>12: break
        q+=w; k+=1
    return k, q-p
def pass0_exit(s, end):
    p=s
    while p<end: p=nxt(p)
    return p
iters=[]; unmet=0
for t in range(1, N//512 - 4):
    s=512*t
    # true exit of chunk t-1: first true boundary >= s
    e=s
    while not true[e]: e+=1
    x0=pass0_exit(s, s+512)
    pa, pq = s, e; it=0
    while True:
        if pa==pq: break
        behind, ahead = min(pa,pq), max(pa,pq)
        if behind - s >= 128: unmet+=1; break
        n1=run1(behind)
        it+=1
        if behind+n1>=ahead: adv=ahead-behind
        else:
            p1=behind+n1
            code = not bits[p1] if n1==31 else True
            k,wt=lut(p1)
            if k and behind+n1+wt<=ahead: adv=n1+wt
            elif code: adv=n1+2*z[p1]+1
            else: adv=n1
        if pa<pq: pa+=adv
        else: pq+=adv
    iters.append(it)
iters=np.array(iters)
print(kind, "chunks", iters.size, "unmet", unmet, "mean iters", iters.mean(), "pct 50/90/99", np.percentile(iters,[50,90,99]), "max", iters.max())
w=iters[:iters.size//63*63].reshape(-1,63).max(1)
print("per-wave max: mean", w.mean(), "pct 50/90", np.percentile(w,[50,90]))

def lutb(p):  # codes complete in next 12 bits: count, bits, boundary offsets (starts of codes 2..k and end)
    q=p; k=0; bnd=[]
    while True:
        w=2*z[q]+1
        if q+w-p>12: break
        q+=w; k+=1; bnd.append(q-p)
    return k, q-p, bnd
iters2=[]
for t in range(1, N//512 - 4):
    s=512*t
    e=s
    while not true[e]: e+=1
    pa, pq = s, e; it=0
    while pa!=pq:
        behind, ahead = min(pa,pq), max(pa,pq)
        if behind - s >= 128: break
        n1=run1(behind); it+=1
        if behind+n1>=ahead: adv=ahead-behind
        else:
            p1=behind+n1
            k,wt,bnd=lutb(p1)
            if k:
                if ahead-p1 in bnd: adv=ahead-behind   # meets inside the table codes
                else: adv=n1+wt
            else:
                code = not bits[p1] if n1==31 else True
                adv = n1+2*z[p1]+1 if code else n1
        if pa<pq: pa+=adv
        else: pq+=adv
    iters2.append(it)
iters2=np.array(iters2)
print("mask-table walk: mean", iters2.mean(), "pct 50/90/99", np.percentile(iters2,[50,90,99]), "max", iters2.max())
w=iters2[:iters2.size//63*63].reshape(-1,63).max(1)
print("per-wave max: mean", w.mean(), "pct 50/90", np.percentile(w,[50,90]))

for W in (2,3,4,6):
    nb=iters.size//252
    a=iters[:nb*252].reshape(nb,4,63)
    now=a.max(2).sum(1).mean()
    comp=(np.minimum(a.max(2),W).sum(1) + np.maximum(a-W,0).reshape(nb,-1).max(1)).mean()
    print("W",W,"per-block walk iterations: now",now,"compacted",comp)
