"""Self-synchronisation distance of the Exp-Golomb stream (the decode's resolve walk).

For every 512-bit chunk of the oracle-written stream of a 1080p-wide slice, a parse from the chunk's
first bit is followed until it lands on a true code boundary; prints the distance distribution.
CPU only; the oracle is the stream writer (test infrastructure).  Usage: python tools/eg_sync_sim.py [ramp|uniform]"""
import os, sys, numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO); sys.path.insert(0, os.path.join(REPO, 'oracle'))
import importlib; pkg=importlib.import_module('3ddctvideoencoding_amd'); import oracle
fr = pkg.synthetic.frames(1920, 1080, 8, kind=sys.argv[1] if len(sys.argv)>1 else "ramp")[:, :256, :]
fr = np.ascontiguousarray(fr)
plan = oracle.Plan(8,8,8)
q = plan.encode_q(fr)
vals = q.reshape(-1,512)[:, pkg.diagonal_order(8,8,8)].ravel().astype(np.int64)
code = np.where(vals<=0, -2*vals, 2*vals-1)+1
n = np.floor(np.log2(code.astype(np.float64))).astype(np.int64)+1
L = 2*n-1
print("values", vals.size, "bits", L.sum(), "bits/value", L.sum()/vals.size)
bits = np.unpackbits(np.frombuffer(oracle.eg_write(vals.astype(np.int32)), np.uint8))[:L.sum()]
N = bits.size
true = np.zeros(N+1, bool); true[np.concatenate([[0], np.cumsum(L)])] = True
# zeros run length from each position
z = np.zeros(N+1, np.int64)
for i in range(N-1, -1, -1):
    z[i] = 0 if bits[i] else z[i+1]+1
ds=[]
for s in range(512, N-2000, 512):
    p = s
    while not true[p]:
        p += 2*z[p]+1
    ds.append(p-s)
ds=np.array(ds)
print("chunks", ds.size, "d percentiles 50/90/99/99.9/max", np.percentile(ds,[50,90,99,99.9]), ds.max())
for w in (64,128,256,512):
    print("frac d>=%d: %.5f" % (w, (ds>=w).mean()))
