"""Diagnostic: at the first divergent decode step, compare the last layer's q and K/V
caches (GPU vs oracle, device order) and recompute the divergent head's attention in
numpy under ggml's semantics (sequential double sums vs exact fsum), to say which side
leaves ggml's arithmetic."""
import ctypes as C
import math
import sys

sys.path.insert(0, "llama-gguf-inference_amd"); sys.path.insert(0, "oracle"); sys.path.insert(0, "tests")
import numpy as np
import torch

torch.zeros(1, device="cuda")
import llmi
from llmi._lib import lib
import pyoracle as po

preset = sys.argv[1] if len(sys.argv) > 1 else "tiny-mixed-d128"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 37
n_layer = int(sys.argv[3]) if len(sys.argv) > 3 else 1
path = f"/tmp/{preset}-L{n_layer}.gguf"
llmi.write_synthetic_gguf(path, preset, seed=1, n_layer=n_layer)
rng = np.random.default_rng(11 + n)
prompt = [1] + [int(t) for t in rng.integers(3, 700, n - 1)]
po.set_dot_order(po.DEVICE_ORDER)
NC = max(128, n + 8)
om = po.OracleModel(path, n_ctx=NC)
m = llmi.Model(path)
c = llmi.Context(m, n_ctx=NC)
H, HK = m.n_head, m.n_head_kv; D = m.n_embd // H
G = H // HK
L = po.lib()
def otap(w, size, dt=np.float32):
    b = np.zeros(size, dt); L.or_tap(om._h, w, b.ctypes.data_as(C.c_void_p)); return b
def gtap(w, size, dt=np.float32):
    b = np.zeros(size, dt); assert lib().llmi_debug_tap(c._h, w, b.ctypes.data_as(C.c_void_p)) == 0; return b
h2f = lambda u: u.view(np.float16).astype(np.float32)
f2h = lambda x: x.astype(np.float32).astype(np.float16)
expf = lambda x: np.float32(L.or_expf(C.c_float(float(x))))
L.or_expf.restype = C.c_float; L.or_expf.argtypes = [C.c_float]

def attn(q, K, V, pos, exact):
    out = np.zeros(H * D, np.float32); P = []
    scale = np.float32(1.0) / np.sqrt(np.float32(D))
    for h in range(H):
        g = h // G
        qh = h2f(f2h(q[h * D:(h + 1) * D]).view(np.uint16))
        w = np.zeros(pos + 1, np.float32)
        for t in range(pos + 1):
            prods = (h2f(K[t, g]) * qh).astype(np.float32)  # exact f32 products
            s = math.fsum(map(float, prods)) if exact else sum(float(p) for p in prods)
            w[t] = np.float32(s) * scale
        mx = w.max()
        e = np.array([expf(x - mx) for x in w], np.float32)
        S = math.fsum(map(float, e)) if exact else sum(float(x) for x in e)
        inv = np.float32(1.0 / S)
        p = h2f(f2h(e * inv).view(np.uint16)); P.append(p)
        for d in range(D):
            prods = (h2f(V[:pos + 1, g, d]) * p).astype(np.float32)
            out[h * D + d] = np.float32(math.fsum(map(float, prods)) if exact else sum(float(x) for x in prods))
    return out, P

for pos, t in enumerate(prompt):
    lo = om.decode(t, pos)
    assert c.decode([t], pos=[pos]) == 0
    lg = c.logits(-1)
    oa, ga = otap(3, H * D), gtap(3, H * D)
    if float(np.abs(lg - lo).max()) == 0 and np.array_equal(oa, ga):
        continue
    print("first divergence at pos", pos, "tok", t, "logit diff", float(np.abs(lg - lo).max()))
    oq, gq = otap(2, H * D), gtap(2, H * D)
    print("q equal:", np.array_equal(oq, gq))
    ok = otap(7, om.n_ctx * HK * D, np.uint16).reshape(-1, HK, D)
    ov = otap(8, om.n_ctx * HK * D, np.uint16).reshape(-1, HK, D)
    GN = c.n_ctx
    gk = gtap(7, HK * GN * D, np.uint16).reshape(HK, GN, D).transpose(1, 0, 2)
    gv = gtap(8, HK * D * GN, np.uint16).reshape(HK, D, GN).transpose(2, 0, 1)
    print("K cache equal:", np.array_equal(ok[:pos + 1], gk[:pos + 1]), "V cache equal:", np.array_equal(ov[:pos + 1], gv[:pos + 1]))
    for nm, K, V in (("oracle-cache", ok, ov), ("gpu-cache", gk, gv)):
        for exact in (False, True):
            a, P = attn(oq, K, V, pos, exact)
            print(nm, "exact" if exact else "seq", "== oracle att:", np.array_equal(a, oa), "== gpu att:", np.array_equal(a, ga),
                  "maxdiff vs oracle", float(np.abs(a - oa).max()), "vs gpu", float(np.abs(a - ga).max()))
    hd = np.nonzero(np.abs(oa - ga).reshape(H, D).max(1))[0]
    print("differing heads", hd.tolist())
    np.savez("gpurun_out/d9.npz", q=oq, K=ok[:pos + 1], V=ov[:pos + 1], oa=oa, ga=ga, pos=pos, H=H, HK=HK, D=D)
    break
print("done")
