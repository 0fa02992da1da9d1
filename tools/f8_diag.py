import sys
sys.path.insert(0, "tests"); sys.path.insert(0, ".")
import numpy as np, torch
from test_mfma_numerics import e4m3_bits, _e4m3_values
from generative_ranking_recommender_amd import _lib
DEV = torch.device("cuda", 0)
lib = _lib.load()
def probe(a, b, c=None):
    c = np.zeros((32, 32), np.float32) if c is None else c
    ta = torch.from_numpy(e4m3_bits(a)).to(DEV); tb = torch.from_numpy(e4m3_bits(b)).to(DEV)
    tc = torch.from_numpy(c).to(DEV); td = torch.empty((32, 32), dtype=torch.float32, device=DEV)
    _lib.check(lib.rqsid_mfma_probe(2, ta.data_ptr(), tb.data_ptr(), tc.data_ptr(), td.data_ptr(), torch.cuda.current_stream().cuda_stream), "p")
    torch.cuda.synchronize(); return td.cpu().numpy().astype(np.float64)
rng = np.random.default_rng(11)
for name, lo in (("with subnormals", -9), ("normals only", -6)):
    worst = 0; nexact = 0; tot = 0
    for _ in range(6):
        def vals(shape):
            e = rng.integers(lo, 9, shape); f = rng.integers(0, 8, shape) / 8.0
            v = np.where(e < -6, 2.0 ** e, (1 + f) * 2.0 ** e); v = np.minimum(v, 448.0)
            return v * rng.choice([-1.0, 1.0], shape)
        a = vals((32, 64)); b = vals((64, 32))
        d = probe(a, b); ex = a @ b
        pmax = (np.abs(a)[:, :, None] * np.abs(b)[None]).max(1)
        r = (np.abs(d - ex) - 2.0 ** -24 * np.abs(d)) / (2.0 ** -23 * pmax)
        worst = max(worst, r.max()); nexact += (d == ex.astype(np.float32)).sum(); tot += d.size
    print(name, "worst ratio", worst, "exact fraction", nexact / tot)
# subnormal flush probe: one product 2^-9 * 1
a = np.zeros((32, 64)); b = np.zeros((64, 32)); a[0, 0] = 2.0 ** -9; b[0, 0] = 1.0; a[1, 0] = 2.0 ** -6; b[0, 1] = 1.0
d = probe(a, b); print("subnormal x 1 ->", d[0, 0], "min normal x 1 ->", d[1, 1])
# alignment: one big product 2^16 plus 16 products of 2^-8 (half an fp32 ulp of 2^16)
a = np.zeros((32, 64)); b = np.zeros((64, 32)); a[2, 0] = 256; b[0, 2] = 256
for k in range(1, 17): a[2, k] = 2.0 ** -4; b[k, 2] = 2.0 ** -4
d = probe(a, b); print("2^16 + 16 x 2^-8 ->", d[2, 2] - 65536, "exact 0.0625")
