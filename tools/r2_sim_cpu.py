"""CPU restatement of the bench's fitted-codebook construction up to the level-2 residual rows r2 (bench.py
fitted_codebooks: K-Means(128) of the rows, per-parent K-Means(128) of the normalised level-1 residuals) and
what the first iteration of its K=2560 fit sees: zero residual rows (one-member clusters), zero centres among
2560 sampled rows, and how many rows have > 8 candidates within a distance gap (torch CPU, ~2 min).
Used to explain the re-score cliff."""
import torch, time, sys
from pathlib import Path
sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import bench
torch.set_num_threads(8)
dev = torch.device('cpu')
n = 1_000_000
t = time.time()
x = bench.make_rows(n, 10_000 + 4321, dev)
gen = torch.Generator(device=dev).manual_seed(4321)
def nearest(x, c):
    out = torch.empty(x.shape[0], dtype=torch.long)
    cn = (c.double() ** 2).sum(1)
    for i in range(0, x.shape[0], 65536):
        xb = x[i:i+65536].double()
        d = cn[None, :] - 2 * xb @ c.double().T
        out[i:i+65536] = d.argmin(1)
    return out
def lloyd(x, k, iters):
    n = x.shape[0]
    init = torch.randperm(n, generator=gen)[:k] if n >= k else torch.randint(0, n, (k,), generator=gen)
    c = x[init].clone()
    for _ in range(iters):
        a = nearest(x, c)
        s = torch.zeros((k, x.shape[1]), dtype=torch.float64).index_add_(0, a, x.double())
        cnt = torch.bincount(a, minlength=k)
        nz = cnt > 0
        c[nz] = (s[nz] / cnt[nz, None]).float()
    return c
def resid(x, c, a):
    r = x - c[a]
    return r / (r.norm(dim=1, keepdim=True) + 1e-8)
c0 = lloyd(x, 128, 10); a0 = nearest(x, c0); r1 = resid(x, c0, a0)
print('c0', time.time() - t, flush=True)
order = torch.argsort(a0, stable=True); cnt0 = torch.bincount(a0, minlength=128).tolist()
c1 = torch.empty((128 * 128, 512)); a1 = torch.empty(n, dtype=torch.long)
st = 0
for p in range(128):
    rows = order[st:st + cnt0[p]]; st += cnt0[p]
    sub = r1[rows] if len(rows) else r1[:1]
    cp = lloyd(sub, 128, 10); c1[p*128:(p+1)*128] = cp
    if len(rows): a1[rows] = nearest(sub, cp) + p * 128
print('c1', time.time() - t, flush=True)
r2 = resid(r1, c1, a1)
z = (r2.abs().sum(1) == 0)
sizes = torch.bincount(a1, minlength=128*128)
print('zero rows', int(z.sum()), 'singleton clusters', int((sizes == 1).sum()), 'empty', int((sizes == 0).sum()), flush=True)
cidx = torch.randperm(n, generator=gen)[:2560]
c = r2[cidx]
print('zero centres', int((c.abs().sum(1) == 0).sum()), 'unique', int(torch.unique(c, dim=0).shape[0]), flush=True)
xs = r2[:20000].double()
d = (c.double() ** 2).sum(1)[None, :] - 2 * xs @ c.double().T + (xs ** 2).sum(1)[:, None]
srt = torch.sort(d, 1).values
gap = srt - srt[:, :1]
for th in (1e-4, 1e-3, 4e-3):
    print(th, 'rows with >8 within', int(((gap <= th).sum(1) > 8).sum()), flush=True)
# exclude zero centres (dedup keeps one)
