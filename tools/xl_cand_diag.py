"""XL level-2 candidate working sets: distinct candidate centres per XCD-contiguous tile range, for the current
segment order and for candidate-affinity orders of the (l1, l2) groups (diagnostic for DESIGN 3.1d)."""
import sys
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import bench  # noqa: E402

bench.NEED, bench.N_CAND, bench.PRESET = [256, 256, 512], 5120, "xl"
dev = torch.device("cuda", 0)
cb = bench.fitted_codebooks(dev)
m = torch.from_numpy(cb["match"]).to(dev)  # [groups, 5120] uint8
G, K = m.shape
# rows per group in the bench's row distribution (a 2M sample encoded by the nearest-centre chain is costly;
# use equal weights: the XCD split is by tiles, roughly by rows, and groups hold similar row counts)
def union_per_xcd(order):
    out = []
    for x in range(8):
        sel = order[x * G // 8:(x + 1) * G // 8]
        out.append(int((m[sel].amax(0) > 0).sum().item()))
    return out
ident = torch.arange(G, device=dev)
print("groups", G, "cands", K, "per group", int(m[0].sum()))
print("segment order (identity):", union_per_xcd(ident))
# affinity orders: by the group's lowest candidate column, by a 1-d projection of the candidate-set centroid
cols = m.float()
c2 = torch.from_numpy(cb["c2"]).to(dev)
cen = (cols @ c2) / cols.sum(1, keepdim=True).clamp(min=1)
u, s, v = torch.pca_lowrank(cen, q=8)
for q in range(3):
    print(f"order by PC{q}:", union_per_xcd(torch.argsort(cen @ v[:, q])))
# k-means(8) of the candidate-set centroids (Lloyd, 20 iterations)
g = torch.Generator(device=dev).manual_seed(0)
cc = cen[torch.randperm(G, device=dev, generator=g)[:8]].clone()
for _ in range(20):
    a = torch.cdist(cen, cc).argmin(1)
    for j in range(8):
        if (a == j).any():
            cc[j] = cen[a == j].mean(0)
a = torch.cdist(cen, cc).argmin(1)
print("k-means(8) cluster sizes", torch.bincount(a, minlength=8).tolist())
print("order by k-means(8) cluster:", union_per_xcd(torch.argsort(a, stable=True)))
