"""XL level-2 candidate overlap between (l1, l2) groups (diagnostic for packing two groups into one screen tile:
a packed tile streams the union of its groups' candidate sets once, so it pays only when that union is much
smaller than the two sets).  Reports, on the fitted XL codebooks, the overlap of each group with its segment-order
neighbour, with its best partner under the same level-0 parent, and with its best partner anywhere."""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import bench  # noqa: E402

bench.NEED, bench.N_CAND, bench.PRESET = [256, 256, 512], 5120, "xl"
dev = torch.device("cuda", 0)
cb = bench.fitted_codebooks(dev)
m = torch.from_numpy(cb["match"]).to(dev).half()  # [groups, 5120]
G, K = m.shape
per = int(m[0].sum().item())
q = torch.tensor([0.1, 0.5, 0.9], device=dev)


def show(name, ov):
    ov = ov.float()
    print(f"{name}: overlap quantiles (10/50/90 %) {[round(v) for v in torch.quantile(ov, q).tolist()]} of {per}, "
          f"mean {ov.mean().item():.1f}", flush=True)


show("segment-order neighbour", (m[:-1] * m[1:]).sum(1))
P = bench.NEED[1]
best_par = torch.empty(G, device=dev)
for p in range(G // P):
    blk = m[p * P:(p + 1) * P]
    o = blk @ blk.T
    o.fill_diagonal_(0)
    best_par[p * P:(p + 1) * P] = o.max(1).values.float()
show("best partner, same level-0 parent", best_par)
best = torch.empty(G, device=dev)
for s in range(0, G, 2048):
    o = m[s:s + 2048] @ m.T
    idx = torch.arange(s, min(s + 2048, G), device=dev)
    o[idx - s, idx] = 0
    best[s:s + 2048] = o.max(1).values.float()
show("best partner, any group", best)
