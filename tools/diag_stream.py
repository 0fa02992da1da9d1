#!/usr/bin/env python3
"""Diagnostics (GPU): streamed vs per-tile screen, per level and for plain nearest at several k."""
import os
import sys
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from generative_ranking_recommender_amd import ops, synth  # noqa: E402
from generative_ranking_recommender_amd.encode import HIERARCHICAL_TRAIN, RQEncoder  # noqa: E402


def var(v, fn):
    os.environ["RQSID_SCREEN_VARIANT"] = str(v)
    out = fn()
    torch.cuda.synchronize()
    return out


dev = torch.device("cuda", 0)
rng = np.random.default_rng(0)
for k in (16, 100, 128, 256):
    for n in (20000, 70000):
        c = rng.standard_normal((k, 512)).astype(np.float32)
        x = (c[rng.integers(0, k, n)] + 0.3 * rng.standard_normal((n, 512))).astype(np.float32)
        pc = ops.prepare_centers(torch.from_numpy(c).to(dev))
        xg = torch.from_numpy(x).to(dev)
        a = var(5, lambda: ops.nearest(xg, pc).cpu().numpy())
        b = var(0, lambda: ops.nearest(xg, pc).cpu().numpy())
        bad = np.nonzero(a != b)[0]
        print(f"nearest k={k} n={n}: {len(bad)} differ; first rows {bad[:8].tolist()} stream {a[bad[:8]].tolist()} "
              f"tile {b[bad[:8]].tolist()}", flush=True)
cb = synth.encode_codebooks(seed=5, need=(16, 16, 32), n_cand=320, pool_rows=8192)
x = torch.from_numpy(synth.mixture_rows(0, 40000)).to(dev)
enc = RQEncoder([torch.from_numpy(cb[k]) for k in ("c0", "c1", "c2")], [16, 16, 32],
                match=torch.from_numpy(cb["match"]), semantics=HIERARCHICAL_TRAIN, device=dev)
a = var(5, lambda: enc.encode(x).cpu().numpy())
b = var(0, lambda: enc.encode(x).cpu().numpy())
print("encode small per level differ:", [(int((a[:, l] != b[:, l]).sum())) for l in range(3)], flush=True)
