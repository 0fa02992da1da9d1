#!/usr/bin/env python3
"""Diagnostics (GPU): segment sizes of the encode's L1 / L2 segments on the bench workload and the
row-slot fill of 128- and 256-row tiles (rows / (tiles * tile_rows)): the share of screen work spent on
padding rows of partial tiles."""
import os
import sys
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from generative_ranking_recommender_amd import synth  # noqa: E402
from generative_ranking_recommender_amd.encode import HIERARCHICAL_TRAIN, RQEncoder  # noqa: E402
import bench  # noqa: E402


def main(n=10_000_000):
    dev = torch.device("cuda", 0)
    cb = bench.codebooks(os.environ.get("BENCH_CODEBOOKS", "fitted"), dev)
    enc = RQEncoder([torch.from_numpy(cb[k]) for k in ("c0", "c1", "c2")], [128, 128, 256],
                    match=torch.from_numpy(cb["match"]), semantics=HIERARCHICAL_TRAIN, device=dev)
    x = torch.from_numpy(synth.mixture_rows(0, n)).to(dev)
    ids = enc.encode(x).cpu().numpy().astype(np.int64)
    for name, key, nseg in (("L1", ids[:, 0], 128), ("L2", ids[:, 0] * 128 + ids[:, 1], 16384)):
        sz = np.bincount(key, minlength=nseg)
        nz = sz[sz > 0]
        q = np.percentile(nz, [1, 10, 50, 90, 99])
        line = f"{name}: {len(nz)} non-empty segments of {nseg}, rows/segment p1/p10/p50/p90/p99 = " + \
            "/".join(f"{v:.0f}" for v in q)
        for t in (64, 128, 256):
            tiles = int(np.ceil(nz / t).sum())
            line += f"; {t}-row tiles {tiles} fill {n / (tiles * t):.3f}"
        print(line, flush=True)


if __name__ == "__main__":
    main(*(int(a) for a in sys.argv[1:]))
