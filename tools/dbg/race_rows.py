#!/usr/bin/env python3
"""Diagnostics (GPU): rows where the resident screen (variant 6) differs from the per-tile screen on the
partial-tile nearest case; prints tile / row-in-tile / block structure of the mismatches."""
import os
import sys
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent.parent))
from generative_ranking_recommender_amd import ops  # noqa: E402


def run(var, x, pc):
    os.environ["RQSID_SCREEN_VARIANT"] = var
    return ops.nearest(x, pc).cpu().numpy()


for k in [int(v) for v in os.environ.get("RACE_KS", "128,200").split(",")]:
    rng = np.random.default_rng(k)
    c = rng.standard_normal((k, 512)).astype(np.float32)
    x = (c[rng.integers(0, k, 30000)] + 0.3 * rng.standard_normal((30000, 512))).astype(np.float32)
    xg, pc = torch.from_numpy(x).cuda(), ops.prepare_centers(torch.from_numpy(c).cuda())
    for rep in range(3):
        got = run("6", xg, pc)  # the test's order: the resident form first, then the per-tile reference
        ref = run("1", xg, pc)
        bad = np.nonzero(got != ref)[0]
        tiles = np.unique(bad // 32)
        print(f"k={k} rep={rep}: {len(bad)} rows differ in {len(tiles)} tiles; first rows {bad[:12].tolist()}; "
              f"rows-in-tile {np.unique(bad % 32)[:20].tolist()}; got {got[bad[:6]].tolist()} ref {ref[bad[:6]].tolist()}",
              flush=True)
