#!/usr/bin/env python3
"""Diagnostics (GPU): histogram of rqsid_assign's re-score work items per encode level
(n = listed candidates, -1 = every candidate, -2 = penalty) on the bench workload."""
import os
import sys
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from generative_ranking_recommender_amd import ops, synth  # noqa: E402
import generative_ranking_recommender_amd.encode as encmod  # noqa: E402
from generative_ranking_recommender_amd.encode import HIERARCHICAL_TRAIN, RQEncoder  # noqa: E402
import bench  # noqa: E402


def main(n=1_000_000, seed=99):
    dev = torch.device("cuda", 0)
    cb = bench.codebooks(os.environ.get("BENCH_CODEBOOKS", "fitted"), dev)
    enc = RQEncoder([torch.from_numpy(cb[k]) for k in ("c0", "c1", "c2")], [128, 128, 256],
                    match=torch.from_numpy(cb["match"]), semantics=HIERARCHICAL_TRAIN, device=dev)
    x = torch.from_numpy(synth.mixture_rows(0, n)).to(dev)
    orig = ops.assign
    lvl = {"i": 0}

    def hook(*a, **k):
        out = orig(*a, **k)
        ws = k.get("workspace")
        torch.cuda.synchronize()
        cnt = int(ws.buf[:4].view(torch.int32).item())
        nr = a[0].shape[0]
        allw = ws.buf[256:256 + 32 * nr].view(torch.int32).view(nr, 8)
        if lvl["i"] == 2 and os.environ.get("RQSID_SCREEN_VARIANT", "0") == "0":
            # the ping-pong form stores items at work[row] and lists the rows in the compact-list area
            off = 256 + 32 * nr + (nr * 4 + 255) // 256 * 256
            idx = ws.buf[off:off + 4 * cnt].view(torch.int32).long()
            items = allw[idx].cpu().numpy()
        else:
            items = allw[:cnt].cpu().numpy()
        ns = items[:, 2]
        vals, counts = np.unique(ns, return_counts=True)
        print(f"level {lvl['i']}: {cnt} items ({cnt / n:.2%}) " +
              " ".join(f"n={v}:{c}" for v, c in zip(vals, counts)), flush=True)
        lvl["i"] += 1
        return out

    encmod.ops.assign = hook
    enc.encode(x)


if __name__ == "__main__":
    main(*(int(a) for a in sys.argv[1:]))
