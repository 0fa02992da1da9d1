#!/usr/bin/env python3
"""Diagnostics (GPU, stamps build: tools/ab_build.sh with EXTRA=-DRQSID_STAMPS): per encode level, the
screen kernel's (stream or per-tile) wave-0 cycles per block split into chunk waits, epilogue and the rest."""
import ctypes
import os
import sys
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import bench  # noqa: E402
from generative_ranking_recommender_amd import _lib, ops  # noqa: E402
import generative_ranking_recommender_amd.encode as encmod  # noqa: E402
from generative_ranking_recommender_amd.encode import HIERARCHICAL_TRAIN, RQEncoder  # noqa: E402


def main(n=int(os.environ.get("SWEEP_ROWS", 10_000_000))):
    dev = torch.device("cuda", 0)
    z = np.load(os.environ["SWEEP_CB"])
    cb = {k: z[k] for k in z.files}
    enc = RQEncoder([torch.from_numpy(cb[k]) for k in ("c0", "c1", "c2")], [128, 128, 256],
                    match=torch.from_numpy(cb["match"]), semantics=HIERARCHICAL_TRAIN, device=dev)
    x = bench.make_rows(n, 0, dev)
    lib = _lib.load()
    fn = lib.rqsid_debug_stamps if os.environ.get("RQSID_SCREEN_VARIANT") == "5" else lib.rqsid_debug_stamps_tile
    fn.argtypes = [ctypes.c_void_p]
    buf = (ctypes.c_ulonglong * 8)()
    enc.encode(x)
    torch.cuda.synchronize()
    fn(buf)
    orig = ops.assign
    res = []

    def hook(*a, **k):
        out = orig(*a, **k)
        torch.cuda.synchronize()
        fn(buf)
        res.append(list(buf))
        return out

    encmod.ops.assign = hook
    enc.encode(x)
    stream = os.environ.get("RQSID_SCREEN_VARIANT") == "5"
    if stream and os.environ.get("RQSID_STREAM_SHAPE") == "88":  # ping-pong: per group {total, wait, compute, epilogue}
        for lvl, v in enumerate(res):
            for g in (0, 1):
                tot, wt, cp, ep = v[4 * g:4 * g + 4]
                f = lambda x: f"{100 * x / max(tot, 1):.1f}%"
                print(f"L{lvl} group {g}: cycles {tot:.4g}  wait+barrier {f(wt)}  compute {f(cp)}  epilogue {f(ep)}  "
                      f"issue/header {f(tot - wt - cp - ep)}", flush=True)
        return
    for lvl, (tot, wt, ep, x, pro, *_) in enumerate(res):
        # x = cycles in the ring's DMA issue; pro = per-tile prologue (stream kernel: next-header steps)
        iss = x
        f = lambda v: f"{100 * v / max(tot, 1):.1f}%"
        print(f"L{lvl}: cycles {tot:.4g}  prologue {f(pro)}  wait {f(wt)}  dma issue {f(iss)}  epilogue {f(ep)}  "
              f"compute {f(tot - wt - ep - iss - pro)}", flush=True)


if __name__ == "__main__":
    main()
