#!/usr/bin/env python3
"""Diagnostics (GPU, stamps build: EXTRA=-DRQSID_STAMPS MODES=0 tools/ab_build.sh): per encode level, the
warp-specialised resident screen's cycles per tile for candidate wave 0 and producer wave 8, by phase."""
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

PH = {0: {0: "loop", 1: "wait_ready", 2: "mfma", 3: "reload", 5: "e2_wait_posted", 6: "e2", 4: "epi1"},
      1: {0: "loop", 1: "wait_consumed", 2: "segprep", 3: "produce"}}


def main(n=int(os.environ.get("SWEEP_ROWS", 10_000_000))):
    dev = torch.device("cuda", 0)
    z = np.load(os.environ["SWEEP_CB"])
    cb = {k: z[k] for k in z.files}
    enc = RQEncoder([torch.from_numpy(cb[k]) for k in ("c0", "c1", "c2")], [128, 128, 256],
                    match=torch.from_numpy(cb["match"]), semantics=HIERARCHICAL_TRAIN, device=dev)
    x = bench.make_rows(n, 0, dev)
    lib = _lib.load()
    fn = lib.rqsid_debug_stamps_res
    fn.argtypes = [ctypes.c_void_p]
    buf = (ctypes.c_ulonglong * 32)()
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
    for lvl, v in enumerate(res):
        for role in (0, 1):
            w = v[16 * role:16 * role + 16]
            tiles = max(w[7], 1)
            if w[0] == 0:
                continue
            parts = " ".join(f"{name}={w[k] / tiles:.0f}" for k, name in PH[role].items())
            print(f"L{lvl} {'producer' if role else 'candidate'}: cycles/tile {parts}  (tiles {w[7]})", flush=True)


if __name__ == "__main__":
    main()
