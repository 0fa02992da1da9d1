#!/usr/bin/env python3
"""Time rqsid_assign per encode level on the bench workload (HIP events), for A/B of kernel variants
selected by environment variables (run once per variant)."""
import os
import sys
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import bench  # noqa: E402
from generative_ranking_recommender_amd import ops, synth  # noqa: E402
import generative_ranking_recommender_amd.encode as encmod  # noqa: E402
from generative_ranking_recommender_amd.encode import HIERARCHICAL_TRAIN, RQEncoder  # noqa: E402


def main(n=int(os.environ.get("SWEEP_ROWS", 10_000_000)), reps=int(os.environ.get("SWEEP_REPS", 5))):
    dev = torch.device("cuda", 0)
    cache = os.environ.get("SWEEP_CB")  # codebooks fitted once with the real library (A/B builds reuse them)
    if cache and os.path.exists(cache):
        z = np.load(cache)
        cb = {k: z[k] for k in z.files}
    else:
        cb = bench.codebooks(os.environ.get("BENCH_CODEBOOKS", "fitted"), dev)
        if cache:
            np.savez(cache, **cb)
    enc = RQEncoder([torch.from_numpy(cb[k]) for k in ("c0", "c1", "c2")], [128, 128, 256],
                    match=torch.from_numpy(cb["match"]), semantics=HIERARCHICAL_TRAIN, device=dev)
    x = bench.make_rows(n, 0, dev)
    for _ in range(2):
        enc.encode(x)
    timer = bench.Timed()
    orig = ops.assign
    lvl = {"i": 0}

    def hook(*a, **k):
        name = f"L{lvl['i']}"
        lvl["i"] += 1
        return timer.wrap(name, orig)(*a, **k)

    encmod.ops.assign = hook
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        lvl["i"] = 0
        enc.encode(x)
    e.record()
    torch.cuda.synchronize()
    ms = timer.mean_ms()
    encmod.ops.assign = orig
    enc.encode(x, count_rescored=True)
    print(f"lib={os.environ.get('RQSID_LIB', 'default')} variant={os.environ.get('RQSID_SCREEN_VARIANT', '0')} step={s.elapsed_time(e) / reps:.2f} ms " +
          " ".join(f"{k}={v:.3f}" for k, v in sorted(ms.items())) + f" rescored={list(enc.last_rescored)}", flush=True)


if __name__ == "__main__":
    main()
