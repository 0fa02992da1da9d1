"""Re-score cliff diagnosis: time one exact `nearest` of rows against K centres whose
fp16 screen bound admits many candidates, with and without the fp32 re-screen, and histogram the work items
the screen / re-screen left (n = -1: every candidate).  Inputs: 'iso' = random unit vectors; 'r2' = the
bench's normalised level-2 residual rows (bench.fitted_codebooks' construction) against K of those rows
(the first iteration of its K=2560 Lloyd fit)."""
import json
import os
import sys
import time
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import bench  # noqa: E402
from generative_ranking_recommender_amd import ops  # noqa: E402


def r2_rows(n, dev):
    gen = torch.Generator(device=dev).manual_seed(4321)
    x = bench.make_rows(n, 10_000 + 4321, dev)
    c0 = bench._lloyd(x, 128, 10, gen)
    a0 = ops.nearest(x, ops.prepare_centers(c0))
    r1 = ops.residual(x, c0, a0, normalize=True)
    order = torch.argsort(a0, stable=True)
    cnt0 = torch.bincount(a0.long(), minlength=128).cpu().tolist()
    c1 = torch.empty((128 * 128, 512), dtype=torch.float32, device=dev)
    a1 = torch.empty(n, dtype=torch.int32, device=dev)
    start = 0
    for p in range(128):
        rows = order[start:start + cnt0[p]]
        start += cnt0[p]
        sub = r1[rows] if len(rows) else r1[:1]
        cp = bench._lloyd(sub, 128, 10, gen)
        c1[p * 128:(p + 1) * 128] = cp
        if len(rows):
            a1[rows] = ops.nearest(sub, ops.prepare_centers(cp)) + p * 128
    return ops.residual(r1, c1, a1, normalize=True), gen


def items(ws):
    b = ws.buf.cpu().numpy()
    cnt = int(b[:4].view(np.int32)[0])
    w = b[256:256 + 32 * cnt].view(np.int32).reshape(-1, 8)
    ns = w[:, 2]
    return {"items": cnt, "every_candidate": int((ns == -1).sum()), "listed": int((ns > 0).sum()),
            "n_hist": {int(k): int(v) for k, v in zip(*np.unique(ns, return_counts=True))}}


def main():
    dev = torch.device("cuda", 0)
    n, k = 1_000_000, 2560
    out = []
    for kind in ("iso", "r2"):
        if kind == "iso":
            g = torch.Generator(device=dev).manual_seed(7)
            x = torch.nn.functional.normalize(torch.randn((n, 512), device=dev, generator=g), dim=1)
            c = torch.nn.functional.normalize(torch.randn((k, 512), device=dev, generator=g), dim=1)
        else:
            x, gen = r2_rows(n, dev)
            c = x[torch.randperm(n, device=dev, generator=gen)[:k]].clone()
        if kind == "r2":
            # what the overflowing rows look like: NaN / zero rows and centres, and the fp64 distance
            # spread of a few rows' nearest candidates
            xs = x[:64].double()
            d = torch.cdist(xs, c.double()) ** 2
            srt = torch.sort(d, dim=1).values
            print(json.dumps({"input": kind, "nan_rows": int(torch.isnan(x).any(1).sum()),
                              "nan_centres": int(torch.isnan(c).any(1).sum()),
                              "zero_rows": int((x.abs().sum(1) == 0).sum()),
                              "zero_centres": int((c.abs().sum(1) == 0).sum()),
                              "row_norm_min_max": [float(x.norm(dim=1).min()), float(x.norm(dim=1).max())],
                              "unique_centres": int(torch.unique(c, dim=0).shape[0]),
                              "d2_best9_of_row0": [float(v) for v in srt[0, :9]],
                              "within_1e-4_of_min": [int(v) for v in ((srt - srt[:, :1]) <= 1e-4).sum(1)[:16]]}),
                  flush=True)
        pc = ops.prepare_centers(c)
        ws = ops.AssignWorkspace(n, dev)
        for nr in ("0", "1"):
            os.environ["RQSID_NO_RESCREEN"] = nr
            ops.nearest(x, pc, workspace=ws)
            torch.cuda.synchronize()
            t = time.perf_counter()
            a = ops.nearest(x, pc, workspace=ws)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t
            rec = {"input": kind, "rescreen": nr == "0", "ms": round(dt * 1e3, 2), **items(ws)}
            print(json.dumps(rec), flush=True)
            out.append(rec)
        os.environ["RQSID_NO_RESCREEN"] = "0"


if __name__ == "__main__":
    main()
