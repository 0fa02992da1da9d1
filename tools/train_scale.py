"""Training cost at scale: one iteration of every phase of HierarchicalRQKMeans.train at
the PROD shape ([128,1280,1280] / need [128,128,256]) timed on N rows resident in HBM, multiplied by the
reference's iteration schedule (_calculate_adaptive_iter_limit, hierarchical_rq_kmeans.py:288-366; 20
for the candidate fits, :787) into a projected end-to-end training time.  Complements tools/train_bench.py,
which runs the whole trainer (feasible to ~1M rows inside one GPU call).

Phases (each = the trainer's own ops, see balancekmeans.batched_fit / KMeans.fit):
  level0      balanced fit_by_min_loss iteration, K=128: fp16 scores, auction_lap_half, centroid update,
              min-loss nearest histogram
  middle      one lockstep iteration of the 128 parents' balanced sub-fits (K=128 each)
  candidates  one balanced fit iteration with K=1280 (fp16 cdist, pairwise_distance_half), x2 fits
  groups      one lockstep iteration of the (l1,l2) groups' sub-fits (K=256; groups >= 512 rows)

    python tools/train_scale.py --rows 10000000 --out gpurun_out/train_scale.json
"""
import argparse
import json
import sys
import time
from pathlib import Path

import numpy as np
import torch

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO))
from generative_ranking_recommender_amd import ops  # noqa: E402
from generative_ranking_recommender_amd.hierarchical_rq_kmeans import adaptive_iter_limit  # noqa: E402

import bench  # noqa: E402  (make_rows)


def timed(fn, reps=1):
    fn()  # warm-up (workspaces, graph capture)
    torch.cuda.synchronize()
    t = time.perf_counter()
    out = None
    for _ in range(reps):
        out = fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps, out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=10_000_000)
    ap.add_argument("--out", default="")
    ap.add_argument("--preset", choices=("prod", "xl"), default="prod",
                    help="prod: need [128,128,256], lc [128,1280,1280]; xl (configs[4]): need [256,256,512], "
                         "lc [256,2560,2560] (run at its per-rank share, 6.25M rows)")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    n = a.rows
    need, lc = ([128, 128, 256], [128, 1280, 1280]) if a.preset == "prod" else ([256, 256, 512], [256, 2560, 2560])
    x = bench.make_rows(n, 0, dev)
    g = torch.Generator(device=dev).manual_seed(7)
    res = {"rows": n, "preset": a.preset, "need_clusters": need, "layer_clusters": lc, "phases": {}}

    # level 0: K=128 balanced fit_by_min_loss iteration
    c0 = x[torch.randperm(n, device=dev, generator=g)[:need[0]]].clone()

    def level0():
        w = ops.auction_scores(x, c0, half=False)
        a0, r = ops.auction(w)
        ops.centroid_update(x, a0, need[0], c0.clone())
        torch.bincount(ops.nearest(x, ops.prepare_centers(c0)).long(), minlength=need[0])
        return r
    t0, r0 = timed(level0)
    it0 = adaptive_iter_limit(n, lc[0], 0, 100)
    res["phases"]["level0"] = {"s_per_iteration": round(t0, 3), "auction_rounds": r0, "iterations": it0,
                               "projected_s": round(t0 * it0, 1)}

    # middle: the rows' level-0 parents as segments, 128 sub-fits of K=128 in lockstep
    ids0 = ops.nearest(x, ops.prepare_centers(c0))
    r1 = ops.residual(x, c0, ids0, normalize=True)
    order = torch.sort(ids0.long(), stable=True)[1]
    sizes = torch.bincount(ids0.long(), minlength=need[0]).cpu().numpy()
    xo = r1[order].contiguous()
    del r1
    lay = ops.SegmentLayout(sizes, dev)
    starts = np.concatenate([[0], np.cumsum(sizes)[:-1]])
    pick = np.concatenate([s + np.random.default_rng(1).choice(max(int(m), 1), need[1], replace=int(m) < need[1])
                           for s, m in zip(starts, sizes)])
    c1 = xo[torch.from_numpy(pick).to(dev)].clone()

    def middle():
        w = ops.seg_auction_scores(xo, c1, need[1], lay)
        a1, rr = ops.seg_auction(w, need[1], lay)
        ops.centroid_update(xo, lay.seg_of_row * need[1] + a1.long(), need[0] * need[1], c1.clone())
        return int(rr.max().item())
    t1, r1r = timed(middle)
    it1 = max(adaptive_iter_limit(int(m), need[1], 1, 100, is_sub_cluster=True) for m in sizes)
    res["phases"]["middle"] = {"s_per_iteration": round(t1, 3), "auction_rounds_max": r1r, "iterations": it1,
                               "parents": int((sizes > 0).sum()), "projected_s": round(t1 * it1, 1)}
    del xo

    # candidate fits: K=lc[2] (1280 / 2560) with fp16 distances (half: K >= 512), 20 iterations, two fits
    cc = x[torch.randperm(n, device=dev, generator=g)[:lc[2]]].clone()

    def candidates():
        w = ops.auction_scores(x, cc, half=True)
        a2, r = ops.auction(w)
        del w
        ops.centroid_update(x, a2, lc[2], cc.clone())
        return r
    t2, r2 = timed(candidates)
    res["phases"]["candidates"] = {"s_per_iteration": round(t2, 3), "auction_rounds": r2, "iterations": 2 * 20,
                                   "projected_s": round(t2 * 40, 1)}

    # match-matrix groups: (l1, l2) groups of >= 2 need rows fit K=need[2] (iterations of the group size)
    groups = need[0] * need[1]
    gid = torch.randint(0, groups, (n,), device=dev, generator=g)
    gs = torch.bincount(gid, minlength=groups).cpu().numpy()
    big = np.nonzero(gs >= 2 * need[2])[0]
    if len(big):
        keep = torch.isin(gid, torch.from_numpy(big).to(dev))
        rows = torch.nonzero(keep).flatten()
        order = rows[torch.sort(gid[rows], stable=True)[1]]
        del rows, keep
        xg = x[order].contiguous()
        bs = gs[big]
        layg = ops.SegmentLayout(bs, dev)
        bst = np.concatenate([[0], np.cumsum(bs)[:-1]])
        pick = np.concatenate([s + np.random.default_rng(2).choice(int(m), need[2], replace=False)
                               for s, m in zip(bst, bs)])
        cg = xg[torch.from_numpy(pick).to(dev)].clone()

        def grp():
            w = ops.seg_auction_scores(xg, cg, need[2], layg)
            a3, rr = ops.seg_auction(w, need[2], layg)
            ops.centroid_update(xg, layg.seg_of_row * need[2] + a3.long(), len(big) * need[2], cg.clone())
            return int(rr.max().item())
        t3, r3 = timed(grp)
        it3 = max(adaptive_iter_limit(int(m), need[2], 2, base_iter_limit=20) for m in bs)
        res["phases"]["groups"] = {"s_per_iteration": round(t3, 3), "auction_rounds_max": r3, "iterations": it3,
                                   "groups": int(len(big)), "rows": int(bs.sum()), "projected_s": round(t3 * it3, 1),
                                   "note": "uniform random (l1,l2) groups: a trained model's groups are uneven"}
    else:
        res["phases"]["groups"] = {"groups": 0, "projected_s": 0.0,
                                   "note": f"no (l1,l2) group of a uniform random split reaches {2 * need[2]} rows: "
                                           "every group takes its rows / a row sample (no sub-fit)"}
    res["projected_total_s"] = round(sum(p["projected_s"] for p in res["phases"].values()), 1)
    res["method"] = ("one timed iteration per phase after a warm-up, x the reference's iteration schedule; "
                     "encode passes and host bookkeeping excluded")
    print(json.dumps(res), flush=True)
    if a.out:
        Path(a.out).write_text(json.dumps(res) + "\n")


if __name__ == "__main__":
    main()
