#!/usr/bin/env python3
"""Level-1 and level-2 screens with the rows bucketed per (row window, segment) instead of per segment:
does limiting the address range a tile's gathered rows span (pages / TLB reach) speed the gathered
levels?  Times rqsid_assign (HIP events) on the bench workload; IDs must equal the standard bucketing."""
import os
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import bench  # noqa: E402
from generative_ranking_recommender_amd import ops  # noqa: E402
from generative_ranking_recommender_amd.encode import HIERARCHICAL_TRAIN, RQEncoder  # noqa: E402


def timed(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


def main(n=int(os.environ.get("SWEEP_ROWS", 10_000_000))):
    dev = torch.device("cuda", 0)
    cb = bench.codebooks(os.environ.get("BENCH_CODEBOOKS", "fitted"), dev)
    enc = RQEncoder([torch.from_numpy(cb[k]) for k in ("c0", "c1", "c2")], [128, 128, 256],
                    match=torch.from_numpy(cb["match"]), semantics=HIERARCHICAL_TRAIN, device=dev)
    x = bench.make_rows(n, 0, dev)
    ids = enc.encode(x).t().contiguous()  # [3, n]
    ws = ops.AssignWorkspace(n, dev)
    rows = torch.arange(n, device=dev, dtype=torch.int64)
    n1 = torch.empty(n, dtype=torch.float32, device=dev)
    # level 1: segment = l0 (128); windowed: W * 128 segments, key = window * 128 + l0
    for W in (1, 2, 4, 8, 16, 32):
        win = (rows * W // n).to(torch.int32)
        key = win * 128 + ids[0]
        b = ops.bucket(key, 128 * W)
        seg = torch.arange(128 * W, device=dev, dtype=torch.int32)
        l0 = seg % 128
        cand = ops.Candidates(l0 * 128, torch.full_like(l0, 128), 128)
        fr = ops.FusedResidual(1, True, enc.pcs[0].centers, l0, den_out=n1)
        out_l = torch.empty(n, dtype=torch.int32, device=dev)
        out_g = torch.empty(n, dtype=torch.int32, device=dev)
        ms = timed(lambda: ops.assign(x, enc.pcs[1], b, cand, out_local=out_l, out_global=out_g, workspace=ws,
                                      fused=fr))
        ok = torch.equal(out_l, ids[1])
        print(f"L1 windows={W:3d} segments={128 * W:5d} tiles={b.max_tiles:7d} {ms:.3f} ms ids_equal={ok}", flush=True)
    # level 2: segment = l0 * 128 + l1 (16384 groups); windowed: W * 16384
    seg_ca, seg_cb = enc._last_segment_rows(dev)
    cand2 = enc.cands[2]
    for W in (1, 2, 4):
        win = (rows * W // n).to(torch.int32)
        g = ids[0] * 128 + ids[1]
        key = win * 16384 + g
        b = ops.bucket(key, 16384 * W)
        gs = torch.arange(16384 * W, device=dev) % 16384
        c2 = ops.Candidates(cand2.base[gs].contiguous(), cand2.count[gs].contiguous(), cand2.count_max, cand2.idx,
                            None if cand2.flags is None else cand2.flags[gs].contiguous(), cand2.lid)
        fr = ops.FusedResidual(2, True, enc.pcs[0].centers, seg_ca[gs].contiguous(), enc.pcs[1].centers,
                               seg_cb[gs].contiguous(), den_in=n1)
        out_l = torch.empty(n, dtype=torch.int32, device=dev)
        out_g = torch.empty(n, dtype=torch.int32, device=dev)
        ms = timed(lambda: ops.assign(x, enc.pcs[2], b, c2, out_local=out_l, out_global=out_g, workspace=ws, fused=fr))
        ok = torch.equal(out_l, ids[2])
        print(f"L2 windows={W:3d} segments={16384 * W:5d} tiles={b.max_tiles:7d} {ms:.3f} ms ids_equal={ok}", flush=True)


if __name__ == "__main__":
    main()
