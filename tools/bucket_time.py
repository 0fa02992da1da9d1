#!/usr/bin/env python3
"""Time rqsid_bucket (ops.bucket) on N uniform keys (default 10M at S = 128 and 16384, the PROD levels; BUCKET_N
and BUCKET_S="256,65536" for the XL ones) with HIP events over 10 calls, and check the result is a counting sort
(keys non-decreasing along row_index, every row once).  RQSID_BUCKET_WIDE sets the rows per block for S > 4096
(A/B)."""
import os, sys, time, torch
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
from generative_ranking_recommender_amd import ops
dev = torch.device("cuda", 0)
g = torch.Generator(device=dev).manual_seed(3)
N = int(os.environ.get("BUCKET_N", 10_000_000))
for S in [int(v) for v in os.environ.get("BUCKET_S", "128,16384").split(",")]:
    keys = torch.randint(0, S, (N,), device=dev, generator=g, dtype=torch.int32)
    ws = ops.bucket_workspace(S, dev)
    for _ in range(3):
        b = ops.bucket(keys, S, workspace=ws)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        b = ops.bucket(keys, S, workspace=ws)
    e1.record(); torch.cuda.synchronize()
    ri = b.row_index.long(); off = b.seg_row_off.long()
    ks = keys.long()[ri]
    ok = bool((ks[1:] >= ks[:-1]).all()) and int(off[-1]) == keys.numel() and torch.equal(torch.sort(ri).values, torch.arange(keys.numel(), device=dev))
    print(f"S={S} wide={os.environ.get('RQSID_BUCKET_WIDE','default')} ms={e0.elapsed_time(e1)/10:.3f} valid={ok}", flush=True)
