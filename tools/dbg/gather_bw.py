#!/usr/bin/env python3
"""Diagnostics (GPU): HBM read rate of 2-KiB rows in sequential vs random (segment-sorted) order —
whether the L2 screen's row gather, not its compute, sets its floor.  torch kernels only."""
import torch

n, d = 10_000_000, 512
dev = torch.device("cuda", 0)
x = torch.randn(n, d, device=dev)
seq = torch.arange(n, device=dev)
rnd = torch.randperm(n, device=dev)
blk = (torch.randperm(n // 64, device=dev)[:, None] * 64 + torch.arange(64, device=dev)).reshape(-1)


def timeit(f, reps=5):
    f()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        f()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


out = torch.empty_like(x)
for name, idx in (("sequential", seq), ("random rows", rnd), ("random 64-row runs", blk)):
    ms = timeit(lambda: torch.index_select(x, 0, idx, out=out))
    print(f"{name:20s} {ms:7.3f} ms  {2 * n * d * 4 / ms / 1e9:7.1f} TB/s (read+write)", flush=True)
# read-only: sum of gathered rows by a reduction kernel is not available without a copy; the
# index_select above moves 2x the bytes (read + write), the write stream sequential in all three cases
