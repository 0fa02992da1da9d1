#!/usr/bin/env python3
"""Diagnostics (GPU): cost of 10M scattered 4-byte writes (a permuted ID store, as the segment-ordered
screens do) vs sequential writes vs a permuted gather.  torch kernels only."""
import torch

n = 10_000_000
dev = torch.device("cuda", 0)
perm = torch.randperm(n, device=dev)
seq = torch.arange(n, device=dev)
vals = torch.randint(0, 1 << 20, (n,), dtype=torch.int32, device=dev)
out = torch.empty(n, dtype=torch.int32, device=dev)
blk = (torch.randperm(n // 32, device=dev)[:, None] * 32 + torch.arange(32, device=dev)).reshape(-1)


def timeit(f, reps=10):
    f()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        f()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


print(f"sequential write   {timeit(lambda: out.index_copy_(0, seq, vals)):.3f} ms", flush=True)
print(f"scattered write    {timeit(lambda: out.index_copy_(0, perm, vals)):.3f} ms", flush=True)
print(f"32-run scattered   {timeit(lambda: out.index_copy_(0, blk, vals)):.3f} ms", flush=True)
print(f"permuted gather    {timeit(lambda: torch.index_select(vals, 0, perm, out=out)):.3f} ms", flush=True)
