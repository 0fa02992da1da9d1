"""Row-sharded K-Means across GPUs: one process per GPU, torch.distributed over RCCL
("nccl" on ROCm) on the xGMI links, rows split in contiguous blocks.

Per Lloyd iteration every rank assigns its own rows (rqsid_assign), accumulates per-cluster fp64 sums
and counts of its rows (rqsid_centroid_accumulate), and ONE all_reduce(SUM) of the fused
``[K*D + K]`` fp64 buffer gives every rank the global update (K=128: 0.5 MB; the 16384-centre level in
lockstep: 64 MB).  Everything that depends on the global state (the shift, the stopping test, the
RNG draws of initialisation and empty clusters) is computed redundantly on every rank from identical
inputs, so all ranks hold bit-identical centres and make identical decisions without further
exchange.  Random rows (initial centres, empty-cluster refills) are drawn with the same global
numpy / torch RNG calls as the single-process reference (balancekmeans/__init__.py:240-256, 321-322)
on every rank, and the rank that owns each drawn row contributes it through one all_reduce.

The local assign and accumulate steps are the GPU kernels; tests substitute the CPU oracle to check
the sharding and collective logic with the ``gloo`` backend on a CPU-only host.
"""
from __future__ import annotations

from typing import Callable, Optional, Tuple

import numpy as np
import torch
import torch.distributed as dist

from . import ops


def shard_bounds(n: int, rank: int, world: int) -> Tuple[int, int]:
    """Contiguous row block of ``rank`` (the first ``n % world`` ranks get one extra row)."""
    base, extra = divmod(n, world)
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


def _gpu_assign(x: torch.Tensor, centers: torch.Tensor) -> torch.Tensor:
    return ops.nearest(x, ops.prepare_centers(centers.float().contiguous())).long()


def _gpu_accumulate(x: torch.Tensor, a: torch.Tensor, k: int):
    sums, counts = ops.centroid_sums(x, a, k)
    return sums, counts.to(torch.float64)


class ShardedLloyd:
    """Unbalanced K-Means (``KMeans.fit`` with balanced=False, balancekmeans/__init__.py:368-465) over
    row shards.  ``x_local`` holds rows [start, stop) of the global matrix of ``n_global`` rows."""

    def __init__(self, n_clusters: int, x_local: torch.Tensor, n_global: int, group=None,
                 assign_fn: Optional[Callable] = None, accumulate_fn: Optional[Callable] = None):
        self.k = n_clusters
        self.x = x_local
        self.n = n_global
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self.start, self.stop = shard_bounds(n_global, self.rank, self.world)
        if x_local.shape[0] != self.stop - self.start:
            raise ValueError(f"rank {self.rank}: expected rows [{self.start}, {self.stop}) of {n_global}")
        self.assign_fn = assign_fn or _gpu_assign
        self.accumulate_fn = accumulate_fn or _gpu_accumulate
        self.cluster_centers = None

    def _rows(self, idx: np.ndarray) -> torch.Tensor:
        """Global rows ``idx`` on every rank: owners fill their rows, one all_reduce(SUM)."""
        buf = torch.zeros((len(idx), self.x.shape[1]), dtype=torch.float64, device=self.x.device)
        own = (idx >= self.start) & (idx < self.stop)
        if own.any():
            pos = torch.from_numpy(np.nonzero(own)[0]).to(self.x.device)
            src = torch.from_numpy(idx[own] - self.start).to(self.x.device)
            buf[pos] = self.x[src].double()
        dist.all_reduce(buf, group=self.group)
        return buf.to(self.x.dtype)

    def initialize(self) -> torch.Tensor:
        replace = self.k > self.n
        return self._rows(np.asarray(np.random.choice(self.n, self.k, replace=replace)))

    def step(self, centers: torch.Tensor):
        a = self.assign_fn(self.x, centers)
        sums, counts = self.accumulate_fn(self.x, a, self.k)
        buf = torch.cat([sums.reshape(-1), counts.reshape(-1).to(sums.dtype)])
        dist.all_reduce(buf, group=self.group)
        d = self.x.shape[1]
        sums, counts = buf[: self.k * d].reshape(self.k, d), buf[self.k * d:]
        new = centers.clone()
        nz = counts > 0
        new[nz] = (sums[nz] / counts[nz].unsqueeze(1)).to(new.dtype)
        empty = torch.nonzero(~nz).flatten().cpu().tolist()
        if empty:
            # the reference's per-cluster loop draws torch.randint(len(X), (1,)) for each empty cluster
            draws = np.asarray([int(torch.randint(self.n, (1,)).item()) for _ in empty])
            new[torch.tensor(empty, device=new.device)] = self._rows(draws)
        return new, a, counts

    def fit(self, tol: float = 1e-3, iter_limit: int = 0):
        centers = self.initialize()
        it = 0
        while True:
            prev = centers
            centers, a, _ = self.step(centers)
            shift = float(torch.sum(torch.sqrt(torch.sum((centers.double() - prev.double()) ** 2, dim=1))).item())
            it += 1
            if shift ** 2 < tol or (iter_limit != 0 and it >= iter_limit):
                break
        self.cluster_centers = centers
        return a
