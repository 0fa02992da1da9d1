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


class Comm:
    """The collectives of the sharded trainer over one torch.distributed group.  RCCL ("nccl") reduces
    device tensors in place; gloo (the CPU test backend, also used for several ranks sharing one GPU in
    the GPU tests) stages device tensors through host memory.  Variable-size gathers exchange the
    sizes first and pad to the largest share."""

    def __init__(self, group=None):
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self.stage = dist.get_backend(group) == "gloo"

    def _host(self, t: torch.Tensor) -> torch.Tensor:
        """The tensor the backend can take: host memory for gloo, device memory for RCCL."""
        if self.stage:
            return t.cpu() if t.is_cuda else t
        return t if t.is_cuda else t.to(torch.device("cuda", torch.cuda.current_device()))

    def all_reduce(self, t: torch.Tensor, op=dist.ReduceOp.SUM) -> torch.Tensor:
        h = self._host(t.contiguous())
        dist.all_reduce(h, op=op, group=self.group)
        if h is not t:
            t.copy_(h)
        return t

    def _sizes(self, n: int, device: torch.device):
        t = self._host(torch.tensor([n], dtype=torch.int64))
        parts = [torch.zeros_like(t) for _ in range(self.world)]
        dist.all_gather(parts, t, group=self.group)
        return [int(p.item()) for p in parts]

    def all_gather_list(self, t: torch.Tensor):
        """Every rank's tensor (first dimensions may differ), in rank order, on t's device."""
        t = t.contiguous()
        sizes = self._sizes(t.shape[0], t.device)
        width = max(sizes)
        src = self._host(t)
        pad = torch.zeros((width,) + tuple(t.shape[1:]), dtype=t.dtype, device=src.device)
        pad[:t.shape[0]] = src
        parts = [torch.zeros_like(pad) for _ in range(self.world)]
        dist.all_gather(parts, pad, group=self.group)
        return [p[:m].to(t.device) for p, m in zip(parts, sizes)]

    def all_gather_rows(self, t: torch.Tensor) -> torch.Tensor:
        """Concatenation over ranks (rank order) of every rank's rows."""
        return torch.cat(self.all_gather_list(t), 0)

    def all_to_all_rows(self, t: torch.Tensor, send_counts) -> torch.Tensor:
        """Rows t[offsets of send_counts[r]] go to rank r; returns the rows received, in rank order."""
        send_counts = [int(c) for c in send_counts]
        sc = self._host(torch.tensor(send_counts, dtype=torch.int64))
        rc = torch.zeros_like(sc)
        dist.all_to_all_single(rc, sc, group=self.group)
        recv = [int(c) for c in rc.cpu()]
        src = self._host(t.contiguous())
        out = torch.empty((sum(recv),) + tuple(t.shape[1:]), dtype=t.dtype, device=src.device)
        dist.all_to_all_single(out, src, recv, send_counts, group=self.group)
        return out.to(t.device)


def balanced_ranges(sizes, world: int):
    """Contiguous segment ranges [bounds[r], bounds[r+1]) per rank with about equal rows (segments stay
    whole: the sub-fits of one parent / group are independent of the others)."""
    sizes = np.asarray(sizes, dtype=np.int64)
    cum = np.concatenate([[0], np.cumsum(sizes)])
    total = cum[-1]
    bounds = [0]
    for r in range(1, world):
        bounds.append(int(max(bounds[-1], np.searchsorted(cum, total * r / world, side="left"))))
    bounds.append(len(sizes))
    return np.asarray(bounds, dtype=np.int64)


def regroup_rows(comm: "Comm", x_local: torch.Tensor, keys_local: torch.Tensor, bounds, extra=None):
    """Send every local row to the rank owning its segment (keys in [bounds[r], bounds[r+1]) -> rank r);
    returns the received rows in segment order, rows of one segment in ascending global row order (the
    order of torch.where(ids == g) / group_rows in one process), plus any ``extra`` per-row tensors
    regrouped the same way."""
    keys = keys_local.long()
    owner = torch.bucketize(keys, torch.as_tensor(bounds[1:-1], dtype=torch.int64, device=keys.device), right=True)
    order = torch.sort(owner, stable=True)[1]
    counts = torch.bincount(owner, minlength=comm.world).cpu().tolist()
    send = [x_local[order]] + [e[order] for e in (extra or [])] + [keys[order]]
    recv = [comm.all_to_all_rows(t, counts) for t in send]
    k = recv[-1]
    perm = torch.sort(k, stable=True)[1]  # sources arrive in rank order = ascending global row order
    return [r[perm] for r in recv]


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
    """K-Means (``KMeans.fit`` / ``KMeans.fit_by_min_loss``, balancekmeans/__init__.py:259-465) over row
    shards: unbalanced (nearest centre) or, with ``balanced``, the reference's training assignment through
    a row-sharded auction (ShardedAuction).  ``x_local`` holds rows [start, stop) of the global matrix of
    ``n_global`` rows.  Every rank ends every iteration with bit-identical centres and takes the same
    decisions (shift, min-loss bookkeeping, RNG draws) as the single-process fit."""

    def __init__(self, n_clusters: int, x_local: torch.Tensor, n_global: int, group=None,
                 assign_fn: Optional[Callable] = None, accumulate_fn: Optional[Callable] = None,
                 balanced: bool = False, half: bool = False, nearest_fn: Optional[Callable] = None):
        self.k = n_clusters
        self.x = x_local
        self.n = n_global
        self.group = group
        self.comm = Comm(group)
        self.rank, self.world = self.comm.rank, self.comm.world
        self.start, self.stop = shard_bounds(n_global, self.rank, self.world)
        if x_local.shape[0] != self.stop - self.start:
            raise ValueError(f"rank {self.rank}: expected rows [{self.start}, {self.stop}) of {n_global}")
        if assign_fn is None:
            # balanced (KMeans(balanced=True), the reference's training): the row-sharded auction
            assign_fn = (lambda x, c: sharded_balanced_assign(x, c, n_global, half, group)) if balanced else _gpu_assign
        self.assign_fn = assign_fn
        if nearest_fn is None:  # the min-loss histogram's assignment (balancekmeans._loss_assign: fp16 first argmin with half)
            from .balancekmeans import _loss_assign
            nearest_fn = lambda x, c: _loss_assign(x, c.float().contiguous(), half)  # noqa: E731
        self.nearest_fn = nearest_fn
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
        self.comm.all_reduce(buf)
        return buf.to(self.x.dtype)

    def initialize(self) -> torch.Tensor:
        """KMeans.initialize (:240-256): the same np.random.choice draw on every rank."""
        replace = self.k > self.n
        return self._rows(np.asarray(np.random.choice(self.n, self.k, replace=replace))).contiguous()

    def step(self, centers: torch.Tensor):
        a = self.assign_fn(self.x, centers)
        sums, counts = self.accumulate_fn(self.x, a, self.k)
        buf = torch.cat([sums.reshape(-1), counts.reshape(-1).to(sums.dtype)])
        self.comm.all_reduce(buf)
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
        return new.contiguous(), a, counts

    @staticmethod
    def _shift(c: torch.Tensor, prev: torch.Tensor) -> float:
        """KMeans._shift / the reference's center_shift (:343-348), in fp32 like the single-process fit."""
        return float(torch.sum(torch.sqrt(torch.sum((c - prev) ** 2, dim=1))).item())

    def fit(self, tol: float = 1e-3, iter_limit: int = 0):
        """KMeans.fit (:368-465).  Returns this rank's last assignment."""
        centers = self.initialize()
        it = 0
        while True:
            prev = centers
            centers, a, _ = self.step(centers)
            shift = self._shift(centers, prev)
            it += 1
            if shift ** 2 < tol or (iter_limit != 0 and it >= iter_limit):
                break
        self.cluster_centers = centers
        return a

    def fit_by_min_loss(self, target_nodes_num, tol: float = 1e-3, iter_limit: int = 0):
        """KMeans.fit_by_min_loss (:259-365): re-initialised every 10 iterations; after each update the
        global nearest-centre histogram (one all_reduce of K counts) gives the overflow
        loss sum(max(0, count - target)); the centres of the smallest loss (the latest of equal ones) win."""
        centers = self.initialize()
        it = 0
        min_loss, best = float("inf"), None
        while True:
            if it > 0 and it % 10 == 0:
                centers = self.initialize()
            prev = centers
            centers, _, _ = self.step(centers)
            hist = torch.bincount(self.nearest_fn(self.x, centers).long().reshape(-1), minlength=self.k)
            hist = self.comm.all_reduce(hist.to(torch.int64))
            over = hist - target_nodes_num
            cur_loss = float(over[over > 0].sum().item()) if bool((over > 0).any()) else 0
            if cur_loss <= min_loss:
                min_loss, best = cur_loss, centers.clone()
            shift = self._shift(centers, prev)
            it += 1
            if shift ** 2 < tol or (iter_limit != 0 and it >= iter_limit):
                break
        self.cluster_centers = best
        return None


# ----------------------------------------------------------------------------------------------------
# Row-sharded balanced assignment (SURVEY.md §8e "auction rebalance": one exchange per round)
# ----------------------------------------------------------------------------------------------------
class GpuAuctionPasses:
    """The passes of one rank's share of an auction_lap_half (include/rqsid.h rqsid_dauction_*) on its
    worker-major fp16 scores [K][n_local]; the buffers the driver reduces are views into the workspace."""

    def __init__(self, scores_wj: torch.Tensor, n_global: int):
        import ctypes
        self.w = scores_wj.to(torch.float16).contiguous()
        ops._require_device(self.w)
        self.k, self.n_local = self.w.shape
        self.n_global = int(n_global)
        lib = ops.lib()
        self.lib = lib
        self.wsb = int(lib.rqsid_dauction_workspace_bytes(self.n_local, self.k))
        self.ws = torch.zeros(self.wsb, dtype=torch.uint8, device=self.w.device)
        offs = (ctypes.c_int64 * 6)()
        ops._lib.check(lib.rqsid_dauction_layout(self.n_local, self.k, offs), "rqsid_dauction_layout")
        k = self.k
        self._mm = self.ws[offs[0]:offs[0] + 8].view(torch.int32)
        # the K x 256 radix histograms and, after them, the count of ranks whose bid list overflowed (the
        # row-sharded list rounds, auction_seg.hip da_*): one buffer, one all_reduce
        self._hist = self.ws[offs[1]:offs[1] + (k * 256 + 1) * 4].view(torch.int32)
        self._eqtot = self.ws[offs[2]:offs[2] + k * 4].view(torch.int32)
        self._have = self.ws[offs[3]:offs[3] + 4].view(torch.int32)
        self._flag = self.ws[offs[4]:offs[4] + 1]
        self._rounds = self.ws[offs[5]:offs[5] + 4].view(torch.int32)
        self.out = torch.full((max(self.n_local, 1),), -1, dtype=torch.int32, device=self.w.device)
        self._mode = self.ws[192:196].view(torch.int32)  # the coming slot's mode (include/rqsid.h)
        self.list_only = False  # set by the driver per slot: launch the list kernels alone

    def _args(self):
        return (ops._ptr(self.w) if self.n_local else None, self.k, self.n_local, self.n_global)

    def _tail(self):
        return (ops._ptr(self.ws), self.wsb, ops._stream())

    def begin(self) -> torch.Tensor:
        ops._lib.check(self.lib.rqsid_dauction_begin(*self._args(), ops._ptr(self.out), *self._tail()),
                       "rqsid_dauction_begin")
        return self._mm.to(torch.int64) & 0xFFFFFFFF  # {max key, min key} of this rank's scores

    def set_minmax(self, mx: int, mn: int) -> None:
        self._mm.copy_(torch.tensor([mx, mn], dtype=torch.int64).to(torch.int32))
        ops._lib.check(self.lib.rqsid_dauction_eps(*self._args(), *self._tail()), "rqsid_dauction_eps")

    def _list_pass(self, step: int, rank_off=None) -> None:
        ops._lib.check(self.lib.rqsid_dauction_list_pass(*self._args(), int(step), ops._ptr(rank_off), *self._tail()),
                       "rqsid_dauction_list_pass")

    def hist(self, low: int) -> torch.Tensor:
        if self.list_only:
            if not low:
                self._list_pass(-1)
            self._list_pass(int(low))
            return self._hist
        ops._lib.check(self.lib.rqsid_dauction_hist(*self._args(), int(low), *self._tail()), "rqsid_dauction_hist")
        return self._hist

    def select(self, low: int) -> None:
        ops._lib.check(self.lib.rqsid_dauction_select(*self._args(), int(low), *self._tail()),
                       "rqsid_dauction_select")

    def eqcount(self) -> torch.Tensor:
        if self.list_only:
            self._list_pass(2)
            return self._eqtot
        ops._lib.check(self.lib.rqsid_dauction_eqcount(*self._args(), *self._tail()), "rqsid_dauction_eqcount")
        return self._eqtot

    def bid(self, rank_off: torch.Tensor) -> None:
        ro = rank_off.to(torch.int32).to(self.w.device).contiguous()
        if self.list_only:
            self._list_pass(3, ro)
            return
        ops._lib.check(self.lib.rqsid_dauction_bid(*self._args(), ops._ptr(ro), *self._tail()), "rqsid_dauction_bid")

    def resolve(self) -> torch.Tensor:
        ops._lib.check(self.lib.rqsid_dauction_resolve(*self._args(), ops._ptr(self.out), *self._tail()),
                       "rqsid_dauction_resolve")
        return self._have

    def end_round(self) -> None:
        ops._lib.check(self.lib.rqsid_dauction_end_round(*self._args(), *self._tail()), "rqsid_dauction_end_round")

    def live(self) -> bool:
        """Still bidding (host sync): end_round clears it once the reduced `have` covers every job."""
        return bool(int(self._flag.item()) & 1)

    def debug(self) -> list:
        """{mode, round, longest list, mean list, lkb[0], T[0], overflow word, lists over capacity} (host sync)"""
        out = torch.zeros(8, dtype=torch.int32, device=self.w.device)
        ops._lib.check(self.lib.rqsid_dauction_debug(*self._args(), ops._ptr(out), *self._tail()), "rqsid_dauction_debug")
        return out.cpu().tolist()

    def lists_hold(self) -> bool:
        """The coming slot runs from the bid lists (host sync; the same on every rank: it is decided from
        reduced data only)."""
        return int(self._mode.item()) == 1

    def rounds_run(self) -> int:
        return int(self._rounds.item())

    def result(self) -> torch.Tensor:
        return self.out[:self.n_local]


_STATS = __import__("os").environ.get("RQSID_DAUCTION_STATS", "0") not in ("", "0")


class ShardedAuction:
    """auction_lap_half (balancekmeans/__init__.py:12-140) over jobs split in contiguous blocks across the
    ranks of ``group`` (rank r's block follows rank r-1's).  Per round: the two radix histograms of every
    worker's values are summed over the ranks (2 x all_reduce of K*256 int32), the counts of values equal
    to each worker's threshold are all-gathered (each rank's tie ranks start after the lower ranks'), and
    the count of jobs with a bidder is summed (all_reduce of one int32).  Every rank ends each round with
    identical thresholds and the same stop decision, and the assignment equals the single-process auction
    of the whole matrix (same fp16 operations, same tie rule).  The stop decision is taken on the device
    (end_round clears the live flag; later passes are no-ops), so the host reads it once per ``poll``
    rounds instead of synchronising every round.  From round 32 (16 at K >= 1024) the GPU passes run
    rounds from per-rank bid lists (auction_seg.hip da_*, same collectives); at each poll the host also
    reads whether the lists hold and then launches list-only slots (rqsid_dauction_list_pass)."""

    poll = 8

    def __init__(self, group=None):
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        # gloo (the CPU test backend) stages device tensors through host memory; RCCL reduces in place
        self.stage = dist.get_backend(group) == "gloo"

    def _all_reduce(self, t: torch.Tensor, op=dist.ReduceOp.SUM) -> None:
        if self.stage and t.is_cuda:
            h = t.cpu()
            dist.all_reduce(h, op=op, group=self.group)
            t.copy_(h)
        else:
            dist.all_reduce(t, op=op, group=self.group)

    def _all_gather(self, t: torch.Tensor):
        src = t.cpu() if self.stage and t.is_cuda else t.contiguous()
        parts = [torch.zeros_like(src) for _ in range(self.world)]
        dist.all_gather(parts, src, group=self.group)
        return [p.to(t.device) for p in parts]

    # environment switches librqsid reads on each rank for the row-sharded list rounds (auction_seg.hip
    # seg_carve / rqsid_dauction_begin): they decide lkb, the list start and whether lists run at all, so
    # ranks that disagree would split between list and sweep slots inside the same collectives
    _SETTINGS = ("RQSID_DAUCTION_LIST", "RQSID_LIST_DELTA", "RQSID_LIST_START")

    def _check_uniform_settings(self) -> None:
        """Raise unless every rank of the group runs with the same list settings (two tiny all_reduces)."""
        import os
        vals = []
        for name in self._SETTINGS:
            v = os.environ.get(name)
            try:
                vals.append(-1 if v is None else int(v))
            except ValueError:
                vals.append(-2)
        dev = torch.device("cpu") if self.stage else torch.device("cuda", torch.cuda.current_device())
        lo = torch.tensor(vals, dtype=torch.int64, device=dev)
        hi = lo.clone()
        dist.all_reduce(lo, op=dist.ReduceOp.MIN, group=self.group)
        dist.all_reduce(hi, op=dist.ReduceOp.MAX, group=self.group)
        if not torch.equal(lo, hi):
            raise RuntimeError(f"sharded auction: ranks disagree on {dict(zip(self._SETTINGS, vals))} "
                               f"(min {lo.tolist()}, max {hi.tolist()}); set them alike on every rank")

    def run(self, passes, n_global: int, k: int, max_rounds: int = 0):
        """Returns (this rank's assignment, rounds run)."""
        if n_global == 0:
            return passes.result(), 0
        if self.world > 1:
            self._check_uniform_settings()
        if k == 1:
            raise ValueError("auction: a single worker cannot bid on N + 1 jobs")
        mm = passes.begin()
        if n_global < k:  # the reference's argmin(-D) fallback, per job (begin wrote it)
            return passes.result(), 0
        mx, mn = mm[0:1].clone(), mm[1:2].clone()
        self._all_reduce(mx, dist.ReduceOp.MAX)
        self._all_reduce(mn, dist.ReduceOp.MIN)
        passes.set_minmax(int(mx.item()), int(mn.item()))
        issued = 0
        lists = getattr(passes, "lists_hold", None)
        while True:
            for low in (0, 1):
                h = passes.hist(low)
                self._all_reduce(h)
                passes.select(low)
            e = passes.eqcount()
            parts = self._all_gather(e)
            rank_off = torch.zeros_like(e)
            for r in range(self.rank):
                rank_off += parts[r]
            passes.bid(rank_off)
            have = passes.resolve()
            self._all_reduce(have)
            passes.end_round()  # the device compares the reduced count with n_global
            issued += 1
            if issued % self.poll and not (max_rounds and issued >= max_rounds):
                continue
            if not passes.live():
                return passes.result(), passes.rounds_run()
            # the cap counts real rounds: a void list slot (rounds from lists that did not hold) advances no
            # round, so the number of slots issued may exceed the rounds run
            if max_rounds and passes.rounds_run() >= max_rounds:
                raise RuntimeError(f"auction: no complete assignment after {max_rounds} rounds")
            if _STATS and hasattr(passes, "debug"):
                print("dauction slot", issued, passes.debug(), flush=True)
            if lists is not None:
                # the next slots launch the list kernels alone while the lists hold (a slot that meets a sweep
                # round is void and the poll after it returns to full slots); every rank reads the same mode
                passes.list_only = lists()


def _force_sharded() -> bool:
    """RQSID_SHARDED_AUCTION=1: a world-1 group runs the row-sharded protocol too (ShardedAuction over the
    group's collectives) instead of the single-process auction, so one rank measures what each rank of a
    larger world runs (tools/train_bench.py --sharded)."""
    import os
    return os.environ.get("RQSID_SHARDED_AUCTION", "0") not in ("", "0")


def sharded_balanced_assign(x_local: torch.Tensor, centers: torch.Tensor, n_global: int, half: bool = False,
                            group=None) -> torch.Tensor:
    """auction_lap_half(-pairwise_distance(X, C)) with X row-sharded: each rank scores its rows against all
    centres (rqsid_auction_scores) and the ranks run one ShardedAuction.  Returns this rank's worker ids."""
    w = ops.auction_scores(x_local.contiguous(), centers.float().contiguous(), half=half)
    if dist.get_world_size(group) == 1 and not _force_sharded():
        # one rank holds every job: the single-process auction of the same scores (identical assignment,
        # see ShardedAuction), which also runs the bid-list rounds the per-round collectives cannot
        a, _ = ops.auction(w)
        return a.long()
    a, _ = ShardedAuction(group).run(GpuAuctionPasses(w, n_global), n_global, centers.shape[0])
    return a.long()
