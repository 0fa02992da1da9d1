"""Balanced K-Means on MI355X — the module API of the reference's ``balancekmeans`` package
(src/semantic_id_generator/balancekmeans/__init__.py), with every arithmetic step on the HIP
kernels of ``librqsid.so``:

* distances + argmin  -> ``rqsid_assign`` (exact argmin; the reference's fp32 ``torch.cdist``
  + ``torch.argmin``, :489-534, 576-603); ``distance='cosine'`` -> ``rqsid_pairwise_cosine`` (:625-655)
* balanced assignment -> ``rqsid_auction_scores`` + ``rqsid_auction_lap_half`` (:12-140)
* centroid update     -> ``rqsid_centroid_accumulate/finalize`` (fp64 sums, :315-324)

Host-side orchestration (RNG draws, loop control, the loss bookkeeping of ``fit_by_min_loss``)
follows the reference statement by statement so that seeded runs draw the same numpy / torch
random numbers in the same order: ``np.random.choice`` for initial centres (:240-256) and the
CPU ``torch.randint`` for empty clusters (:321-322).  There is no CPU compute path: tensors are
moved to the GPU and the kernels raise if ``librqsid.so`` or the GPU is missing.
"""
from __future__ import annotations

import itertools
import logging
from typing import Optional

import numpy as np
import torch

from . import ops

logger = logging.getLogger(__name__)

# Step tracer for every K-Means fit of this module (tests certify each iteration against the oracle):
# None, or a callable taking one dict per iteration.  KMeans.fit / fit_by_min_loss send
# {"kind": "fit", "owner" (one number per KMeans object), "x", "half", "iteration", "centers_in", "scores"
# ([K][N] fp16 or None), "assign", "centers_out", "loss"/"target" (fit_by_min_loss: the overflow loss of
# centers_out, else None)}; batched_fit sends {"kind": "batched", "owner" (one number per fit_segments
# call), "seg_base" (global index of the window's first segment), "window" (attempt number), "x"
# (segment-ordered rows), "half", "iteration", "active" (bool [S]), "off" (segment row offsets),
# "centers_in", "scores" (flat per-segment [K][N_s] blocks or None), "assign" (local ids), "centers_out",
# "loss" (per segment, min-loss mode) / "target"}.
TRACE = None
_TRACE_OWNERS = itertools.count()


def _device(device) -> torch.device:
    if device is None or (isinstance(device, torch.device) and device.type == "cpu") or device == "cpu":
        # the reference defaults to CPU; this framework has no CPU compute path
        return torch.device("cuda", torch.cuda.current_device() if torch.cuda.is_available() else 0)
    return torch.device(device)


def _to_dev(x: torch.Tensor, device: torch.device) -> torch.Tensor:
    if not isinstance(x, torch.Tensor):
        x = torch.as_tensor(np.asarray(x))
    return x.float().to(device).contiguous()


def pairwise_distance_full(data1, data2, device=None, batch_size: int = 10000) -> torch.Tensor:
    """balancekmeans/__init__.py:576-603: fp32 [N, K] Euclidean distances (``batch_size`` is
    accepted for signature compatibility; the kernel streams rows itself)."""
    dev = _device(device)
    return ops.pairwise_distance(_to_dev(data1, dev), _to_dev(data2, dev))


def pairwise_distance_half(data1, data2, device=None, batch_size: int = 20000) -> torch.Tensor:
    """balancekmeans/__init__.py:536-574: fp16 [N, K] distances of the fp16-rounded operands,
    clamped at 1e-5."""
    dev = _device(device)
    return (-ops.auction_scores(_to_dev(data1, dev), _to_dev(data2, dev), half=True)).t().contiguous()


def pairwise_cosine(data1, data2, device=None, batch_size: int = 1000) -> torch.Tensor:
    """balancekmeans/__init__.py:625-655: fp32 [N, K] cosine distances 1 - x.c / (|x||c|)
    (``rqsid_pairwise_cosine``; ``batch_size`` is accepted for signature compatibility)."""
    dev = _device(device)
    return ops.pairwise_cosine(_to_dev(data1, dev), _to_dev(data2, dev))


def auction_lap_half(job_and_worker_to_score: torch.Tensor, return_token_to_worker: bool = True) -> torch.Tensor:
    """balancekmeans/__init__.py:12-140 on the GPU.  ``job_and_worker_to_score`` is N x K (= -distance).
    Returns the worker of every job (int64, on the input's device)."""
    s = job_and_worker_to_score
    if not return_token_to_worker:
        raise NotImplementedError("return_token_to_worker=False is unused by the reference's callers")
    dev = s.device if s.device.type == "cuda" else _device(None)
    n, k = s.shape
    if torch.isnan(s).any():
        raise Exception("NaN distance")  # :36-38
    w = s.to(dev).half().t().contiguous()
    a, rounds = ops.auction(w)
    logger.debug("auction_lap_half: %d jobs, %d workers, %d rounds", n, k, rounds)
    return a.long()


def auction_lap_full(job_and_worker_to_score: torch.Tensor, return_token_to_worker: bool = True):
    """balancekmeans/__init__.py:142-210: the fp32 auction (``rqsid_auction_lap_full``), reached through
    ``KMeans.predict(balanced=True)`` (:523-525).  Returns the worker of every job (int64, on the scores'
    device), like the reference with return_token_to_worker=True."""
    s = job_and_worker_to_score
    if not return_token_to_worker:
        raise NotImplementedError("return_token_to_worker=False is unused by the reference's callers")
    dev = s.device if s.device.type == "cuda" else _device(None)
    if torch.isnan(s).any():
        raise Exception("NaN distance")  # :152-154
    w = s.to(dev).float().t().contiguous()
    a, rounds = ops.auction_full(w)
    logger.debug("auction_lap_full: %d jobs, %d workers, %d rounds", s.shape[0], s.shape[1], rounds)
    return a.long()


class KMeans:
    """balancekmeans.KMeans (:223-534): same constructor, ``fit``, ``fit_by_min_loss``, ``predict``."""

    def __init__(self, n_clusters=None, cluster_centers=None, device=torch.device("cpu"), balanced=False):
        self.n_clusters = n_clusters
        self.cluster_centers = cluster_centers
        self.device = _device(device)
        self.balanced = balanced
        self.last_auction_rounds = []
        self.trace = TRACE  # per-iteration step tracer (see TRACE)
        self._owner = next(_TRACE_OWNERS)

    # --- persistence (npz instead of the reference's pickle, :230-239) --------------------------
    @classmethod
    def load(cls, path_to_file):
        with np.load(path_to_file, allow_pickle=False) as z:
            return cls(int(z["n_clusters"]), torch.from_numpy(z["cluster_centers"]), torch.device("cpu"),
                       bool(z["balanced"]))

    def save(self, path_to_file):
        c = self.cluster_centers
        np.savez(path_to_file, n_clusters=self.n_clusters, balanced=self.balanced,
                 cluster_centers=c.detach().cpu().numpy() if isinstance(c, torch.Tensor) else np.asarray(c))

    # --- reference steps -------------------------------------------------------------------------
    def initialize(self, X: torch.Tensor) -> torch.Tensor:
        """:240-256 — np.random.choice over rows (with replacement only when K > N)."""
        num_samples = len(X)
        if self.n_clusters > num_samples:
            indices = np.random.choice(num_samples, self.n_clusters, replace=True)
        else:
            indices = np.random.choice(num_samples, self.n_clusters, replace=False)
        return X[torch.from_numpy(np.asarray(indices)).to(X.device)].clone()

    def _check_distance(self, distance):
        """'euclidean' (the semantic-ID path) and 'cosine' (:279-280, 625-655); 'soft_dtw' needs the
        reference's numba-CUDA SoftDTW and stays out of scope."""
        if distance not in ("euclidean", "cosine"):
            raise NotImplementedError(f"distance={distance!r}: 'euclidean' and 'cosine' are supported")
        self._distance = distance

    def _assign(self, X: torch.Tensor, half: bool) -> torch.Tensor:
        self._scores, self._x, self._half = None, X, half
        if getattr(self, "_distance", "euclidean") == "cosine":
            # pairwise_cosine for the assignment whatever `half` says (:279-280); argmin = first index
            if self.balanced:
                a, rounds = ops.auction(ops.pairwise_cosine(X, self.cluster_centers, scores=True))
                self.last_auction_rounds.append(rounds)
                return a
            return torch.argmin(ops.pairwise_cosine(X, self.cluster_centers), dim=1)
        if self.balanced:
            w = ops.auction_scores(X, self.cluster_centers, half=half)
            a, rounds = ops.auction(w)
            self.last_auction_rounds.append(rounds)
            if self.trace is not None:
                self._scores = w
            return a
        return ops.nearest(X, ops.prepare_centers(self.cluster_centers))

    def _emit(self, iteration: int, prev: torch.Tensor, a: torch.Tensor, loss=None, target=None) -> None:
        if self.trace is not None and getattr(self, "_distance", "euclidean") == "euclidean":
            self.trace({"kind": "fit", "owner": self._owner, "x": self._x, "half": self._half,
                        "iteration": iteration, "centers_in": prev.clone(), "scores": self._scores,
                        "assign": a.clone(), "centers_out": self.cluster_centers.clone(), "loss": loss,
                        "target": target})

    def _update(self, X: torch.Tensor, a: torch.Tensor) -> torch.Tensor:
        """:314-324 — per-cluster means; an empty cluster takes X[torch.randint(len(X), (1,))] (CPU RNG,
        drawn in cluster order exactly as the reference's loop does)."""
        prev = self.cluster_centers.clone()
        centers, counts = ops.centroid_update(X, a, self.n_clusters, self.cluster_centers)
        empty = torch.nonzero(counts == 0).flatten().cpu().tolist()
        for index in empty:
            centers[index] = X[torch.randint(len(X), (1,))].reshape(-1)
        self.cluster_centers = centers
        return prev

    @staticmethod
    def _shift(c: torch.Tensor, prev: torch.Tensor) -> float:
        return float(torch.sum(torch.sqrt(torch.sum((c - prev) ** 2, dim=1))).item())

    def fit_by_min_loss(self, X, target_nodes_num, distance="euclidean", tol=1e-3, tqdm_flag=True, iter_limit=0,
                        gamma_for_soft_dtw=0.001, half=False, online=False, iter_k=None):
        """:259-365 — Lloyd / auction iterations, re-initialised every 10 iterations, keeping the centres
        of the smallest overflow loss sum(max(0, count - target)) (``<=``: the latest of equal losses)."""
        self._check_distance(distance)
        X = _to_dev(X, self.device)
        if not online or (online and iter_k == 0):
            self.cluster_centers = self.initialize(X)
        self.cluster_centers = self.cluster_centers.float().to(self.device).contiguous()
        iteration = 0
        min_loss, best = float("inf"), None
        while True:
            if iteration > 0 and iteration % 10 == 0:
                self.cluster_centers = self.initialize(X)
            a = self._assign(X, half)
            prev = self._update(X, a)
            if distance == "cosine":
                near = torch.argmin(ops.pairwise_cosine(X, self.cluster_centers), dim=1)
            else:
                near = _loss_assign(X, self.cluster_centers, half)
            counts = torch.bincount(near, minlength=self.n_clusters)
            over = counts - target_nodes_num
            cur_loss = float(over[over > 0].sum().item()) if (over > 0).any() else 0
            self._emit(iteration, prev, a, cur_loss, target_nodes_num)
            logger.debug("fit_by_min_loss: iteration %d loss %s", iteration, cur_loss)
            if cur_loss <= min_loss:
                min_loss = cur_loss
                best = self.cluster_centers.clone()
            center_shift = self._shift(self.cluster_centers, prev)
            iteration += 1
            if center_shift ** 2 < tol:
                break
            if iter_limit != 0 and iteration >= iter_limit:
                break
        self.cluster_centers = best
        return None

    def fit(self, X, distance="euclidean", tol=1e-3, tqdm_flag=True, iter_limit=0, gamma_for_soft_dtw=0.001,
            half=False, online=False, iter_k=None):
        """:368-465 — returns the last assignment (int64, CPU) like the reference."""
        self._check_distance(distance)
        X = _to_dev(X, self.device)
        if not online or (online and iter_k == 0):
            self.cluster_centers = self.initialize(X)
        self.cluster_centers = self.cluster_centers.float().to(self.device).contiguous()
        iteration = 0
        while True:
            a = self._assign(X, half)
            prev = self._update(X, a)
            self._emit(iteration, prev, a)
            center_shift = self._shift(self.cluster_centers, prev)
            iteration += 1
            if center_shift ** 2 < tol:
                break
            if iter_limit != 0 and iteration >= iter_limit:
                break
        return a.long().cpu()

    def predict(self, X, distance="euclidean", gamma_for_soft_dtw=0.001, tqdm_flag=False, return_distances=False,
                balanced=False):
        """:489-534 — nearest centre (exact argmin, lowest index on ties); with balanced=True the fp32
        auction on -distance (:523-525).  int64 on the CPU."""
        self._check_distance(distance)
        X = _to_dev(X, self.device)
        if X.dim() == 1:
            X = X.unsqueeze(0)
        c = self.cluster_centers.float().to(self.device).contiguous()
        if distance == "cosine":
            d = ops.pairwise_cosine(X, c)
            ids = (auction_lap_full(-d) if balanced else torch.argmin(d, dim=1)).long().cpu()
            return (ids, d) if return_distances else ids
        if balanced:
            d = ops.pairwise_distance(X, c)
            ids = auction_lap_full(-d).cpu()
            return (ids, d) if return_distances else ids
        ids = ops.nearest(X, ops.prepare_centers(c)).long().cpu()
        if return_distances:
            return ids, ops.pairwise_distance(X, c)
        return ids


def _loss_assign(X: torch.Tensor, centers: torch.Tensor, half: bool) -> torch.Tensor:
    """The nearest-centre assignment behind fit_by_min_loss's overflow loss (:327-329): the argmin of
    ``pairwise_distance_function(X, C)``, i.e. of the fp32 distances (exact argmin here; the reference's
    fp32 cdist can only differ on a near tie), or with ``half`` of the fp16 distances of
    pairwise_distance_half, whose many EQUAL values make the first index matter: the fp16 scores
    (rqsid_auction_scores, -distance) and their first maximum per row."""
    if not half:
        return ops.nearest(X, ops.prepare_centers(centers)).long()
    w = ops.auction_scores(X, centers, half=True)  # [K][N] fp16 = -distance
    return torch.argmax(w, dim=0)  # first index among equal values


def init_indices(num_samples: int, n_clusters: int) -> np.ndarray:
    """The draw of KMeans.initialize (:240-256): np.random.choice over rows, with replacement only when
    K > N (global numpy RNG)."""
    if n_clusters > num_samples:
        return np.asarray(np.random.choice(num_samples, n_clusters, replace=True))
    return np.asarray(np.random.choice(num_samples, n_clusters, replace=False))


def batched_fit(X: torch.Tensor, layout: "ops.SegmentLayout", n_clusters: int, iter_limits, inits,
                target_nodes_num=None, tol: float = 1e-3, half: bool = False, balanced: bool = True,
                return_info: bool = False, trace_tag: Optional[dict] = None):
    """Many independent K-Means fits advanced in lockstep, one per segment of the segment-ordered rows X
    (segment s = rows layout.off[s] .. layout.off[s+1]), each exactly the iteration of KMeans.fit
    (:368-465; ``target_nodes_num`` None) or KMeans.fit_by_min_loss (:259-365; re-initialised every 10
    iterations, keeping the centres of the smallest overflow loss, the latest of equal losses).

    The reference runs these fits one after another (hierarchical_rq_kmeans.py:703-725, 1010-1019); here
    every iteration of every live segment is one segmented score kernel, one segmented auction
    (rqsid_seg_auction_lap_half, all rounds of all segments in lockstep) and one centroid update over
    S*K clusters.  A segment stops at its own iteration limit or tolerance and is skipped afterwards.

    ``inits[s]`` holds segment s's initialisation draws (row indices local to the segment): inits[s][0]
    for the start and inits[s][i] for the re-initialisation at iteration 10*i.  The caller draws them
    from the global numpy RNG in segment order, so a segment that runs its full iteration budget consumes
    exactly the reference's draws.  Empty clusters take a random row of their segment from the global
    torch RNG, drawn in (iteration, segment, cluster) order.

    Returns (centres f32 [S*K, D], last assignment i32 [N] local to each segment); with ``return_info``
    also {"iterations": i64[S] iterations run per segment, "events": [(segment, iteration), ...] the
    empty-cluster torch draws in the order they were made}.  ``fit_segments`` uses both to prove (or
    restore) the reference's sequential RNG consumption."""
    dev = X.device
    S, K = layout.n_seg, n_clusters
    off = layout.off
    if X.shape[0] != layout.n:
        raise ValueError("batched_fit: rows do not match the segment layout")
    limits = np.asarray(iter_limits, dtype=np.int64).reshape(S)
    min_loss_mode = target_nodes_num is not None

    def gather(draws, segs):
        idx = np.concatenate([off[s] + np.asarray(draws[i], dtype=np.int64) for i, s in enumerate(segs)])
        return X[torch.from_numpy(idx).to(dev)]

    centers = gather([inits[s][0] for s in range(S)], range(S)).float().contiguous()
    active = layout.sizes > 0
    iteration = np.zeros(S, dtype=np.int64)
    min_loss = np.full(S, np.inf)
    best = centers.clone()
    last = torch.full((max(layout.n, 1),), -1, dtype=torch.int32, device=dev)
    seg_row = layout.seg_of_row
    buckets = cand = None
    if min_loss_mode or not balanced:
        buckets = ops.bucket(seg_row, S)
        cand = ops.contiguous_candidates(S, K, dev)
    rows_of = torch.arange(S * K, device=dev).view(S, K)
    events = []
    while active.any():
        if min_loss_mode:
            re = np.nonzero(active & (iteration > 0) & (iteration % 10 == 0))[0]
            if len(re):
                centers[rows_of[torch.from_numpy(re).to(dev)].reshape(-1)] = gather(
                    [inits[s][iteration[s] // 10] for s in re], re).float()
        act_t = torch.from_numpy(active.astype(np.uint8)).to(dev)
        w = None
        if balanced:
            w = ops.seg_auction_scores(X, centers, K, layout, half=half)
            a, _ = ops.seg_auction(w, K, layout, act_t, out=last)
        else:
            a = ops.assign(X, ops.prepare_centers(centers), buckets, cand)[0]
            keep = ~act_t.bool()[seg_row]
            a = torch.where(keep, last[:layout.n], a)
        last[:layout.n] = a
        prev = centers
        gid = seg_row * K + a.long()
        new, counts = ops.centroid_update(X, gid, S * K, centers.clone())
        cnt = counts.cpu().numpy().reshape(S, K)
        for s in np.nonzero(active)[0]:
            for k in np.nonzero(cnt[s] == 0)[0]:
                new[s * K + k] = X[int(off[s]) + int(torch.randint(int(layout.sizes[s]), (1,)).item())]
                events.append((int(s), int(iteration[s])))
        frozen = torch.from_numpy(~active).to(dev)
        new[frozen.repeat_interleave(K)] = prev[frozen.repeat_interleave(K)]
        centers = new.contiguous()
        if TRACE is None:
            w = None  # the auction's score matrix is dead unless traced: free it before the loss scores
        loss = None
        if min_loss_mode:
            if half:  # argmin of the fp16 distances, first index (:327-329 with pairwise_distance_half)
                ws = ops.seg_auction_scores(X, centers, K, layout, half=True)
                loc = torch.cat([ws[K * int(off[s]):K * int(off[s + 1])].view(K, -1).argmax(0)
                                 for s in range(S)]) if layout.n else torch.zeros(0, dtype=torch.int64, device=dev)
                glob = seg_row.long() * K + loc
                del ws
            else:
                glob = ops.assign(X, ops.prepare_centers(centers), buckets, cand)[1].long()
            hist = torch.bincount(glob, minlength=S * K).view(S, K)
            loss = (hist - target_nodes_num).clamp(min=0).sum(1).cpu().numpy()
        if TRACE is not None:
            TRACE({"kind": "batched", "x": X, "half": half, "iteration": iteration.copy(), "active": active.copy(),
                   "off": off.copy(), "centers_in": prev.clone(), "scores": w, "assign": a.clone(),
                   "centers_out": centers.clone(), "loss": None if loss is None else loss.copy(),
                   "target": target_nodes_num, **(trace_tag or {"owner": -1, "seg_base": 0, "window": 0})})
        del w
        shift = torch.sqrt(torch.sum((centers - prev) ** 2, dim=1)).view(S, K).sum(1).cpu().numpy()
        if min_loss_mode:
            better = active & (loss <= min_loss)
            if better.any():
                min_loss[better] = loss[better]
                sel = rows_of[torch.from_numpy(np.nonzero(better)[0]).to(dev)].reshape(-1)
                best[sel] = centers[sel]
        iteration[active] += 1
        done = active & ((shift.astype(np.float64) ** 2 < tol) | ((limits != 0) & (iteration >= limits)))
        active &= ~done
    out = (best if min_loss_mode else centers), last[:layout.n]
    if return_info:
        return out + ({"iterations": iteration.copy(), "events": events},)
    return out


def reinit_draws(iter_limit: int) -> int:
    """Initialisation draws of a fit_by_min_loss run of ``iter_limit`` iterations: its start plus one
    re-initialisation at every iteration 10, 20, ... it reaches (balancekmeans/__init__.py:295, 305-306)."""
    return 1 + max(0, (int(iter_limit) - 1) // 10)


def fit_segments(X: torch.Tensor, sizes, n_clusters: int, iter_limits, inits=None, target_nodes_num=None,
                 tol: float = 1e-3, half: bool = False, max_restarts: int = 3, comm=None, owned=None):
    """The reference's one-after-another sub-fits (hierarchical_rq_kmeans.py:703-731, 1010-1019;
    simplified_semantic_id_generator.py:119-133, 275-278) run in lockstep by ``batched_fit``, with the
    reference's random-number consumption restored exactly.

    X holds the segments' rows in segment order (segment s = the next sizes[s] rows).  Two schedules
    of the reference cannot be known before a fit has run:
    * numpy: ``fit_by_min_loss`` draws a re-initialisation at iteration 10, 20, ... only while it has
      not converged.  With ``target_nodes_num`` set, every segment's start and every re-initialisation
      its budget allows are drawn here, speculatively, in segment order.
    * torch: an empty cluster draws ``torch.randint(len(X), (1,))`` (:321-322); the lockstep loop draws
      in (iteration, segment) order, the reference in (segment, iteration) order.
    After each lockstep run the first segment whose draws differ from the reference's is found (one that
    converged early with unused re-initialisations: the segments after it; a torch draw taken out of the
    reference's order: that segment).  Segments before it are exact and kept; the generators are put in
    the reference's state at that point (numpy: re-drawn from the saved state; torch: the exact draws
    replayed) and the remaining segments run again.  After ``max_restarts`` such restarts the rest runs
    one segment at a time, which is exact by construction.  Without ``target_nodes_num`` (``fit``) the
    caller draws the starts (``inits[s] = [indices]``) in its own order, interleaved with its other draws.

    Segment-parallel (``comm`` = distributed.Comm): every rank passes the same sizes,
    limits and inits and X = the rows of ITS segments ``owned = (s0, s1)`` (contiguous ranges in rank
    order).  Each rank fits its own segments; the centres, iteration counts and empty-cluster events are
    all-gathered and every rank takes the same restart decisions.  A rank's torch draws start from the
    common state advanced by its guess of the lower ranks' draw count (last attempt's count), so the
    stream positions are checked exactly as in one process.

    Returns (centres f32 [S*K, D] of ALL segments, last assignment i32 local to each segment, for the
    rows of X)."""
    dev = X.device
    sizes = np.asarray(sizes, dtype=np.int64)
    S, K = len(sizes), n_clusters
    limits = np.asarray(iter_limits, dtype=np.int64).reshape(S)
    off = np.concatenate([[0], np.cumsum(sizes)])
    o0, o1 = (0, S) if comm is None else (int(owned[0]), int(owned[1]))
    base = int(off[o0])  # X's first row is segment o0's first row
    if X.shape[0] != off[o1] - off[o0]:
        raise ValueError("fit_segments: rows do not match the owned segments")
    min_loss_mode = target_nodes_num is not None
    if min_loss_mode and (limits == 0).any():
        raise ValueError("fit_segments: fit_by_min_loss needs a finite iter_limit per segment")
    if not min_loss_mode and (inits is None or len(inits) != S):
        raise ValueError("fit_segments: fit needs each segment's drawn start")
    centers = torch.empty((S * K, X.shape[1]), dtype=torch.float32, device=dev)
    last = torch.empty((max(X.shape[0], 1),), dtype=torch.int32, device=dev)
    torch_state = torch.get_rng_state()
    owner, window = next(_TRACE_OWNERS), 0
    start, restarts, guess, solo = 0, 0, 0, False
    while start < S:
        # after an attempt that kept nothing (the window's first segment drew out of the reference's order)
        # that segment runs alone, which is exact by construction; every multi-segment window that stopped
        # short (kept nothing or part) counts against the restart budget, so a run of such windows falls
        # back to one segment at a time after max_restarts instead of re-running every remaining segment
        stop = start + 1 if (solo or restarts > max_restarts) else S
        np_states, seg_inits = [], []
        for s in range(start, stop):
            if min_loss_mode:
                np_states.append(np.random.get_state())
                seg_inits.append([init_indices(int(sizes[s]), K) for _ in range(reinit_draws(limits[s]))])
            else:
                seg_inits.append(inits[s])
        m0, m1 = max(start, o0), min(stop, o1)  # this rank's segments of the window
        torch.set_rng_state(torch_state)
        if guess:
            torch.randint(2, (guess,))
        iters = np.zeros(0, dtype=np.int64)
        ev = np.zeros((0, 2), dtype=np.int64)  # (segment, stream position) in this rank's draw order
        c_mine = torch.empty((0, X.shape[1]), dtype=torch.float32, device=dev)
        if m1 > m0:
            layout = ops.SegmentLayout(sizes[m0:m1], dev)
            xs = X[int(off[m0]) - base:int(off[m1]) - base].contiguous()
            c_mine, a, info = batched_fit(xs, layout, K, limits[m0:m1], seg_inits[m0 - start:m1 - start],
                                          target_nodes_num=target_nodes_num, tol=tol, half=half, return_info=True,
                                          trace_tag={"owner": owner, "seg_base": m0, "window": window})
            last[int(off[m0]) - base:int(off[m1]) - base] = a
            iters = np.asarray(info["iterations"], dtype=np.int64)
            ev = np.asarray([(m0 + e[0], guess + t) for t, e in enumerate(info["events"])],
                            dtype=np.int64).reshape(-1, 2)
        if comm is not None:
            c = comm.all_gather_rows(c_mine)
            iters = comm.all_gather_rows(torch.from_numpy(iters)).numpy()
            ev_all = [e.numpy() for e in comm.all_gather_list(torch.from_numpy(ev))]
        else:
            c, ev_all = c_mine, [ev]
        # numpy: the first segment that drew re-initialisations it never used
        bad_np, used = stop, None
        if min_loss_mode:
            for i in range(stop - start):
                u = reinit_draws(max(int(iters[i]), 1))
                if u < len(seg_inits[i]):
                    bad_np, used = start + i, u
                    break
        # torch: the reference's stream position of every draw is its rank in (segment, draw order)
        allev = np.concatenate(ev_all, 0)
        order = np.argsort(allev[:, 0], kind="stable")
        wrong = allev[order[allev[order, 1] != np.arange(len(order))], 0]
        bad_torch = int(wrong.min()) if len(wrong) else stop
        good = min(bad_np + 1, bad_torch, stop)
        centers[start * K:good * K] = c[:(good - start) * K]
        # the generators' state after the kept segments, as the reference leaves it
        if min_loss_mode:
            if good == bad_np + 1:
                np.random.set_state(np_states[bad_np - start])
                for _ in range(used):
                    init_indices(int(sizes[bad_np]), K)
            elif good < stop:
                np.random.set_state(np_states[good - start])
        torch.set_rng_state(torch_state)
        for seg in np.sort(allev[:, 0][allev[:, 0] < good]):
            torch.randint(int(sizes[seg]), (1,))
        torch_state = torch.get_rng_state()
        # next attempt: this rank's draws start after the lower ranks' draws of segments >= good
        guess = int(sum(int((e[:, 0] >= good).sum()) for r, e in enumerate(ev_all) if comm is not None and r < comm.rank))
        solo = good == start
        if good < stop and stop - start > 1:
            restarts += 1
        start = good
        window += 1
    return centers, last[:X.shape[0]]
