"""Step-by-step certification of the GPU trainers against the reference's arithmetic (oracle).

A balanced fit of the reference (balancekmeans/__init__.py:259-465) is, per iteration: fp16 scores
-cdist(X, C) (fp32 ``pairwise_distance_full`` rounded to fp16, or fp16 ``pairwise_distance_half``),
``auction_lap_half`` on them, and the per-cluster means.  The GPU trainers cannot be bit-identical to a
CPU run of the reference: the fp32 accumulation order of the distances differs (an fp16 score can round
the other way), and torch.topk keeps an implementation-defined one of several EQUAL values where the HIP
auction keeps the lowest index.  ``certify_trace`` replays every traced GPU iteration from the GPU's own
input centres and proves that each step is the reference's step up to exactly those two effects:

* scores: every GPU distance lies in the interval any fp32 summation order can produce
  (O.full_dist_interval / O.half_dist_interval); mismatches against the oracle's own rounding are counted;
* auction: on the GPU's scores, the GPU assignment equals the oracle's lowest-index auction bit for bit,
  and the lockstep certificate against torch's own tie choice (O.auction_tie_certificate) is either
  "no divergence" (the reference would assign identically) or a tie-born divergence;
* update: the non-empty centres equal the oracle's means (fp64 sums, 1e-5 relative); an empty cluster
  holds a row of its segment (the reference's torch.randint refill).
"""
from __future__ import annotations

import numpy as np
import torch

from oracle import rq_oracle as O

F32 = np.float32


def _np(t):
    return t.detach().cpu().numpy() if isinstance(t, torch.Tensor) else np.asarray(t)


def certify_step(x: np.ndarray, c_in: np.ndarray, scores_wk16, assign, c_out: np.ndarray, half: bool, stats: dict):
    n, k = len(x), len(c_in)
    a = _np(assign).astype(np.int64)
    if scores_wk16 is not None:
        s = _np(scores_wk16).reshape(k, n).T.astype(np.float16)          # [N][K] fp16 = -distance
        d_gpu = -s.astype(np.float64)
        lo, hi = (O.half_dist_interval if half else O.full_dist_interval)(x, c_in)
        assert ((d_gpu >= lo) & (d_gpu <= hi)).all(), "a GPU score lies outside every summation order's result"
        ref = O.cdist_half(x, c_in) if half else O.cdist_f32(x, c_in).astype(np.float16)
        stats["order_flips"] += int((ref.astype(np.float64) != d_gpu).sum())
        stats["scores"] += n * k
        if n >= k:
            cert = O.auction_tie_certificate(s.astype(F32))
            assert np.array_equal(a, cert["stable"]), "GPU auction != oracle (lowest-index rule) on the same scores"
            assert cert["tie_born"], f"auction divergence at round {cert['round']} ({cert['step']}) is not a tie"
            stats["tie_divergences"] += int(cert["diverged"])
            stats["auctions"] += 1
        else:  # the reference's argmin(-D) fallback (:24-26)
            assert np.array_equal(a, s.astype(F32).argmin(1))
    cnt = np.bincount(a, minlength=k)
    want = c_in.astype(F32).copy()
    for j in range(k):
        if cnt[j]:
            want[j] = (x[a == j].astype(np.float64).sum(0) / cnt[j]).astype(F32)
    full = cnt > 0
    np.testing.assert_allclose(c_out[full], want[full], rtol=1e-5, atol=1e-6)
    for j in np.nonzero(~full)[0]:
        assert (x == c_out[j]).all(1).any(), "an empty cluster's refill is not a row of its data"
    stats["steps"] += 1


def new_stats():
    return {"steps": 0, "auctions": 0, "tie_divergences": 0, "order_flips": 0, "scores": 0}


def certify_trace(events, stats=None, batched_stride: int = 1):
    """events: the dicts balancekmeans.TRACE received; batched events are certified segment by segment
    (every ``batched_stride``-th (segment, iteration) pair: the oracle auction is slow in numpy)."""
    stats = stats or new_stats()
    xs = {}
    for ev in events:
        key = id(ev["x"])
        if key not in xs:
            xs[key] = _np(ev["x"]).astype(F32)
        x, half = xs[key], bool(ev["half"])
        c_in, c_out = _np(ev["centers_in"]), _np(ev["centers_out"])
        if ev["kind"] == "fit":
            certify_step(x, c_in, ev["scores"], ev["assign"], c_out, half, stats)
            continue
        off, act = ev["off"], ev["active"]
        k = len(c_in) // (len(off) - 1)
        a = _np(ev["assign"])
        w = _np(ev["scores"]) if ev["scores"] is not None else None
        it = np.asarray(ev["iteration"])
        for s in np.nonzero(act)[0]:
            if (int(it[s]) + s) % batched_stride:
                continue
            r0, r1 = int(off[s]), int(off[s + 1])
            blk = None if w is None else w[k * r0:k * r1]
            certify_step(x[r0:r1], c_in[s * k:(s + 1) * k], blk, a[r0:r1], c_out[s * k:(s + 1) * k], half, stats)
    return stats


class Recorder:
    """Collects balancekmeans.TRACE events (keeps references: the traced tensors are fresh clones)."""

    def __init__(self):
        self.events = []

    def __call__(self, ev):
        self.events.append(ev)


def sse(x: np.ndarray, centers: np.ndarray, assign: np.ndarray) -> float:
    """Within-cluster sum of squared distances (fp64) of an assignment."""
    d = x.astype(np.float64) - centers.astype(np.float64)[np.asarray(assign, dtype=np.int64)]
    return float((d * d).sum())
