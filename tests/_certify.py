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


def _host_scores(x: np.ndarray, c: np.ndarray, half: bool) -> np.ndarray:
    """[N][K] fp16 distances as the reference computes them on the host: its own torch.cdist call for the
    fp32 path (O.torch_cdist_batched), the oracle's restatement of torch's fp16 cdist for the half path
    (the reference's pairwise_distance_half only runs on CUDA, tests/golden/make_golden.py g_dist_half)."""
    return O.cdist_half(x, c) if half else O.torch_cdist_batched(x, c).astype(np.float16)


def certify_step(x: np.ndarray, c_in: np.ndarray, scores_wk16, assign, c_out: np.ndarray, half: bool, stats: dict,
                 loss=None, target=None) -> bool:
    """Certify one GPU iteration; returns True when the reference, replayed on the host from the same input
    centres, would have taken a different step (a certified divergence: a topk / max tie, an fp16 score
    rounded the other way by the summation order, or a nearest-centre near tie in the min-loss count)."""
    n, k = len(x), len(c_in)
    a = _np(assign).astype(np.int64)
    diverged = False
    if scores_wk16 is not None:
        s = _np(scores_wk16).reshape(k, n).T.astype(np.float16)          # [N][K] fp16 = -distance
        d_gpu = -s.astype(np.float64)
        lo, hi = (O.half_dist_interval if half else O.full_dist_interval)(x, c_in)
        assert ((d_gpu >= lo) & (d_gpu <= hi)).all(), "a GPU score lies outside every summation order's result"
        ref = _host_scores(x, c_in, half)
        flips = int((ref.astype(np.float64) != d_gpu).sum())
        stats["order_flips"] += flips
        stats["scores"] += n * k
        neg_ref = -ref.astype(F32)
        if n >= k:
            cert = O.auction_tie_certificate(s.astype(F32))
            assert np.array_equal(a, cert["stable"]), "GPU auction != oracle (lowest-index rule) on the same scores"
            assert cert["tie_born"], f"auction divergence at round {cert['round']} ({cert['step']}) is not a tie"
            stats["tie_divergences"] += int(cert["diverged"])
            stats["auctions"] += 1
            ref_a = cert["torch"] if flips == 0 else O.auction_lap_half(neg_ref, tie_rule="torch")
            if not np.array_equal(ref_a, a):
                assert cert["diverged"] or flips, "GPU auction != the reference's on identical scores without a tie"
                diverged = True
        else:  # the reference's argmin(-D) fallback (:24-26)
            assert np.array_equal(a, s.astype(F32).argmin(1))
            if not np.array_equal(neg_ref.argmin(1), a):
                assert flips, "argmin fallback differs from the reference's on identical scores"
                diverged = True
    else:  # unbalanced: exact nearest centre vs the reference's fp32 cdist argmin
        ref_a = O.torch_cdist_batched(x, c_in).argmin(1)
        bad = np.nonzero(ref_a != a)[0]
        if len(bad):
            assert O.near_tie(x[bad], c_in, a[bad], ref_a[bad]).all(), "nearest centre differs beyond a near tie"
            diverged = True
    cnt = np.bincount(a, minlength=k)
    want = c_in.astype(F32).copy()
    for j in range(k):
        if cnt[j]:
            want[j] = (x[a == j].astype(np.float64).sum(0) / cnt[j]).astype(F32)
    full = cnt > 0
    np.testing.assert_allclose(c_out[full], want[full], rtol=1e-5, atol=1e-6)
    for j in np.nonzero(~full)[0]:
        assert (x == c_out[j]).all(1).any(), "an empty cluster's refill is not a row of its data"
    if loss is not None:  # fit_by_min_loss's overflow loss of the updated centres (:327-340)
        host = (-_host_scores(x, c_out, True).astype(F32)).argmax(1) if half else O.torch_cdist_batched(x, c_out).argmin(1)
        cnt_h = np.bincount(host, minlength=k)
        host_loss = float(np.maximum(cnt_h - target, 0)[cnt_h > target].sum())
        if host_loss != float(loss):
            if not half:
                gpu = O.nearest(x, c_out, exact=True)
                bad = np.nonzero(gpu != host)[0]
                assert len(bad) and O.near_tie(x[bad], c_out, gpu[bad], host[bad]).all(), \
                    "min-loss count differs beyond near ties"
            stats["loss_divergences"] += 1
            diverged = True
    stats["steps"] += 1
    stats["divergent_steps"] += int(diverged)
    return diverged


COUNTERS = ("steps", "auctions", "tie_divergences", "order_flips", "scores", "divergent_steps", "loss_divergences")


def new_stats():
    return {**{k: 0 for k in COUNTERS}, "segments": {}}


def _mark(stats, key, window, diverged, delta):
    """record one certified step of segment ``key`` in lockstep window ``window``: a later window replaces
    the segment's record (fit_segments re-ran it; the earlier attempt's result was discarded)"""
    cur = stats["segments"].get(key)
    if cur is None or window > cur["window"]:
        cur = stats["segments"][key] = {"window": window, "diverged": False, **{k: 0 for k in COUNTERS}}
    if window == cur["window"]:
        cur["diverged"] |= bool(diverged)
        for k in COUNTERS:
            cur[k] += delta[k]


def summary(stats) -> dict:
    """the counters split by what the run kept: ``kept`` sums the attempts whose results the fit returned
    (the steps the exactness claims rest on); ``discarded`` the speculative lockstep windows fit_segments
    threw away and re-ran; ``all`` both (every traced, certified step)"""
    kept = {k: sum(v[k] for v in stats["segments"].values()) for k in COUNTERS}
    total = {k: stats[k] for k in COUNTERS}
    return {"all": total, "kept": kept, "discarded": {k: total[k] - kept[k] for k in COUNTERS},
            "kept_divergent_segments": sum(bool(v["diverged"]) for v in stats["segments"].values())}


def certify_trace(events, stats=None):
    """events: the dicts balancekmeans.TRACE received, every one certified (batched events segment by
    segment).  ``stats["segments"]`` maps (owner, global segment) -> {"diverged", "steps"} over the attempt
    that produced the kept result (fit_segments may re-run a segment in a later window): a segment whose
    steps never diverged must have reproduced the reference's result exactly."""
    stats = stats or new_stats()
    xs = {}
    for ev in events:
        key = id(ev["x"])
        if key not in xs:
            xs[key] = _np(ev["x"]).astype(F32)
        x, half = xs[key], bool(ev["half"])
        c_in, c_out = _np(ev["centers_in"]), _np(ev["centers_out"])
        if ev["kind"] == "fit":
            before = {k: stats[k] for k in COUNTERS}
            dv = certify_step(x, c_in, ev["scores"], ev["assign"], c_out, half, stats, ev.get("loss"), ev.get("target"))
            _mark(stats, (ev["owner"], 0), 0, dv, {k: stats[k] - before[k] for k in COUNTERS})
            continue
        off, act = ev["off"], ev["active"]
        k = len(c_in) // (len(off) - 1)
        a = _np(ev["assign"])
        w = _np(ev["scores"]) if ev["scores"] is not None else None
        loss = ev.get("loss")
        for s in np.nonzero(act)[0]:
            r0, r1 = int(off[s]), int(off[s + 1])
            blk = None if w is None else w[k * r0:k * r1]
            before = {k: stats[k] for k in COUNTERS}
            dv = certify_step(x[r0:r1], c_in[s * k:(s + 1) * k], blk, a[r0:r1], c_out[s * k:(s + 1) * k], half, stats,
                              None if loss is None else loss[s], ev.get("target"))
            _mark(stats, (ev["owner"], ev["seg_base"] + int(s)), ev["window"], dv,
                  {kk: stats[kk] - before[kk] for kk in COUNTERS})
    return stats


def diverged_segments(stats, owner) -> set:
    """global segment indices of one fit_segments call (or KMeans object) that took a certified divergence"""
    return {seg for (o, seg), v in stats["segments"].items() if o == owner and v["diverged"]}


def owners(events, kind=None) -> list:
    """trace owners in order of first appearance (one per KMeans object / fit_segments call)"""
    out = []
    for ev in events:
        if (kind is None or ev["kind"] == kind) and ev["owner"] not in out:
            out.append(ev["owner"])
    return out


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


def global_ids(ids: np.ndarray, need, match: np.ndarray = None) -> np.ndarray:
    """the centre rows a 3-level code addresses: level 1 = parent block (id0 * need1 + id1); level 2 = the
    id2-th allowed column of group id0 * need0 + id1 (hierarchical :824, :1055-1086) or, without a match
    matrix (simplified, whose last-level ids are raw candidate indices), id2 itself"""
    g = np.asarray(ids, np.int64).copy()
    g[:, 1] = ids[:, 0] * need[1] + ids[:, 1]
    if match is not None:
        before = ids[:, 0] * need[0] + ids[:, 1]
        cols = np.cumsum(np.asarray(match) == 1, axis=1) - 1
        g[:, 2] = [int(np.nonzero(cols[b] == k)[0][0]) for b, k in zip(before, ids[:, 2])]
    return g


def level_sse(x: np.ndarray, centers, glob: np.ndarray, normalize: bool) -> list:
    """per-level reconstruction SSE of a residual code: level l quantises r_l (r_0 = x, r_{l+1} = the
    residual of r_l against its centre, group-normalised in the hierarchical trainer, :1088-1128)"""
    r = np.asarray(x, F32)
    out = []
    for l, c in enumerate(centers):
        c = np.asarray(c, F32)
        out.append(sse(r, c, glob[:, l]))
        if l < len(centers) - 1:
            r = O.residual(r, c, glob[:, l], normalize=normalize)
    return out
