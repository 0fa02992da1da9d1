"""ORACLE — TEST INFRASTRUCTURE ONLY.  Never imported by the product package.

A CPU (numpy) restatement of the reference hot path, used as the checker by
``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s cpu_baseline leg.
Every function cites the reference file:line it restates
(paths relative to /root/reference/src/semantic_id_generator/).

Pinning: the restatement is checked against golden vectors captured by running
the reference itself in the build container (``tests/golden/make_golden.py``,
fixtures ``tests/golden/*.npz``; see tests/test_oracle_golden.py).

Arithmetic: distances follow torch.cdist's matrix-multiply expansion in fp32
(``sqrt(clamp(|x|^2 + |c|^2 - 2 x.c, 0))``, ATen ``_euclidean_dist``) with a
first-index argmin, exactly the structure the reference runs; summation order
inside BLAS differs from MKL/oneDNN, so two nearly tied centres (relative gap
< ~1e-6) may be ordered differently — ``near_tie`` classifies such rows in fp64.
"""
from __future__ import annotations

import json
from typing import List, Optional, Sequence

import numpy as np

F32 = np.float32


# ---------------------------------------------------------------------------
# distances / argmin
# ---------------------------------------------------------------------------
def cdist_f32(x: np.ndarray, c: np.ndarray) -> np.ndarray:
    """balancekmeans/__init__.py:576-603 pairwise_distance_full -> torch.cdist (mm expansion)."""
    x = x.astype(F32, copy=False)
    c = c.astype(F32, copy=False)
    xn = np.einsum("ij,ij->i", x, x, dtype=F32)[:, None]
    cn = np.einsum("ij,ij->i", c, c, dtype=F32)[None, :]
    d2 = (F32(-2.0) * x) @ c.T + xn + cn
    return np.sqrt(np.maximum(d2, F32(0.0)), dtype=F32)


def pairwise_cosine(x: np.ndarray, c: np.ndarray) -> np.ndarray:
    """balancekmeans/__init__.py:625-655 pairwise_cosine: both operands divided by their fp32 row norms,
    then 1 - the fp32 matrix product (the distance='cosine' option of KMeans, :279-280, 511-512)."""
    x = x.astype(F32, copy=False)
    c = c.astype(F32, copy=False)
    xn = (x / np.sqrt((x.astype(np.float64) ** 2).sum(1, keepdims=True)).astype(F32)).astype(F32)
    cn = (c / np.sqrt((c.astype(np.float64) ** 2).sum(1, keepdims=True)).astype(F32)).astype(F32)
    return (F32(1.0) - xn @ cn.T).astype(F32)


def torch_cdist_batched(x: np.ndarray, c: np.ndarray, batch_size: int = 10000) -> np.ndarray:
    """pairwise_distance_full (balancekmeans/__init__.py:576-603) itself: torch.cdist on the CPU over
    batches of 10000 rows (the third-party arithmetic the reference calls; its summation order is that
    of torch's CPU kernels, so on the host that produced the goldens it reproduces them bit for bit)."""
    import torch
    xt, ct = torch.from_numpy(np.ascontiguousarray(x, F32)), torch.from_numpy(np.ascontiguousarray(c, F32))
    out = np.empty((len(x), len(c)), dtype=F32)
    for i in range(0, len(x), batch_size):
        out[i:i + batch_size] = torch.cdist(xt[i:i + batch_size].unsqueeze(0), ct.unsqueeze(0)).squeeze(0).numpy()
    return out


def cdist_half(x: np.ndarray, c: np.ndarray) -> np.ndarray:
    """pairwise_distance_half (balancekmeans/__init__.py:536-574): ``torch.cdist`` of the fp16-rounded
    operands, clamped at 1e-5, with torch's fp16 arithmetic (ATen ``_euclidean_dist`` on half tensors,
    as measured against torch 2.10 CPU in tests/test_oracle_golden.py):
      |x|^2 = fp16(sum_i fp16(x_i^2))                   (x.pow(2) is an fp16 tensor; fp32 accumulation)
      d^2   = fp16([-2x, |x|^2, 1] . [c, 1, |c|^2])      (fp16 x fp16 products exact; fp32 accumulation)
      d     = fp16(sqrt(max(d^2, 0)));  clamp(min=1e-5)  (the fp16 of 1e-5 is 168 * 2^-24)
    The fp32 accumulation order inside torch's kernels is not reproduced: ``half_dist_interval`` bounds
    what any order can give."""
    f16 = np.float16
    xh = np.asarray(x, F32).astype(f16).astype(F32)
    ch = np.asarray(c, F32).astype(f16).astype(F32)
    xn = (xh * xh).astype(f16).astype(F32).sum(1, dtype=F32).astype(f16).astype(F32)
    cn = (ch * ch).astype(f16).astype(F32).sum(1, dtype=F32).astype(f16).astype(F32)
    d2 = (((F32(-2.0) * xh) @ ch.T + xn[:, None]).astype(F32) + cn[None, :]).astype(F32).astype(f16)
    d = np.sqrt(np.maximum(d2.astype(F32), F32(0.0))).astype(f16)
    return np.maximum(d, f16(1e-5))


def _fp32_sum_bound(n_terms: int) -> float:
    """First-order bound on the relative (to sum |t|) error of an fp32 sum of n terms in any order."""
    return (n_terms - 1) * 2.0 ** -24 * 1.0001


def half_dist_interval(x: np.ndarray, c: np.ndarray):
    """[lo, hi] (fp16 values as float64) of every result ``pairwise_distance_half`` can give under ANY
    fp32 accumulation order of its two sums (the norms and the augmented product): the arbiter for a
    mismatch between two correct implementations (the reference's torch kernels and the HIP kernel)."""
    f16 = np.float16
    xh = np.asarray(x, F32).astype(f16).astype(np.float64)
    ch = np.asarray(c, F32).astype(f16).astype(np.float64)
    d = xh.shape[1]

    def norm_range(v):
        sq = (v * v).astype(f16).astype(np.float64)
        t = sq.sum(1)
        e = _fp32_sum_bound(d) * t
        return (t - e).astype(f16).astype(np.float64), (t + e).astype(f16).astype(np.float64)

    xlo, xhi = norm_range(xh)
    clo, chi = norm_range(ch)
    dot = -2.0 * (xh @ ch.T)
    mag = 2.0 * (np.abs(xh) @ np.abs(ch).T)
    lo = dot + xlo[:, None] + clo[None, :]
    hi = dot + xhi[:, None] + chi[None, :]
    e = _fp32_sum_bound(d + 2) * (mag + xhi[:, None] + chi[None, :])
    lo, hi = lo - e, hi + e

    def fin(v):
        v16 = np.maximum(v.astype(f16).astype(F32), F32(0.0))
        return np.maximum(np.sqrt(v16).astype(f16), f16(1e-5)).astype(np.float64)

    return fin(lo), fin(hi)


def full_dist_interval(x: np.ndarray, c: np.ndarray):
    """[lo, hi] of fp16(cdist_fp32(x, c)) (``auction_lap_half(-pairwise_distance_full)``'s input, :29)
    over any fp32 summation order of torch.cdist's mm expansion (|x|^2, |c|^2 and the augmented
    product)."""
    f16 = np.float16
    xd = np.asarray(x, F32).astype(np.float64)
    cd = np.asarray(c, F32).astype(np.float64)
    d = xd.shape[1]
    xn = (xd * xd).sum(1)
    cn = (cd * cd).sum(1)
    exact = xn[:, None] + cn[None, :] - 2.0 * (xd @ cd.T)
    e = _fp32_sum_bound(d + 2) * (2.0 * (np.abs(xd) @ np.abs(cd).T) + xn[:, None] + cn[None, :]) * 2.0
    lo = np.sqrt(np.maximum(exact - e, 0.0)).astype(F32).astype(f16).astype(np.float64)
    hi = np.sqrt(np.maximum(exact + e, 0.0)).astype(F32).astype(f16).astype(np.float64)
    return lo, hi


def uncertified(got, ref, lo, hi) -> np.ndarray:
    """Mask of entries where got != ref and one of them lies outside the [lo, hi] interval any
    summation order can produce (a real arithmetic difference, not an order effect)."""
    g = np.asarray(got, np.float64)
    r = np.asarray(ref, np.float64)
    return (g != r) & ((g < lo) | (g > hi) | (r < lo) | (r > hi))


def exact_d2(x: np.ndarray, c: np.ndarray) -> np.ndarray:
    """fp64 squared distances (the arbiter for near ties)."""
    x = x.astype(np.float64)
    c = c.astype(np.float64)
    d = (x * x).sum(1)[:, None] + (c * c).sum(1)[None, :] - 2.0 * (x @ c.T)
    # identical centres have identical exact distances; the blocked GEMM can round their columns
    # differently, so duplicates copy their first occurrence's column (exact ties -> lowest index)
    _, first, inv = np.unique(c, axis=0, return_index=True, return_inverse=True)
    src = first[inv.reshape(-1)]
    if (src != np.arange(len(c))).any():
        d = d[:, src]
    return d


def _dist(x: np.ndarray, c: np.ndarray, exact: bool) -> np.ndarray:
    """fp32 cdist (the reference's arithmetic) or, with exact=True, fp64 squared distances:
    the argmin of the latter is the exact nearest centre, which is what the HIP kernels
    return (lowest index on exact ties)."""
    return exact_d2(x, c) if exact else cdist_f32(x, c)


def nearest(x: np.ndarray, c: np.ndarray, chunk: int = 65536, exact: bool = False) -> np.ndarray:
    """KMeans.predict (balancekmeans/__init__.py:489-534): argmin of cdist, first index on ties."""
    out = np.empty(len(x), dtype=np.int64)
    for i in range(0, len(x), chunk):
        out[i:i + chunk] = _dist(x[i:i + chunk], c, exact).argmin(1)
    return out


def segmented_nearest(x: np.ndarray, c: np.ndarray, seg: np.ndarray, allowed: List[np.ndarray],
                      penalty: str = "10000", exact: bool = False) -> np.ndarray:
    """Masked argmin of hierarchical_rq_kmeans.py:876-890 / :942-952 / :1207-1221 / :1274-1288
    and simplified_semantic_id_generator.py:149-161 / :319-328.

    Row i may only take centres ``allowed[seg[i]]`` (global indices, ascending).  With the
    hierarchical ``+10000*(1-mask)`` the masked-out centres can never win while the
    allowed distances stay below 10000 (always true for normalised residuals), so the
    restatement computes the restricted argmin directly; an EMPTY allowed set reproduces
    ``argmin(fl32(d + 10000))`` over every centre. Returns global indices."""
    out = np.empty(len(x), dtype=np.int64)
    order = np.argsort(seg, kind="stable")
    bounds = np.searchsorted(seg[order], np.arange(len(allowed) + 1))
    for s in range(len(allowed)):
        rows = order[bounds[s]:bounds[s + 1]]
        if len(rows) == 0:
            continue
        a = allowed[s]
        if len(a) == 0:
            if penalty == "inf":
                out[rows] = 0  # argmin over an all-inf row
            else:
                if exact:
                    d = np.sqrt(np.maximum(exact_d2(x[rows], c), 0).astype(F32)).astype(F32)
                else:
                    d = cdist_f32(x[rows], c)
                out[rows] = (d + F32(10000.0)).argmin(1)
            continue
        out[rows] = a[_dist(x[rows], c[a], exact).argmin(1)]
    return out


def near_tie(x: np.ndarray, c: np.ndarray, a: np.ndarray, b: np.ndarray, rel: float = 1e-6) -> np.ndarray:
    """True where centres a[i] and b[i] are within ``rel`` (relative, fp64) of each other for row i."""
    x = x.astype(np.float64)
    da = ((x - c[a].astype(np.float64)) ** 2).sum(1)
    db = ((x - c[b].astype(np.float64)) ** 2).sum(1)
    return np.abs(np.sqrt(da) - np.sqrt(db)) <= rel * np.maximum(np.sqrt(np.maximum(da, db)), 1e-30)


# ---------------------------------------------------------------------------
# residuals / weights
# ---------------------------------------------------------------------------
def residual(x: np.ndarray, c: np.ndarray, ids: np.ndarray, group_dims: Sequence[int] = (),
             normalize: bool = True) -> np.ndarray:
    """_compute_residuals_with_centers (hierarchical_rq_kmeans.py:1088-1128): r = x - c[id]; per
    dimension group r_g /= (||r_g|| + 1e-8) in fp32.  normalize=False: simplified :78-96.
    The norm is taken in fp64 and rounded once (torch's fp32 reduction may differ by 1 ulp)."""
    r = (x.astype(F32) - c.astype(F32)[ids]).astype(F32)
    if not normalize:
        return r
    gd = list(group_dims) or [x.shape[1]]
    s = 0
    for g in gd:
        blk = r[:, s:s + g]
        n = np.sqrt((blk.astype(np.float64) ** 2).sum(1, keepdims=True)).astype(F32)
        r[:, s:s + g] = blk / (n + F32(1e-8))
        s += g
    return r


def apply_weights(x: np.ndarray, group_dims: Sequence[int], weights: Sequence[float]) -> np.ndarray:
    """_apply_weights (hierarchical_rq_kmeans.py:583-604)."""
    w = np.concatenate([np.full(g, wv, dtype=F32) for g, wv in zip(group_dims, weights)])
    return (x.astype(F32) * w[None, :]).astype(F32)


# ---------------------------------------------------------------------------
# multi-level encode
# ---------------------------------------------------------------------------
def match_allowed(match: np.ndarray) -> List[np.ndarray]:
    return [np.nonzero(row)[0] for row in np.asarray(match)]


def merge_match_ids(match: np.ndarray, raw: np.ndarray, before: np.ndarray) -> np.ndarray:
    """_merge_match_matrix_cluster_ids (hierarchical_rq_kmeans.py:1055-1086): rank of the raw
    column among the group's allowed columns; a column outside the allowed set raises KeyError."""
    m = np.asarray(match) == 1
    rank = np.cumsum(m, axis=1) - 1
    ok = m[before, raw]
    if not ok.all():
        i = int(np.nonzero(~ok)[0][0])
        raise KeyError(int(raw[i]))
    return rank[before, raw].astype(np.int64)


def encode(x: np.ndarray, centers: Sequence[np.ndarray], need: Sequence[int],
           match: Optional[np.ndarray] = None, group_dims: Sequence[int] = (),
           weights: Optional[Sequence[Sequence[float]]] = None, *, normalize: bool = True,
           match_lookup: bool = True, residual_global_id: bool = True, remap_last: bool = True,
           last_group_mult: str = "need_l_minus_2", residual_from_weighted: bool = False,
           exact: bool = False) -> np.ndarray:
    """HierarchicalRQKMeans.predict (hierarchical_rq_kmeans.py:539-581, levels :1146-1305) and the
    training-time reassignment it mirrors (:839-966); simplified path with normalize=False,
    remap_last=False, last_group_mult='need_minus_2' (simplified :145-172, :305-331).
    Flags as in generative_ranking_recommender_amd.encode.LevelSemantics."""
    L = len(centers)
    d = x.shape[1]
    gd = list(group_dims) or [d]
    cur = x.astype(F32)
    ids: List[np.ndarray] = []
    for l in range(L):
        w = cur if weights is None else apply_weights(cur, gd, weights[l])
        c = np.asarray(centers[l], dtype=F32)
        if l == 0:
            glob = nearest(w, c, exact=exact)
            out = glob
        elif l < L - 1:
            prev = ids[l - 1]
            nb = need[l]
            allowed = [np.arange(p * nb, (p + 1) * nb) for p in range(need[l - 1])]
            glob = segmented_nearest(w, c, prev, allowed, penalty="10000" if normalize else "inf", exact=exact)
            out = glob % nb
        else:
            if match_lookup:
                mult = need[l - 2] if last_group_mult == "need_l_minus_2" else need[-2]
                before = ids[l - 2] * mult + ids[l - 1]
                allowed = match_allowed(match)
                if before.max() >= len(allowed):
                    raise IndexError("before-id out of range")
                glob = segmented_nearest(w, c, before, allowed, penalty="10000" if normalize else "inf",
                                         exact=exact)
                out = merge_match_ids(match, glob, before) if remap_last else glob
            else:
                glob = nearest(w, c, exact=exact)
                out = glob
        ids.append(out.astype(np.int64))
        if l < L - 1:
            src = w if residual_from_weighted else cur
            cur = residual(src, c, glob if residual_global_id else out, gd, normalize)
    return np.stack(ids, 1)


# ---------------------------------------------------------------------------
# Lloyd update + balanced auction + K-Means drivers
# ---------------------------------------------------------------------------
def centroid_update(x: np.ndarray, assign: np.ndarray, centers: np.ndarray, randint) -> np.ndarray:
    """balancekmeans/__init__.py:314-324: C[k] = mean(X[a==k]); empty -> X[randint(N)]
    (``randint`` stands in for the reference's torch CPU RNG draw ``torch.randint(len(X), (1,))``)."""
    c = centers.astype(F32).copy()
    for k in range(len(c)):
        sel = x[assign == k]
        if len(sel) == 0:
            c[k] = x[int(randint(len(x)))]
        else:
            c[k] = (sel.astype(np.float64).sum(0) / len(sel)).astype(F32)
    return c


def auction_lap_half(job_and_worker_to_score: np.ndarray, tie_rule: str = "torch",
                     max_rounds: Optional[int] = None) -> np.ndarray:
    """balancekmeans/__init__.py:12-140 (return_token_to_worker=True), restated on fp16 numpy arrays.

    Every fp16 operation of the reference is reproduced with one rounding per op.  The one
    implementation-defined step is which of several EQUAL values ``torch.topk`` keeps at the
    selection boundary (and which equal bidder ``max(dim=0)`` reports).  ``tie_rule="torch"``
    delegates exactly those two selections to torch's CPU kernels (the third-party code the
    reference calls; torch 2.10.0 here), which pins the oracle to the reference on tied
    inputs too; ``tie_rule="stable"`` keeps the lowest job / worker index instead (the rule
    the GPU kernels use, identical whenever the fp16 scores have no ties).  ``max_rounds`` stops after
    that many rounds and returns None (bench.py's bounded CPU-baseline sample only)."""
    s = np.asarray(job_and_worker_to_score, dtype=F32)
    num_jobs, num_workers = s.shape
    if num_jobs < num_workers:
        return s.argmin(1).astype(np.int64)  # :24-26
    s16 = s.astype(np.float16)
    spread = np.float16(s16.max().astype(F32) - s16.min().astype(F32))   # fp16 op: rounds
    eps = np.float16(F32(spread) / F32(50.0))                             # fp16 op: rounds
    eps = max(eps, np.float16(1e-4))
    if np.isnan(s16).any():
        raise Exception("NaN distance")
    w = np.ascontiguousarray(s16.T)  # [workers, jobs]
    jpw = num_jobs // num_workers
    value = w.copy()
    cost = np.zeros(num_jobs, dtype=np.float16)
    counter = 0
    index = None
    jobs_without_bidder = None
    if tie_rule == "torch":
        import torch
    while True:
        if tie_rule == "torch":
            tv, ti = torch.from_numpy(value).topk(jpw + 1, dim=1)
            top_index = ti.numpy()
        else:
            top_index = _stable_top(value, jpw + 1)
        top_values = np.take_along_axis(value, top_index, 1)
        inc = ((top_values[:, :-1].astype(F32) - top_values[:, -1:].astype(F32)).astype(np.float16).astype(F32)
               + F32(eps)).astype(np.float16)
        bids = np.zeros((num_workers, num_jobs), dtype=np.float16)
        np.put_along_axis(bids, top_index[:, :-1], inc, 1)
        if counter < 100 and index is not None:
            bids.reshape(-1)[index] = eps
        if counter > 1000:
            bids.reshape(-1)[jobs_without_bidder] = eps
        jobs_with_bidder = np.nonzero((bids > 0).any(0))[0]
        jobs_without_bidder = np.nonzero((bids == 0).all(0))[0]
        sub = bids[:, jobs_with_bidder]
        if tie_rule == "torch":
            hb, hbr = torch.from_numpy(np.ascontiguousarray(sub)).max(dim=0)
            high_bidders, high_bids = hbr.numpy(), hb.numpy()
        else:
            high_bidders = sub.argmax(0)
            high_bids = sub[high_bidders, np.arange(len(jobs_with_bidder))]
        if len(high_bidders) == num_jobs:
            return high_bidders.astype(np.int64)
        prev = (cost.copy(), index)
        cost[jobs_with_bidder] = (cost[jobs_with_bidder].astype(F32) + high_bids.astype(F32)).astype(np.float16)
        value = (w.astype(F32) - cost[None, :].astype(F32)).astype(np.float16)
        index = high_bidders * num_jobs + jobs_with_bidder
        value.reshape(-1)[index] = w.reshape(-1)[index]
        counter += 1
        if max_rounds is not None and counter >= max_rounds:
            return None
        counter = _fast_forward(counter, prev, cost, index, max_rounds)


def auction_rounds_torch_cpu(job_and_worker_to_score: np.ndarray, rounds: int) -> float:
    """Seconds per round of auction_lap_half (:12-140) on the host, with the reference's tensor operations
    (torch CPU fp16: topk of jpw+1 per worker, bid scatter, retention overwrite, max over bidders, cost
    and value update) -- the CPU-baseline leg of bench.py, which times ``rounds`` rounds of one auction
    (the numpy restatement above is the checker; its per-round cost is ~20x torch's)."""
    import time

    import torch
    w = torch.from_numpy(np.ascontiguousarray(np.asarray(job_and_worker_to_score, F32).T)).half()
    k, n = w.shape
    jpw = n // k
    eps = max((w.max() - w.min()) / 50, torch.tensor(1e-4, dtype=torch.float16))
    val = w.clone()
    cost = torch.zeros(n, dtype=torch.float16)
    keep = None
    t0 = time.perf_counter()
    for _ in range(rounds):
        top_v, top_i = val.topk(jpw + 1, dim=1)
        bid = torch.zeros_like(w)
        bid.scatter_(1, top_i[:, :-1], (top_v[:, :-1] - top_v[:, -1:]) + eps)
        if keep is not None:
            bid.view(-1)[keep] = eps
        has = (bid > 0).any(0)
        jobs = has.nonzero().squeeze(1)
        hb, hw = bid[:, jobs].max(dim=0)
        cost[jobs] += hb
        val = w - cost
        keep = hw * n + jobs
        val.view(-1)[keep] = w.view(-1)[keep]
    return (time.perf_counter() - t0) / rounds


def _desc_key16(v16: np.ndarray) -> np.ndarray:
    """uint16 keys whose ascending order is the DESCENDING order of fp16 values, with -0 == +0 (equal
    values get equal keys, so a stable sort keeps the lowest index among them; 16-bit keys take numpy's
    radix sort)."""
    b = np.asarray(v16, np.float16).view(np.uint16)
    b = np.where(b == 0x8000, np.uint16(0), b).astype(np.uint16)
    asc = np.where(b & 0x8000, ~b, b | np.uint16(0x8000)).astype(np.uint16)
    return (np.uint16(0xFFFF) - asc).astype(np.uint16)


def _stable_top(value: np.ndarray, n: int) -> np.ndarray:
    """indices of the n largest fp16 values per row, lowest index first among equal values"""
    return np.argsort(_desc_key16(value), axis=1, kind="stable")[:, :n]


def _fast_forward(counter: int, prev, cost: np.ndarray, index: np.ndarray, max_rounds=None) -> int:
    """A round of auction_lap_half is a function of (cost, last winners ``index``, and which of the
    counter's regimes it is in: retention bids while counter < 100, leftover bids once counter > 1000).
    When a round left cost and winners unchanged (value is rebuilt from them), every later round of the
    same regime repeats it, so the loop may jump to the regime's last round: the exact same result in
    far fewer host rounds (the 1002-round runs of N % K != 0 spend most rounds waiting for round 1000)."""
    if max_rounds is not None or prev[1] is None or not np.array_equal(prev[0], cost) \
            or not np.array_equal(prev[1], index):
        return counter
    if counter < 100:          # rounds counter..99: retention bids, as the round just run
        return 100
    if 101 <= counter <= 1000:  # rounds counter..1000: neither retention nor leftover bids
        return 1001
    return counter


def _auction_select(value: np.ndarray, jpw: int, tie_rule: str) -> np.ndarray:
    """top_index of ``value.topk(jpw + 1, dim=1)`` (balancekmeans/__init__.py:64-73) under a tie rule."""
    if tie_rule == "torch":
        import torch
        return torch.from_numpy(value).topk(jpw + 1, dim=1)[1].numpy()
    return _stable_top(value, jpw + 1)


def _auction_max(sub: np.ndarray, tie_rule: str):
    """``bids[:, jobs_with_bidder].max(dim=0)`` (:104) -> (high_bids, high_bidders)."""
    if tie_rule == "torch":
        import torch
        hb, hbr = torch.from_numpy(np.ascontiguousarray(sub)).max(dim=0)
        return hb.numpy(), hbr.numpy()
    hbr = sub.argmax(0)
    return sub[hbr, np.arange(sub.shape[1])], hbr


def auction_tie_certificate(job_and_worker_to_score: np.ndarray) -> dict:
    """Certify that two implementations of auction_lap_half (:12-140) that differ only in which of
    several EQUAL values they keep can disagree: the reference's own choice (torch.topk / torch.max on
    the CPU, ``tie_rule="torch"``) and the lowest-index rule of the HIP kernels (``"stable"``) are run in
    lockstep on the same fp16 scores.  While the two states are identical, every round's two selections
    are compared; the first round where they differ is returned with ``tie_born`` = every differing
    selection is among jobs whose value equals that worker's (jpw+1)-th largest (the topk boundary),
    or, for the max over bidders, among equal bids.  After that round the trajectories legitimately
    part.  Two selections whose top-jpw job SETS agree are the same step even when a different one of
    several equal values sits at position jpw+1: the bids (value - (jpw+1)-th value + eps on the top jpw)
    are identical.  Returns {"diverged", "round", "step", "tie_born", "torch", "stable"} (the two results;
    without a divergence both are the lockstep run's)."""
    s = np.asarray(job_and_worker_to_score, dtype=F32)
    num_jobs, num_workers = s.shape
    out = {"diverged": False, "round": -1, "step": None, "tie_born": True}
    if num_jobs < num_workers:
        out["torch"] = out["stable"] = auction_lap_half(s)
        return out

    def parted(**kw):
        out.update(diverged=True, **kw)
        out["torch"] = auction_lap_half(s, tie_rule="torch")
        out["stable"] = auction_lap_half(s, tie_rule="stable")
        return out
    s16 = s.astype(np.float16)
    spread = np.float16(s16.max().astype(F32) - s16.min().astype(F32))
    eps = max(np.float16(F32(spread) / F32(50.0)), np.float16(1e-4))
    w = np.ascontiguousarray(s16.T)
    jpw = num_jobs // num_workers
    value = w.copy()
    cost = np.zeros(num_jobs, dtype=np.float16)
    counter, index, jobs_without_bidder = 0, None, None
    while True:
        ti = _auction_select(value, jpw, "torch")
        si = _auction_select(value, jpw, "stable")
        for wk in range(num_workers):
            # the bids depend on WHICH jobs are in the top jpw and on the (jpw+1)-th VALUE, not on which of
            # several equal values sits at position jpw+1: only a different bid set parts the trajectories
            bt, bs = set(ti[wk, :-1].tolist()), set(si[wk, :-1].tolist())
            if bt != bs:
                thr = value[wk, si[wk, -1]]
                diff = bt ^ bs
                return parted(round=counter, step="topk",
                              tie_born=bool(value[wk, ti[wk, -1]] == thr and all(value[wk, j] == thr for j in diff)))
        top_values = np.take_along_axis(value, ti, 1)
        inc = ((top_values[:, :-1].astype(F32) - top_values[:, -1:].astype(F32)).astype(np.float16).astype(F32)
               + F32(eps)).astype(np.float16)
        bids = np.zeros((num_workers, num_jobs), dtype=np.float16)
        np.put_along_axis(bids, ti[:, :-1], inc, 1)
        if counter < 100 and index is not None:
            bids.reshape(-1)[index] = eps
        if counter > 1000:
            bids.reshape(-1)[jobs_without_bidder] = eps
        jobs_with_bidder = np.nonzero((bids > 0).any(0))[0]
        jobs_without_bidder = np.nonzero((bids == 0).all(0))[0]
        sub = bids[:, jobs_with_bidder]
        hb, hbr = _auction_max(sub, "torch")
        hb_s, hbr_s = _auction_max(sub, "stable")
        if not np.array_equal(hbr, hbr_s):
            k = np.nonzero(hbr != hbr_s)[0]
            return parted(round=counter, step="max", tie_born=bool((sub[hbr[k], k] == sub[hbr_s[k], k]).all()))
        if len(hbr) == num_jobs:
            out["torch"] = out["stable"] = hbr.astype(np.int64)
            return out
        prev = (cost.copy(), index)
        cost[jobs_with_bidder] = (cost[jobs_with_bidder].astype(F32) + hb.astype(F32)).astype(np.float16)
        value = (w.astype(F32) - cost[None, :].astype(F32)).astype(np.float16)
        index = hbr * num_jobs + jobs_with_bidder
        value.reshape(-1)[index] = w.reshape(-1)[index]
        counter = _fast_forward(counter + 1, prev, cost, index)


def assignment_quality(job_and_worker_to_score: np.ndarray, assign: np.ndarray) -> dict:
    """What a balanced assignment optimises and promises: the total fp32 score of the chosen pairs and
    the per-worker job counts (the balance histogram)."""
    s = np.asarray(job_and_worker_to_score, dtype=np.float64)
    a = np.asarray(assign, dtype=np.int64)
    return {"score": float(s[np.arange(len(a)), a].sum()),
            "counts": np.bincount(a, minlength=s.shape[1])}


def auction_lap_full(job_and_worker_to_score: np.ndarray, tie_rule: str = "torch") -> np.ndarray:
    """balancekmeans/__init__.py:142-210 (return_token_to_worker=True): the fp32 auction, reached only
    through ``KMeans.predict(balanced=True)`` (:523-525).  Same steps as ``auction_lap_half`` in fp32, with
    one rounding per op, and two differences of the reference: no N < K fallback (with jobs_per_worker
    = 0 nothing bids until the leftover rule gives every job to worker 0 after round 1000), and eps from
    the fp32 spread.  ``tie_rule`` as in ``auction_lap_half``."""
    s = np.asarray(job_and_worker_to_score, dtype=F32)
    num_jobs, num_workers = s.shape
    eps = F32(F32(s.max() - s.min()) / F32(50.0))
    eps = max(eps, F32(1e-4))
    if np.isnan(s).any():
        raise Exception("NaN distance")
    w = np.ascontiguousarray(s.T)  # [workers, jobs]
    jpw = num_jobs // num_workers
    value = w.copy()
    cost = np.zeros(num_jobs, dtype=F32)
    counter = 0
    index = None
    jobs_without_bidder = None
    if tie_rule == "torch":
        import torch
    while True:
        if tie_rule == "torch":
            tv, ti = torch.from_numpy(value).topk(jpw + 1, dim=1)
            top_index = ti.numpy()
        else:
            order = np.lexsort((np.arange(num_jobs)[None, :].repeat(num_workers, 0), -value), axis=1)
            top_index = order[:, :jpw + 1]
        top_values = np.take_along_axis(value, top_index, 1)
        inc = (top_values[:, :-1] - top_values[:, -1:]) + eps
        bids = np.zeros((num_workers, num_jobs), dtype=F32)
        np.put_along_axis(bids, top_index[:, :-1], inc, 1)
        if counter < 100 and index is not None:
            bids.reshape(-1)[index] = eps
        if counter > 1000:
            bids.reshape(-1)[jobs_without_bidder] = eps
        jobs_with_bidder = np.nonzero((bids > 0).any(0))[0]
        jobs_without_bidder = np.nonzero((bids == 0).all(0))[0]
        sub = bids[:, jobs_with_bidder]
        if tie_rule == "torch":
            hb, hbr = torch.from_numpy(np.ascontiguousarray(sub)).max(dim=0)
            high_bidders, high_bids = hbr.numpy(), hb.numpy()
        else:
            high_bidders = sub.argmax(0)
            high_bids = sub[high_bidders, np.arange(len(jobs_with_bidder))]
        if len(high_bidders) == num_jobs:
            return high_bidders.astype(np.int64)
        cost[jobs_with_bidder] += high_bids
        value = w - cost[None, :]
        index = high_bidders * num_jobs + jobs_with_bidder
        value.reshape(-1)[index] = w.reshape(-1)[index]
        counter += 1


class LegacyRNG:
    """The reference draws init indices from numpy's global legacy RNG (np.random.choice,
    balancekmeans/__init__.py:250-253) and empty-cluster rows from torch's CPU RNG."""

    def __init__(self, np_seed: int, torch_randint):
        self.np = np.random.RandomState(np_seed)
        self.torch_randint = torch_randint

    def choice(self, n, k):
        return self.np.choice(n, k, replace=k > n)


def kmeans_fit(x: np.ndarray, k: int, rng: LegacyRNG, iter_limit: int, balanced: bool, tol: float = 1e-3,
               min_loss_target: Optional[float] = None, dist_fn=None):
    """KMeans.fit (balancekmeans/__init__.py:368-465) and, with min_loss_target, KMeans.fit_by_min_loss
    (:259-365).  Returns (centers, last assignment).  ``dist_fn`` replaces the fp32 distance (default
    ``cdist_f32``; ``torch_cdist_batched`` is the reference's own torch.cdist call, bit for bit on the
    same host)."""
    cdist_f32 = dist_fn or globals()["cdist_f32"]
    x = x.astype(F32)
    c = x[rng.choice(len(x), k)].copy()
    it = 0
    best_loss, best_c = float("inf"), None
    while True:
        if min_loss_target is not None and it > 0 and it % 10 == 0:
            c = x[rng.choice(len(x), k)].copy()
        d = cdist_f32(x, c)
        a = auction_lap_half(-d) if balanced else d.argmin(1)
        prev = c.copy()
        c = centroid_update(x, a, c, rng.torch_randint)
        if min_loss_target is not None:
            cnt = np.bincount(cdist_f32(x, c).argmin(1), minlength=k)
            loss = float(np.maximum(cnt - min_loss_target, 0)[cnt > min_loss_target].sum())
            if loss <= best_loss:
                best_loss, best_c = loss, c.copy()
        shift = np.sqrt(((c.astype(np.float64) - prev) ** 2).sum(1)).sum()
        it += 1
        if shift ** 2 < tol or (iter_limit != 0 and it >= iter_limit):
            break
    return (best_c if min_loss_target is not None else c), a


# ---------------------------------------------------------------------------
# last-layer match matrix (hierarchical :968-1053, simplified :247-303)
# ---------------------------------------------------------------------------
def greedy_unique_nearest(sub: np.ndarray, cand: np.ndarray, n_take: int, dist: str = "cdist") -> List[int]:
    """The greedy step of the match-matrix builders: sub-centre j (in order) takes its nearest candidate
    not taken yet.  ``dist="cdist"``: hierarchical_rq_kmeans.py:1024-1036 (fp32 torch.cdist, the used
    columns set to inf, torch.argmin = first index); ``dist="norm"``: simplified…:279-291 (fp32
    np.linalg.norm of the differences, argsort, first unused; the sort's order among EQUAL distances is
    unspecified in the reference, lowest index here).  Returns the taken columns in pick order."""
    if dist == "cdist":
        d = cdist_f32(sub, cand)
    else:
        d = np.linalg.norm(sub.astype(F32)[:, None, :] - cand.astype(F32)[None, :, :], axis=2)
    used: List[int] = []
    for j in range(n_take):
        row = d[j].astype(F32).copy()
        if used:
            row[used] = np.inf
        used.append(int(np.argmin(row)))  # first index among equal values (argsort(kind=stable) agrees)
    return used


def greedy_certificate(sub: np.ndarray, cand: np.ndarray, n_take: int) -> dict:
    """Which columns EVERY correct fp32 implementation of the greedy step must take.  Distances are
    exact (fp64) with the bound of any fp32 summation order of either distance form (torch.cdist's
    mm expansion or the norm of the differences) plus the final sqrt rounding; step j is determined when
    the exact nearest unused column's upper bound is below every other unused column's lower bound.
    Returns {"determined": all steps determined, "step": first undetermined step (or n_take), "taken":
    the determined columns in order, "tied": the columns that could win the undetermined step}."""
    s = np.asarray(sub, F32).astype(np.float64)
    c = np.asarray(cand, F32).astype(np.float64)
    sn, cn = (s * s).sum(1), (c * c).sum(1)
    d2 = sn[:, None] + cn[None, :] - 2.0 * (s @ c.T)
    e = _fp32_sum_bound(s.shape[1] + 2) * (2.0 * (np.abs(s) @ np.abs(c).T) + sn[:, None] + cn[None, :]) * 2.0
    e = e + 2.0 ** -21 * np.abs(d2)
    taken: List[int] = []
    free = np.ones(len(c), bool)
    for j in range(n_take):
        dj = np.where(free, d2[j], np.inf)
        m = int(np.argmin(dj))
        rivals = free & (d2[j] - e[j] <= d2[j, m] + e[j, m])
        rivals[m] = False
        if rivals.any():
            return {"determined": False, "step": j, "taken": taken, "tied": sorted([m] + np.nonzero(rivals)[0].tolist())}
        taken.append(m)
        free[m] = False
    return {"determined": True, "step": n_take, "taken": taken, "tied": []}


def assign_last_match_matrix(x: np.ndarray, l1: np.ndarray, l2: np.ndarray, cand: np.ndarray,
                             prev_prev_need: int, prev_need: int, need: int, trunc: int, fit_fn,
                             subs_out: Optional[list] = None) -> np.ndarray:
    """HierarchicalRQKMeans._assign_last_match_matrix (hierarchical_rq_kmeans.py:968-1053) on the global
    numpy RNG: per (l1, l2) group in order — no rows: all-zero row (:999-1001); <= need rows: the rows
    (:1005-1006); < trunc rows: ``np.random.choice(n, need, replace=False)`` of them (:1007-1010); else
    ``fit_fn(rows)`` (the balanced sub-K-Means, :1011-1018; it must draw its own initialisation); the
    greedy step (:1020-1036); the random fill (:1042-1049).  ``subs_out`` collects each non-empty group's
    greedy operand."""
    n_cand = len(cand)
    out = np.zeros((prev_prev_need * prev_need, n_cand), dtype=np.uint8)
    for i in range(prev_prev_need):
        for j in range(prev_need):
            idx = np.nonzero((l1 == i) & (l2 == j))[0]
            if len(idx) == 0:
                continue
            sub = x[idx]
            if len(idx) <= need:
                centers = sub
            elif len(idx) < trunc:
                centers = sub[np.random.choice(len(idx), need, replace=False)]
            else:
                centers = fit_fn(sub)
            if subs_out is not None:
                subs_out.append(np.asarray(centers, F32))
            taken = set(greedy_unique_nearest(centers, cand, min(len(centers), need), "cdist"))
            if len(taken) < need:
                for _ in range(need - len(taken)):
                    r = np.random.randint(n_cand)
                    while r in taken:
                        r = np.random.randint(n_cand)
                    taken.add(r)
            out[i * prev_need + j, sorted(taken)] = 1
    return out


def dynamic_match_matrix(x: np.ndarray, l1: np.ndarray, l2: np.ndarray, cand: np.ndarray, n_prev1: int,
                         n_prev2: int, need: int, fit_fn, subs_out: Optional[list] = None) -> np.ndarray:
    """SimplifiedHierarchicalRQ._get_dynamic_match_matrix (simplified_semantic_id_generator.py:247-303):
    per (l1, l2) group — no rows: ``need`` candidates drawn with np.random.choice(replace=False) (:267-268);
    <= need rows: the rows (:269-270); else ``fit_fn(rows)`` (``fit(iter_limit=20)``, :271-276); the greedy
    step over every sub-centre (:279-291); the fill ``while len < need: randint`` (:293-296)."""
    n_cand = len(cand)
    out = np.zeros((n_prev1 * n_prev2, n_cand), dtype=np.uint8)
    for i in range(n_prev1):
        for j in range(n_prev2):
            idx = np.nonzero((l1 == i) & (l2 == j))[0]
            if len(idx) == 0:
                centers = cand[np.random.choice(n_cand, need, replace=False)]
            elif len(idx) <= need:
                centers = x[idx]
            else:
                centers = fit_fn(x[idx])
            if subs_out is not None:
                subs_out.append(np.asarray(centers, F32))
            taken = set(greedy_unique_nearest(centers, cand, len(centers), "norm"))
            while len(taken) < need:
                r = np.random.randint(n_cand)
                if r not in taken:
                    taken.add(r)
            out[i * n_prev2 + j, sorted(taken)] = 1
    return out


def recorded_fits(centres: Sequence[np.ndarray], k: int):
    """A ``fit_fn`` for the builders above that replays recorded sub-K-Means results: it draws the fit's
    initialisation (KMeans.initialize, balancekmeans/__init__.py:240-256; a balanced fit of N >= K rows
    draws nothing else from numpy) and returns the next recorded centres."""
    it = iter(centres)

    def fit(rows):
        np.random.choice(len(rows), k, replace=k > len(rows))
        return next(it)
    return fit


def adaptive_iter_limit(num_samples: int, n_clusters: int, layer: int, base_iter_limit: int = 100,
                        is_sub_cluster: bool = False) -> int:
    """_calculate_adaptive_iter_limit (hierarchical_rq_kmeans.py:288-366)."""
    spc = num_samples / max(n_clusters, 1)
    if is_sub_cluster:
        it = 15 if num_samples < 5000 else 20 if num_samples < 10000 else 25 if num_samples < 20000 else 30
        if spc < 50:
            it = max(10, int(it * 0.8))
        elif spc > 200:
            it = int(it * 1.2)
        return max(10, it)
    if num_samples < 5000:
        it = max(10, int(base_iter_limit * 0.2))
    elif num_samples < 10000:
        it = max(15, int(base_iter_limit * 0.3))
    elif num_samples < 50000:
        it = max(30, int(base_iter_limit * 0.5))
    elif num_samples < 100000:
        it = max(50, int(base_iter_limit * 0.7))
    elif num_samples < 500000:
        it = base_iter_limit
    elif num_samples < 1000000:
        it = int(base_iter_limit * 1.2)
    else:
        it = int(base_iter_limit * 1.5)
    if n_clusters > 512:
        it = int(it * 1.3)
    elif n_clusters > 256:
        it = int(it * 1.15)
    if layer > 1:
        it = max(10, int(it * 0.9))
    if spc < 50:
        it = int(it * 1.2)
    return max(10, it)


def jsonl_lines(song_ids: Sequence[str], ids: np.ndarray) -> bytes:
    """save_semantic_ids (simplified :368-385) / _save_semantic_ids (train_semantic_ids.py:239-264)."""
    return "".join(json.dumps({"song_id": s, "semantic_ids": [int(v) for v in row]}) + "\n"
                   for s, row in zip(song_ids, ids)).encode()
