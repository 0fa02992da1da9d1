"""The list-round argument of auction_seg.hip (sa_list_round_kernel), checked on the host.

A sweep round records, per worker, every job whose value key is >= its list base lkb = T_prev - 64 keys
(T_prev: the worker's last threshold); a later round may take its threshold T (the (jpw+1)-th largest value),
its tie ranks and its bids from that list alone while T_prev >= lkb and >= jpw + 1 listed values are >= lkb,
because values only fall between rounds except the previous winner's (its raw score), and a worker only wins
a job it bid on from a listed value.  The simulation below runs the reference's auction (oracle fp16
arithmetic, lowest-index tie rule, the GPU's rule) and, in every round a worker would take from its list,
asserts that the list's selection (T, the values above it, the first `need` equal values in job order)
IS the selection over all N values -- on random and heavily tied inputs, through the retention (< 100) and
leftover (> 1000) rounds.  No GPU: this pins the invariant the kernel relies on."""
import numpy as np
import pytest

from oracle import rq_oracle as O

F32 = np.float32
DELTA = 64


def _asc_key(v16):
    return (0xFFFF - O._desc_key16(v16).astype(np.int64))  # ascending order key (-0 == +0)


def _run(s32, delta=DELTA):
    s16 = s32.astype(np.float16)
    n, k = s16.shape
    w = np.ascontiguousarray(s16.T)
    jpw = n // k
    spread = np.float16(s16.max().astype(F32) - s16.min().astype(F32))
    eps = max(np.float16(F32(spread) / F32(50.0)), np.float16(1e-4))
    cost = np.zeros(n, np.float16)
    hb = np.full(n, -1)
    counter, index, no_bidder = 0, None, None
    lists = [None] * k          # (jobs, base key) per worker
    t_prev = [None] * k
    list_rounds = 0
    while True:
        value = (w.astype(F32) - cost[None, :].astype(F32)).astype(np.float16)
        own = hb >= 0
        value[hb[own], np.nonzero(own)[0]] = w[hb[own], np.nonzero(own)[0]]
        keys = _asc_key(value)
        top = O._stable_top(value, jpw + 1)
        for wk in range(k):
            lst = lists[wk]
            ok = lst is not None and counter <= 1000 and t_prev[wk] is not None and t_prev[wk] >= lst[1]
            if ok:
                jobs = lst[0]
                lk = keys[wk, jobs]
                if (lk >= lst[1]).sum() < jpw + 1:
                    ok = False
            if ok:  # the list round's selection must be the sweep's
                cand = jobs[lk >= lst[1]]
                order = cand[np.lexsort((cand, -keys[wk, cand]))]
                sel = order[:jpw + 1]
                assert keys[wk, sel[-1]] == keys[wk, top[wk, -1]], "list threshold != sweep threshold"
                assert set(sel[:-1].tolist()) == set(top[wk, :-1].tolist()), "list bidders != sweep bidders"
                list_rounds += 1
            else:   # the sweep rebuilds the list: jobs with key >= T_prev - delta
                if t_prev[wk] is not None:
                    base = t_prev[wk] - delta
                    lists[wk] = (np.nonzero(keys[wk] >= base)[0], base)
                else:
                    lists[wk] = None
            t_prev[wk] = int(keys[wk, top[wk, -1]])
        # the round itself (balancekmeans/__init__.py:64-126), lowest-index rule
        tv = np.take_along_axis(value, top, 1)
        inc = ((tv[:, :-1].astype(F32) - tv[:, -1:].astype(F32)).astype(np.float16).astype(F32)
               + F32(eps)).astype(np.float16)
        bids = np.zeros((k, n), np.float16)
        np.put_along_axis(bids, top[:, :-1], inc, 1)
        if counter < 100 and index is not None:
            bids.reshape(-1)[index] = eps
        if counter > 1000:
            bids.reshape(-1)[no_bidder] = eps
        with_b = np.nonzero((bids > 0).any(0))[0]
        no_bidder = np.nonzero((bids == 0).all(0))[0]
        sub = bids[:, with_b]
        win = sub.argmax(0)
        if len(win) == n:
            return win, counter + 1, list_rounds
        cost[with_b] = (cost[with_b].astype(F32) + sub[win, np.arange(len(with_b))].astype(F32)).astype(np.float16)
        hb[:] = -1
        hb[with_b] = win
        index = win * n + with_b
        counter += 1


@pytest.mark.parametrize("n,k,levels,seed", [(1600, 16, 0, 1), (1603, 16, 0, 2), (2400, 32, 7, 3), (1000, 8, 3, 4),
                                             (3000, 48, 0, 5)])
def test_list_rounds_select_exactly_what_the_sweep_selects(n, k, levels, seed):
    rng = np.random.default_rng(seed)
    d = rng.random((n, k), dtype=np.float32) * 2 + np.float32(0.5)
    if levels:
        d = np.round(d * levels) / levels
    s = (-d).astype(np.float16).astype(np.float32)
    win, rounds, list_rounds = _run(s)
    want = O.auction_lap_half(s, tie_rule="stable")
    assert np.array_equal(win, want)
    if n % k:
        assert rounds == 1002
    assert list_rounds > 0
