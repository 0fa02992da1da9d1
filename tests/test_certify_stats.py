"""The certification record separates the kept trajectory from discarded speculative windows (VERDICT r5
item 7): fit_segments may run a segment in a lockstep window, discard that attempt and re-run it in a later
window; the steps of the discarded attempt are certified like any other but do not count against the
kept result's exactness."""
from tests import _certify


def _delta(**kw):
    d = {k: 0 for k in _certify.COUNTERS}
    d["steps"] = 1
    d.update(kw)
    return d


def test_summary_splits_kept_and_discarded_windows():
    st = _certify.new_stats()
    steps = [((7, 0), 0, True, _delta(tie_divergences=1, divergent_steps=1, auctions=1)),   # discarded later
             ((7, 0), 0, False, _delta(auctions=1)),
             ((7, 0), 1, False, _delta(auctions=1)),                                         # kept attempt
             ((7, 0), 1, False, _delta(auctions=1, order_flips=3)),
             ((7, 1), 0, False, _delta(auctions=1))]                                         # kept (only attempt)
    for key, window, dv, d in steps:
        for k in _certify.COUNTERS:
            st[k] += d[k]
        _certify._mark(st, key, window, dv, d)
    s = _certify.summary(st)
    assert s["all"]["steps"] == 5 and s["all"]["tie_divergences"] == 1 and s["all"]["divergent_steps"] == 1
    assert s["kept"]["steps"] == 3 and s["kept"]["tie_divergences"] == 0 and s["kept"]["divergent_steps"] == 0
    assert s["kept"]["order_flips"] == 3
    assert s["discarded"]["steps"] == 2 and s["discarded"]["tie_divergences"] == 1
    assert s["kept_divergent_segments"] == 0
    assert not any(v["diverged"] for v in st["segments"].values())


def test_an_older_window_never_replaces_the_kept_attempt():
    st = _certify.new_stats()
    _certify._mark(st, (1, 4), 2, False, _delta())
    _certify._mark(st, (1, 4), 1, True, _delta(divergent_steps=1))
    assert st["segments"][(1, 4)]["window"] == 2 and not st["segments"][(1, 4)]["diverged"]
    assert _certify.summary(st)["kept"]["steps"] == 1
