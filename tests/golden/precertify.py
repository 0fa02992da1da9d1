"""Pre-certify candidate training fixtures against the REFERENCE run (build container only).

VERDICT r4 asked for trainer goldens whose reference run takes no tie-born step, so that the per-segment
"no certified divergence => identical to the reference" rule of tests/test_gpu_reference_parity.py is
exercised on a real trainer run instead of being vacuous.  This script runs the reference trainer on a
candidate input (make_golden.py's harness) with hooks on its balanced fits and reports, per fit and per
segment (parent / group):

* auction calls whose two tie rules part (O.auction_tie_certificate: torch.topk / max's own choice
  against the lowest-index rule of the HIP kernels) -- a tie-born divergence the GPU would take;
* fp16 scores that sit so close to an fp16 rounding boundary that another fp32 summation order could
  round them the other way (relative distance < FRAGILE), and whether flipping all of them changes the
  auction's result (if not, the step is order-robust);
* near ties of the min-loss nearest-centre count and of the final predict (fp64 relative gap < 1e-6).

A fixture is usable when level 0, most parents, both candidate fits and most groups are clean.  Nothing
in the package or the GPU tests imports this file.
"""
from __future__ import annotations

import sys
from pathlib import Path

import numpy as np
import torch

HERE = Path(__file__).resolve().parent
sys.path.insert(0, str(HERE.parent.parent))
sys.path.insert(0, str(HERE))
import make_golden as MG  # noqa: E402  (installs the reference harness)
from oracle import rq_oracle as O  # noqa: E402

ref_bk, ref_h, ref_s = MG.ref_bk, MG.ref_h, MG.ref_s
FRAGILE = 4e-6


def _fragile(d32: np.ndarray) -> np.ndarray:
    """entries whose fp16 rounding another summation order could flip (relative gap to the nearest fp16
    rounding midpoint below FRAGILE)"""
    h = d32.astype(np.float16).astype(np.float64)
    up = np.nextafter(d32.astype(np.float16), np.float16(np.inf)).astype(np.float64)
    dn = np.nextafter(d32.astype(np.float16), np.float16(-np.inf)).astype(np.float64)
    mid = np.minimum(np.abs(d32 - (h + up) / 2), np.abs(d32 - (h + dn) / 2))
    return mid < FRAGILE * np.abs(d32.astype(np.float64)) + 1e-30


class Recorder:
    """Tags every balanced fit of the reference and records each auction input (fp32 -D) under it."""

    def __init__(self):
        self.stack, self.fits, self.n = [], [], 0

    def install(self):
        rec = self
        orig_fit, orig_fbml, orig_auction = ref_bk.KMeans.fit, ref_bk.KMeans.fit_by_min_loss, ref_bk.auction_lap_half

        def fit(km, X, *a, **kw):
            rec.fits.append({"kind": "fit", "k": km.n_clusters, "n": len(X), "calls": []})
            rec.stack.append(rec.fits[-1])
            try:
                return orig_fit(km, X, *a, **kw)
            finally:
                rec.stack.pop()

        def fbml(km, X, *a, **kw):
            rec.fits.append({"kind": "fbml", "k": km.n_clusters, "n": len(X), "calls": []})
            rec.stack.append(rec.fits[-1])
            try:
                return orig_fbml(km, X, *a, **kw)
            finally:
                rec.stack.pop()

        def auction(s, *a, **kw):
            if rec.stack:
                rec.stack[-1]["calls"].append(s.detach().float().numpy().copy())
            return orig_auction(s, *a, **kw)

        ref_bk.KMeans.fit, ref_bk.KMeans.fit_by_min_loss, ref_bk.auction_lap_half = fit, fbml, auction
        self._orig = (orig_fit, orig_fbml, orig_auction)
        return self

    def remove(self):
        ref_bk.KMeans.fit, ref_bk.KMeans.fit_by_min_loss, ref_bk.auction_lap_half = self._orig


def analyze_fit(f: dict) -> dict:
    ties = fragile = flips_matter = 0
    for s in f["calls"]:
        n, k = s.shape
        if n < k:
            continue
        cert = O.auction_tie_certificate(s)
        if cert["diverged"]:  # a different bid set: does the result part too?
            ties += int(not np.array_equal(cert["torch"], cert["stable"]))
        fr = _fragile(-s.astype(np.float64))
        nf = int(fr.sum())
        fragile += nf
        if nf and np.array_equal(cert["torch"], cert["stable"]):
            s16 = s.astype(np.float16)
            alt = s16.copy()
            # move every fragile value one fp16 step toward its fp32 value's other side
            v = s.astype(np.float64)
            h = s16.astype(np.float64)
            toward = np.where(v > h, np.float16(np.inf), np.float16(-np.inf)).astype(np.float16)
            alt[fr] = np.nextafter(s16[fr], toward[fr])
            a0 = O.auction_lap_half(s16.astype(np.float32), tie_rule="stable")
            a1 = O.auction_lap_half(alt.astype(np.float32), tie_rule="stable")
            flips_matter += int(not np.array_equal(a0, a1))
    return {"kind": f["kind"], "k": f["k"], "n": f["n"], "calls": len(f["calls"]), "ties": ties,
            "fragile": fragile, "flips_matter": flips_matter,
            "clean": ties == 0 and flips_matter == 0}


def run_hierarchical(x: np.ndarray, cfg: dict, seed: int = 42):
    rec = Recorder().install()
    try:
        MG.seed_all(seed)
        m = ref_h.HierarchicalRQKMeans(ref_h.HierarchicalRQKMeansConfig(**cfg), device=torch.device("cpu"))
        tr = m.train(x, resume=False)
    finally:
        rec.remove()
    ids = np.stack([t.cpu().numpy() for t in tr["cluster_ids"]], 1).astype(np.int64)
    return m, ids, [analyze_fit(f) for f in rec.fits]


def run_simplified(x: np.ndarray, cfg: dict, seed: int = 42):
    import os
    import tempfile
    sids = [f"s{i:05d}" for i in range(len(x))]
    rec = Recorder().install()
    try:
        with tempfile.TemporaryDirectory() as td:
            p = os.path.join(td, "vec.csv")
            MG.write_csv(p, sids, x)
            MG.seed_all(seed)
            m = ref_s.SimplifiedHierarchicalRQ(ref_h.HierarchicalRQKMeansConfig(**cfg))
            m.train(p)
    finally:
        rec.remove()
    ids = np.array([m.semantic_ids[s] for s in sids], dtype=np.int64)
    return m, ids, [analyze_fit(f) for f in rec.fits]


def summary(fits):
    out = []
    for i, f in enumerate(fits):
        out.append(f"{i}:{f['kind']}k{f['k']}n{f['n']}{'' if f['clean'] else ' DIRTY(t%d,f%d)' % (f['ties'], f['flips_matter'])}")
    return out
