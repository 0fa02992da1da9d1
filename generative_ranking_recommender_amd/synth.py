"""Deterministic synthetic song-vector catalogues (SURVEY.md §8(d) "Synthetic inputs").

The reference's real input is the Word2Vec CSV written by
``src/common/train_word2vec.py:69-73`` (``song_id,v1..v512``, no header); the
dataset itself is private, so every test and benchmark here runs on a seeded
Gaussian mixture instead:

* ``M`` blob means ``~ N(0, I_D)`` drawn once from ``default_rng(seed)``;
* row block ``b`` draws its blob labels and noise from ``default_rng([seed, b])``,
  so any sharding of the catalogue across ranks sees identical global rows;
* ``x = mean[u] + sigma * N(0, I_D)``, fp32, row-major.

Well separated blobs keep the nearest-centre decision away from fp32 near-ties,
which is what lets the parity tests demand bit-identical IDs.
"""
from __future__ import annotations

import hashlib

import numpy as np

D_DEFAULT = 512
BLOCK_ROWS = 65536


def blob_means(m: int = 4096, d: int = D_DEFAULT, seed: int = 1234) -> np.ndarray:
    return np.random.default_rng(seed).standard_normal((m, d), dtype=np.float32)


def mixture_rows(start: int, stop: int, d: int = D_DEFAULT, m: int = 4096,
                 sigma: float = 0.25, seed: int = 1234,
                 means: np.ndarray | None = None) -> np.ndarray:
    """Rows ``[start, stop)`` of the global catalogue (block-deterministic)."""
    if means is None:
        means = blob_means(m, d, seed)
    out = np.empty((stop - start, d), dtype=np.float32)
    b0, b1 = start // BLOCK_ROWS, (stop - 1) // BLOCK_ROWS if stop > start else -1
    for b in range(b0, b1 + 1):
        rng = np.random.default_rng([seed, b])
        lab = rng.integers(0, m, size=BLOCK_ROWS)
        noise = rng.standard_normal((BLOCK_ROWS, d), dtype=np.float32)
        lo, hi = max(start, b * BLOCK_ROWS), min(stop, (b + 1) * BLOCK_ROWS)
        sl = slice(lo - b * BLOCK_ROWS, hi - b * BLOCK_ROWS)
        out[lo - start:hi - start] = means[lab[sl]] + np.float32(sigma) * noise[sl]
    return out


def small_mixture(n: int, d: int = D_DEFAULT, m: int = 64, sigma: float = 0.25,
                  seed: int = 7) -> np.ndarray:
    """Small one-shot catalogue for unit tests and golden fixtures."""
    rng = np.random.default_rng(seed)
    means = rng.standard_normal((m, d), dtype=np.float32)
    lab = rng.integers(0, m, size=n)
    return (means[lab] + np.float32(sigma) * rng.standard_normal((n, d), dtype=np.float32)).astype(np.float32)


def sha256(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def _normalize_rows(r: np.ndarray) -> np.ndarray:
    """r / (||r|| + 1e-8) in fp32, as ``hierarchical_rq_kmeans.py:1117-1122``."""
    n = np.sqrt((r.astype(np.float64) ** 2).sum(1, keepdims=True)).astype(np.float32)
    return (r / (n + np.float32(1e-8))).astype(np.float32)


def _nearest(x: np.ndarray, c: np.ndarray) -> np.ndarray:
    d = (c.astype(np.float64) ** 2).sum(1)[None, :] - 2.0 * (x.astype(np.float64) @ c.astype(np.float64).T)
    return d.argmin(1)


def encode_codebooks(seed: int = 99, need=(128, 128, 256), n_cand: int = 2560,
                     d: int = D_DEFAULT, pool_rows: int = BLOCK_ROWS) -> dict:
    """Residual-realistic 3-level codebooks of the PROD shape for encode tests/benchmarks.

    ``c0`` = ``need[0]`` catalogue rows (the reference initialises K-Means with data
    rows, ``balancekmeans/__init__.py:240-256``); ``c1`` = per-parent blocks of
    ``need[1]`` normalised level-1 residuals of rows that fall in that parent;
    ``c2`` = ``n_cand`` normalised level-2 residuals; ``match`` = ``need[0]*need[1]``
    rows with exactly ``need[2]`` ones among ``n_cand`` columns (the shape of
    ``_assign_last_match_matrix``, ``hierarchical_rq_kmeans.py:968-1053``).
    Each level samples its own independent pool of rows, so no centre is the
    residual of a row that produced a centre one level up (that would be an exact
    zero vector, duplicated across groups).
    """
    rng = np.random.default_rng(seed)
    base = 1 << 30
    pool0 = mixture_rows(base, base + pool_rows, d=d)
    pool1 = mixture_rows(base + pool_rows, base + 2 * pool_rows, d=d)
    pool2 = mixture_rows(base + 2 * pool_rows, base + 3 * pool_rows, d=d)
    c0 = pool0[rng.choice(pool_rows, need[0], replace=False)].copy()
    a1 = _nearest(pool1, c0)
    r1 = _normalize_rows(pool1 - c0[a1])
    c1 = np.empty((need[0] * need[1], d), dtype=np.float32)
    for p in range(need[0]):
        members = np.nonzero(a1 == p)[0]
        if len(members) == 0:
            members = np.arange(pool_rows)
        pick = rng.choice(members, need[1], replace=len(members) < need[1])
        c1[p * need[1]:(p + 1) * need[1]] = r1[pick]
    a2 = _nearest(pool2, c0)
    r21 = _normalize_rows(pool2 - c0[a2])
    g1 = np.empty(pool_rows, dtype=np.int64)
    for p in range(need[0]):
        members = np.nonzero(a2 == p)[0]
        if len(members):
            g1[members] = p * need[1] + _nearest(r21[members], c1[p * need[1]:(p + 1) * need[1]])
    r2 = _normalize_rows(r21 - c1[g1])
    c2 = r2[rng.choice(pool_rows, n_cand, replace=False)].copy()
    groups = need[0] * need[1]
    match = np.zeros((groups, n_cand), dtype=np.uint8)
    cols = np.argsort(rng.random((groups, n_cand), dtype=np.float32), axis=1)[:, :need[2]]
    np.put_along_axis(match, cols, 1, axis=1)
    return {"c0": c0, "c1": c1, "c2": c2, "match": match}


def codebooks_sha(cb: dict) -> str:
    h = hashlib.sha256()
    for k in ("c0", "c1", "c2", "match"):
        h.update(np.ascontiguousarray(cb[k]).tobytes())
    return h.hexdigest()


def tree_mixture(labels: np.ndarray, fan0: int, fan1: int, n_leaf: int, d: int = D_DEFAULT,
                 scales=(4.0, 1.0, 0.2), noise: float = 0.01, seed: int = 0) -> np.ndarray:
    """A 3-level tree of blobs for training-parity fixtures: row i with labels (a, b, c) is
    ``A[a] + B[a, b] + C[c] + noise`` with |A| >> |B| >> |C| >> noise, so level 0 of a residual K-Means
    separates a, its level-1 residuals (x - mean_a, normalised) separate b inside each parent, and the
    level-2 residuals separate the GLOBAL leaf direction c.  B sums to zero over b for every a and C over
    c, so the blob means are the tree's nodes.  Directions are Gaussian (random, nearly orthogonal at
    D = 512), each offset scaled to its level's norm; float32."""
    rng = np.random.default_rng(seed)

    def dirs(k, scale):
        v = rng.standard_normal((k, d))
        return v / np.linalg.norm(v, axis=1, keepdims=True) * scale

    a_ = dirs(fan0, scales[0])
    b_ = dirs(fan0 * fan1, scales[1]).reshape(fan0, fan1, d)
    b_ -= b_.mean(1, keepdims=True)
    c_ = dirs(n_leaf, scales[2])
    c_ -= c_.mean(0, keepdims=True)
    lab = np.asarray(labels, dtype=np.int64)
    e = rng.standard_normal((len(lab), d)) * (noise / np.sqrt(d))
    x = a_[lab[:, 0]] + b_[lab[:, 0], lab[:, 1]] + c_[lab[:, 2]] + e
    return x.astype(np.float32)
