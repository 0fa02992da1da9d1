#!/usr/bin/env python3
"""Differential test (GPU): v_mfma_f32_32x32x16_f16 against bit-exact software models of its
accumulation, on random inputs built to expose alignment/truncation (wide exponent spreads,
cancellation, subnormals).  Used to pin the accumulation-error model behind the screen's bound
(assign.hip accumulation_rel).  Exact arithmetic on Python integers in units of 2^-48.

Models: D = RNE_f32(C + T), T = sum over groups of floor_to(res, group sum), where the 16 products
are summed exactly in groups of G consecutive k, and every group sum is floored (toward -inf) or
truncated (toward 0) to a resolution of 2^(e - m) with 2^e <= max |group sum| < 2^(e+1)."""
import os
import sys
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from generative_ranking_recommender_amd import _lib  # noqa: E402

DEV = torch.device("cuda", 0)


def f16_int(bits):
    """fp16 bits -> exact integer in units of 2^-24."""
    s, e, m = (bits >> 15) & 1, (bits >> 10) & 31, bits & 1023
    v = m if e == 0 else (1024 + m) << (e - 1)
    return -v if s else v


def f32_int48(x):
    """fp32 value that is a multiple of 2^-48 -> integer in units of 2^-48."""
    num, den = float(x).as_integer_ratio()
    assert (1 << 48) % den == 0, "C not a multiple of 2^-48"
    return num * ((1 << 48) // den)


def rne_f32_from48(x):
    if x == 0:
        return 0.0
    ax = abs(x)
    bl = ax.bit_length()
    if bl > 24:
        sh = bl - 24
        q = ax >> sh
        r = ax - (q << sh)
        half = 1 << (sh - 1)
        if r > half or (r == half and (q & 1)):
            q += 1
        val = float(q) * 2.0 ** (sh - 48)
    else:
        val = float(ax) * 2.0 ** -48
    return np.float32(-val if x < 0 else val)


def model(products, c48, group, m, floor=True):
    gs = [sum(products[i:i + group]) for i in range(0, 16, group)]
    M = max(abs(g) for g in gs)
    if M:
        sh = M.bit_length() - 1 - m
        if sh > 0:
            if floor:
                gs = [(g >> sh) << sh for g in gs]
            else:
                gs = [(abs(g) >> sh << sh) * (1 if g >= 0 else -1) for g in gs]
    return rne_f32_from48(c48 + sum(gs))


MODELS = {f"G{g}_m{m}_{'floor' if fl else 'trunc'}": (g, m, fl)
          for g in (4, 8, 16) for m in (21, 22, 23, 24) for fl in (True, False)}


def gen(kind, rng):
    """A [32,16], B [16,32] fp16 bits; C [32,32] fp32 (multiples of 2^-48)."""
    if kind == "gauss":
        a = rng.standard_normal((32, 16)).astype(np.float16)
        b = (rng.standard_normal((16, 32)) * 0.05).astype(np.float16)
        c = (rng.standard_normal((32, 32)) * 2.0 ** rng.integers(-6, 4, (32, 32))).astype(np.float32)
    elif kind == "wide":
        a = ((1 + rng.integers(0, 1024, (32, 16)) / 1024) * 2.0 ** rng.integers(-12, 15, (32, 16)) *
             rng.choice([-1, 1], (32, 16))).astype(np.float16)
        b = ((1 + rng.integers(0, 1024, (16, 32)) / 1024) * 2.0 ** rng.integers(-12, 15, (16, 32)) *
             rng.choice([-1, 1], (16, 32))).astype(np.float16)
        c = (rng.standard_normal((32, 32)) * 2.0 ** rng.integers(-10, 25, (32, 32))).astype(np.float32)
    elif kind == "cancel":
        a = ((1 + rng.integers(0, 1024, (32, 16)) / 1024) * 2.0 ** rng.integers(-4, 12, (32, 16))).astype(np.float16)
        a[:, 8:] = -a[:, :8] * (rng.random((32, 8)) < 0.5) + a[:, 8:] * (rng.random((32, 8)) >= 0.5)
        b = ((1 + rng.integers(0, 1024, (16, 32)) / 1024) * 2.0 ** rng.integers(-4, 12, (16, 32))).astype(np.float16)
        b[8:] = b[:8]
        c = (rng.standard_normal((32, 32)) * 2.0 ** rng.integers(-4, 20, (32, 32))).astype(np.float32)
        c[rng.random((32, 32)) < 0.3] = 0
    else:  # subnormal
        a = (rng.standard_normal((32, 16)) * 2.0 ** rng.integers(-24, 0, (32, 16))).astype(np.float16)
        b = (rng.standard_normal((16, 32)) * 2.0 ** rng.integers(-24, 4, (16, 32))).astype(np.float16)
        c = (rng.standard_normal((32, 32)) * 2.0 ** rng.integers(-20, 0, (32, 32))).astype(np.float32)
    # C as a multiple of 2^-48
    c = np.where(np.abs(c) < 2.0 ** -24, 0, c).astype(np.float32)
    return a.view(np.uint16), b.view(np.uint16), c


def probe(lib, a, b, c):
    stream = torch.cuda.current_stream().cuda_stream
    ta = torch.from_numpy(a.view(np.int16).copy()).to(DEV)
    tb = torch.from_numpy(b.view(np.int16).copy()).to(DEV)
    tc = torch.from_numpy(np.ascontiguousarray(c, dtype=np.float32)).to(DEV)
    td = torch.empty((32, 32), dtype=torch.float32, device=DEV)
    _lib.check(lib.rqsid_mfma_probe(1, ta.data_ptr(), tb.data_ptr(), tc.data_ptr(), td.data_ptr(), stream), "p")
    torch.cuda.synchronize()
    return td.cpu().numpy()


def explain(lib, a, b, c, i, j):
    """Print one output's products and the hardware result, then re-probe with single products
    removed to see which ones the hardware drops."""
    af = a.view(np.float16).astype(np.float64)
    bf = b.view(np.float16).astype(np.float64)
    prods = af[i] * bf[:, j]
    d = probe(lib, a, b, c)[i, j]
    exact = float(c[i, j]) + prods.sum()
    print(f"  C={float(c[i, j]):.6e} D={float(d):.9e} exact={exact:.9e} err={float(d) - exact:.3e}")
    print("  a=" + " ".join(f"{x:.3e}" for x in af[i]))
    print("  b=" + " ".join(f"{x:.3e}" for x in bf[:, j]))
    print("  p=" + " ".join(f"{x:.3e}" for x in prods))


def main(cases=int(os.environ.get("MFMA_CASES", 40)), seed=0):
    lib = _lib.load()
    rng = np.random.default_rng(seed)
    stream = torch.cuda.current_stream().cuda_stream
    for kind in ("gauss", "wide", "cancel", "subnormal"):
        hits = {k: 0 for k in MODELS}
        total = 0
        worst = 0.0
        worst_case = None
        for _ in range(cases):
            a, b, c = gen(kind, rng)
            ta = torch.from_numpy(a.view(np.int16).copy()).to(DEV)
            tb = torch.from_numpy(b.view(np.int16).copy()).to(DEV)
            tc = torch.from_numpy(c).to(DEV)
            td = torch.empty((32, 32), dtype=torch.float32, device=DEV)
            _lib.check(lib.rqsid_mfma_probe(1, ta.data_ptr(), tb.data_ptr(), tc.data_ptr(), td.data_ptr(), stream), "p")
            torch.cuda.synchronize()
            d = td.cpu().numpy()
            ai = [[f16_int(int(a[i, k])) for k in range(16)] for i in range(32)]
            bi = [[f16_int(int(b[k, j])) for j in range(32)] for k in range(16)]
            for i in range(32):
                for j in range(32):
                    p = [ai[i][k] * bi[k][j] for k in range(16)]
                    c48 = f32_int48(c[i, j])
                    exact = c48 + sum(p)
                    sp = sum(abs(x) for x in p) + abs(c48)
                    if sp:
                        err = abs(float(d[i, j]) * 2.0 ** 48 - exact) / sp
                        if err > worst:
                            worst = err
                            worst_case = (a.copy(), b.copy(), c.copy(), i, j)
                    for name, (g, m, fl) in MODELS.items():
                        if model(p, c48, g, m, fl) == d[i, j]:
                            hits[name] += 1
                    total += 1
        best = sorted(hits.items(), key=lambda kv: -kv[1])[:6]
        print(f"{kind}: {total} outputs; worst |D - exact| / (sum|p| + |C|) = {worst:.3e} "
              f"({worst / 2.0 ** -23:.2f} x 2^-23); best models: " +
              ", ".join(f"{k}={v / total:.5f}" for k, v in best), flush=True)
        if worst_case is not None:
            explain(lib, *worst_case)


if __name__ == "__main__" and not (os.environ.get("MFMA_SWEEP") or os.environ.get("MFMA_ANCHOR") or os.environ.get("MFMA_TRUNC")):
    main()


def sweep(lib, seed=1):
    """Max |D - exact| in units of the product scale 2^k, over random same-scale products (and C of the
    same scale), for products built from normal fp16 inputs and from inputs with one subnormal side."""
    rng = np.random.default_rng(seed)
    for sub in (False, True):
        for k in range(4, -50, -4):
            worst, worst_rel = 0.0, 0.0
            for _ in range(4):
                if sub:   # a subnormal (2^-15 .. 2^-24), b picks up the rest of the scale
                    ea = rng.integers(-24, -14, (32, 16))
                else:
                    ea = np.full((32, 16), k // 2)
                eb = k - ea[:, :1].repeat(32, 1).T[:16]  # per-column exponent so products ~ 2^k
                a = (rng.uniform(0.5, 1, (32, 16)) * rng.choice([-1, 1], (32, 16)) * 2.0 ** ea).astype(np.float16)
                b = (rng.uniform(0.5, 1, (16, 32)) * rng.choice([-1, 1], (16, 32)) *
                     2.0 ** np.clip(eb, -24, 15)).astype(np.float16)
                c = (rng.uniform(-1, 1, (32, 32)) * 2.0 ** (k + 2)).astype(np.float32)
                c = np.where(np.abs(c) < 2.0 ** -48 * 2 ** 23, 0, c).astype(np.float32)
                d = probe(lib, a.view(np.uint16), b.view(np.uint16), c).astype(np.float64)
                af = a.astype(np.float64)
                bf = b.astype(np.float64)
                p = af[:, :, None] * bf[None, :, :]              # [32,16,32] exact in fp64
                exact = c.astype(np.float64) + p.sum(1)           # fp64 rounding << fp32 ulp here
                scale = np.abs(p).sum(1) + np.abs(c)
                err = np.abs(d - exact)
                ok = scale > 0
                worst = max(worst, float((err[ok]).max()))
                worst_rel = max(worst_rel, float((err[ok] / scale[ok]).max()))
            print(f"sub={sub} k={k:4d}: max abs err {worst:.3e} (2^{np.log2(worst) if worst else -999:.1f}), "
                  f"max err/(sum|p|+|C|) {worst_rel / 2.0 ** -23:.2f} x 2^-23", flush=True)


if __name__ == "__main__" and os.environ.get("MFMA_SWEEP"):
    sweep(_lib.load())


def anchor_probe(lib):
    """Does a zero / subnormal fp16 input anchor the alignment window at its NOMINAL exponent (-14)?
    Row 0 of every case: product 0 = a0 * 2^10, products 1..15 = 2^-20 (1 + j/1024) (bits down to
    2^-30).  a0 = 0, the smallest subnormal 2^-24, 2^-20, 2^-15 (subnormal), 2^-14 (normal), or an
    ordinary small normal value for reference."""
    for name, a0 in (("zero", 0.0), ("sub 2^-24", 2.0 ** -24), ("sub 2^-20", 2.0 ** -20), ("sub 2^-15", 2.0 ** -15),
                     ("normal 2^-14", 2.0 ** -14), ("normal 2^-12", 2.0 ** -12), ("none (a0 b0 = 0 via b)", None)):
        a = np.zeros((32, 16), np.float32)
        b = np.zeros((16, 32), np.float32)
        rng = np.random.default_rng(7)
        a[:, 1:] = 2.0 ** -10 * (1 + rng.integers(0, 1024, (32, 15)) / 1024)
        b[1:, :] = 2.0 ** -10
        if a0 is None:
            a[:, 0] = 1.0
            b[0, :] = 0.0
        else:
            a[:, 0] = a0
            b[0, :] = 2.0 ** 10
        a16 = a.astype(np.float16)
        b16 = b.astype(np.float16)
        assert (a16.astype(np.float32) == a).all() and (b16.astype(np.float32) == b).all()
        c = np.zeros((32, 32), np.float32)
        d = probe(lib, a16.view(np.uint16), b16.view(np.uint16), c).astype(np.float64)
        exact = a16.astype(np.float64) @ b16.astype(np.float64)
        err = np.abs(d - exact).max()
        print(f"anchor {name:>24}: max |D - exact| = {err:.3e} (2^{np.log2(err) if err else -999:.1f}); "
              f"products ~2^-20, true product 0 = {0 if a0 is None else a0 * 2 ** 10:.3e}", flush=True)


if __name__ == "__main__" and os.environ.get("MFMA_ANCHOR"):
    anchor_probe(_lib.load())


def truncation_probe(lib, seed=3, trials=64):
    """Worst truncation of the 16-product sum, in units of 2^-23 max|p|, after allowing the final
    round-to-nearest (2^-24 |D|): one anchor product and 15 products 2^-k (k = 1..26) below it whose
    low mantissa bits are all ones (the most a truncating aligner can drop), in every position."""
    rng = np.random.default_rng(seed)
    worst = 0.0
    for trial in range(trials):
        a = np.zeros((32, 16), np.float32)
        b = np.zeros((16, 32), np.float32)
        pos = rng.integers(0, 16, 32)                    # anchor position per row
        for i in range(32):
            for k in range(16):
                if k == pos[i]:
                    a[i, k] = (1 + rng.integers(0, 1024) / 1024) * rng.choice([-1, 1])
                else:
                    e = -int(rng.integers(1, 27))
                    mant = 2047 if rng.random() < 0.7 else int(rng.integers(1024, 2048))
                    a[i, k] = mant / 1024 * 2.0 ** e * (rng.choice([-1, 1]) if trial % 2 else 1)
        b[:, :] = (1 + rng.integers(0, 1024, (16, 32)) / 1024) * (1 if trial % 4 < 2 else rng.choice([-1, 1], (16, 32)))
        a16 = a.astype(np.float16)
        b16 = b.astype(np.float16)
        a16[np.abs(a16.astype(np.float32)) < 2.0 ** -14] = 0  # no subnormal operands (as the screen)
        c = np.zeros((32, 32), np.float32)
        d = probe(lib, a16.view(np.uint16), b16.view(np.uint16), c).astype(np.float64)
        p = a16.astype(np.float64)[:, :, None] * b16.astype(np.float64)[None, :, :]
        exact = p.sum(1)                                   # fp64: exact enough (span < 53 bits)
        pmax = np.abs(p).max(1)
        err = np.maximum(np.abs(d - exact) - 2.0 ** -24 * np.abs(d), 0)
        worst = max(worst, float((err / (2.0 ** -23 * pmax)).max()))
    print(f"truncation probe: worst (|D - sum p| - 2^-24 |D|) / (2^-23 max|p|) = {worst:.3f}", flush=True)
    return worst


if __name__ == "__main__" and os.environ.get("MFMA_TRUNC"):
    truncation_probe(_lib.load())
