#!/usr/bin/env python3
"""Diagnostics (GPU): distribution of the exact top-2 distance gap per encode level on the bench
workload, relative to |v| |c_best| (the scale of the screen's error bound).  Tells what fraction of
rows a screen with a given relative error bound would leave ambiguous.  Plain torch fp64, no rqsid."""
import os
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import bench  # noqa: E402

THR = [3e-3, 1.4e-3, 7e-4, 3e-4, 1e-4, 3e-5, 1e-5, 3e-6, 1e-6]


def level_gaps(v, c, allowed=None):
    """v [n,d] fp32, c [k,d] fp32, allowed [n,k] bool or None -> (best idx, gap/(|v||c_best|))."""
    vd, cd = v.double(), c.double()
    d = (vd * vd).sum(1, keepdim=True) - 2.0 * vd @ cd.T + (cd * cd).sum(1)[None, :]
    if allowed is not None:
        d = torch.where(allowed, d, torch.full_like(d, float("inf")))
    top = torch.topk(d, 2, dim=1, largest=False)
    scale = vd.norm(dim=1) * cd.norm(dim=1)[top.indices[:, 0]]
    return top.indices[:, 0], (top.values[:, 1] - top.values[:, 0]) / scale.clamp(min=1e-30)


ACC = (16 + (512 // 16) / 2 + 1) * 2.0 ** -23 * 1.02  # assign.hip accumulation_rel
MODES = {"1term": (1, 1, 1), "xsplit": (0, 1, 1), "3term": (0, 0, 1), "3term_acc/4": (0, 0, 0.25)}


def emulated_ambiguous(v_pre, c, allowed=None):
    """Fraction of rows a screen cannot decide, per bound model (assign.hip, per-candidate form):
    sc_k = |c_k|^2 - 2/den (vh.ch) (fp64 of the fp16 products), e_k = A |c_k| + B |ec_k| with
    A = 2/den (fx |ex| + fa acc |vh|), B = 2/den fc |vh|; ambiguous if another candidate's sc - e is
    <= min(sc + e).  fx/fc/fa switch the x-rounding / centre-rounding / accumulation terms."""
    vd = v_pre.double()
    den = vd.norm(dim=1)
    vh = v_pre.half().double()
    ch = c.half().double()
    cd = c.double()
    ex = (vd - vh).norm(dim=1)
    ec = (cd - ch).norm(dim=1)
    hn = den + ex
    out = {}
    for name, (fx, fc, fa) in MODES.items():
        if name == "1term":
            dot = vh @ ch.T
        elif name == "xsplit":
            dot = vd @ ch.T
        else:
            dot = vd @ cd.T
        sc = (cd * cd).sum(1)[None, :] - 2.0 * dot / den[:, None]
        A = 2.0 / den * (fx * ex + fa * ACC * hn)
        B = 2.0 / den * hn * fc
        e = A[:, None] * cd.norm(dim=1)[None, :] + B[:, None] * ec[None, :]
        ub, lb = sc + e, sc - e
        if allowed is not None:
            ub = torch.where(allowed, ub, torch.full_like(ub, float("inf")))
            lb = torch.where(allowed, lb, torch.full_like(lb, float("inf")))
        U = ub.min(1, keepdim=True).values
        out[name] = ((lb <= U).sum(1) > 1).double().sum().item()
        # loose epilogue: one per-row bound Emax = A max|c| + B max|ec| over the allowed set;
        # pass iff sc <= min sc + 2 Emax (the cheap count test), and the pass-count histogram
        cn = cd.norm(dim=1)[None, :].expand_as(sc)
        ecn = ec[None, :].expand_as(sc)
        if allowed is not None:
            cn = torch.where(allowed, cn, torch.zeros_like(cn))
            ecn = torch.where(allowed, ecn, torch.zeros_like(ecn))
            scm = torch.where(allowed, sc, torch.full_like(sc, float("inf")))
        else:
            scm = sc
        emax = A * cn.max(1).values + B * ecn.max(1).values
        npass = (scm <= scm.min(1).values[:, None] + 2.0 * emax[:, None]).sum(1)
        out[name + "_loose"] = (npass > 1).double().sum().item()
        out[name + "_loose_ovf8"] = (npass > 8).double().sum().item()
    return out


def normalize(r):
    return r / (r.norm(dim=1, keepdim=True) + 1e-8)


def main(n=int(os.environ.get("GAP_ROWS", 100_000))):
    dev = torch.device("cuda", 0)
    cache = os.environ.get("SWEEP_CB")
    if cache and os.path.exists(cache):
        import numpy as np
        z = np.load(cache)
        cb = {k: z[k] for k in z.files}
    else:
        cb = bench.codebooks(os.environ.get("BENCH_CODEBOOKS", "fitted"), dev)
    c0, c1, c2 = (torch.from_numpy(cb[k]).to(dev) for k in ("c0", "c1", "c2"))
    match = torch.from_numpy(cb["match"]).to(dev).bool()
    x = bench.make_rows(n, 0, dev)
    a0, g0 = level_gaps(x, c0)
    r1 = normalize(x - c0[a0])
    a1 = torch.empty(n, dtype=torch.long, device=dev)
    g1 = torch.empty(n, dtype=torch.float64, device=dev)
    for p in range(c0.shape[0]):
        m = a0 == p
        if m.any():
            i, g = level_gaps(r1[m], c1[p * 128:(p + 1) * 128])
            a1[m], g1[m] = i + p * 128, g
    r2 = normalize(r1 - c1[a1])
    a2, g2 = level_gaps(r2, c2, match[a1])
    keys = [k + suf for k in MODES for suf in ("", "_loose", "_loose_ovf8")]
    amb1 = {k: 0.0 for k in keys}
    for p in range(c0.shape[0]):
        m = a0 == p
        if m.any():
            for k, v in emulated_ambiguous(x[m] - c0[p], c1[p * 128:(p + 1) * 128]).items():
                amb1[k] += v
    amb0 = emulated_ambiguous(x, c0)
    amb2 = {k: 0.0 for k in keys}
    for i in range(0, n, 20000):
        for k, v in emulated_ambiguous(r1[i:i + 20000] - c1[a1[i:i + 20000]], c2, match[a1[i:i + 20000]]).items():
            amb2[k] += v
    for k in keys:
        print(f"emulated ambiguity [{k}]: L0 {amb0[k] / n:.4f} L1 {amb1[k] / n:.4f} L2 {amb2[k] / n:.4f}", flush=True)
    for lvl, g in enumerate((g0, g1, g2)):
        print(f"L{lvl}: median gap {g.median().item():.3e}  " +
              " ".join(f"<{t:.0e}:{(g < t).double().mean().item():.4f}" for t in THR), flush=True)


if __name__ == "__main__":
    main()
