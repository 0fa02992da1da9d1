"""BASELINE configs[2] at its own size: 10M x 512 fp32 rows, PROD codebook shapes.

At 10M rows the row offsets pass 2^31 elements (rows above 4,194,303), so every kernel that indexes x, the
re-score and the bucketing run their 64-bit paths.  Checks: IDs in range at every level; two encodes of the
same rows give identical IDs (determinism); the default dispatch (producer/consumer screen at level 2) and
the per-tile screens everywhere give identical IDs on ALL rows; and an evenly spaced 2048-row sample, half
of it above row 4.19M, is bit-identical to the exact CPU oracle."""
import numpy as np
import pytest
import torch

from generative_ranking_recommender_amd import synth
from generative_ranking_recommender_amd.encode import HIERARCHICAL_TRAIN, RQEncoder
from oracle import rq_oracle as O

pytestmark = pytest.mark.gpu

N = 10_000_000
NEED = [128, 128, 256]
BIG = (1 << 31) // 512  # first row whose element offset is >= 2^31


def _rows(n, dev):
    """The bench's row distribution (Gaussian mixture of synth.blob_means), generated on the device."""
    g = torch.Generator(device=dev).manual_seed(77)
    means = torch.from_numpy(synth.blob_means()).to(dev)
    x = torch.empty((n, 512), dtype=torch.float32, device=dev)
    step = 1 << 20
    for i in range(0, n, step):
        m = min(step, n - i)
        lab = torch.randint(0, means.shape[0], (m,), device=dev, generator=g)
        x[i:i + m] = means[lab] + 0.25 * torch.randn((m, 512), device=dev, generator=g)
    return x


def test_configs2_full_size_encode():
    import os
    dev = torch.device("cuda", 0)
    cb = synth.encode_codebooks(seed=99)
    enc = RQEncoder([torch.from_numpy(cb[k]) for k in ("c0", "c1", "c2")], NEED,
                    match=torch.from_numpy(cb["match"]), semantics=HIERARCHICAL_TRAIN, device=dev)
    x = _rows(N, dev)
    a = enc.encode(x).clone()
    b = enc.encode(x)
    assert torch.equal(a, b), "two encodes of the same rows differ"
    for lvl, k in enumerate(NEED):
        col = a[:, lvl]
        assert int(col.min()) >= 0 and int(col.max()) < k, f"level {lvl} ids out of range"
    old = os.environ.get("RQSID_SCREEN_VARIANT")
    os.environ["RQSID_SCREEN_VARIANT"] = "1"  # the per-tile screens on every level
    try:
        c = enc.encode(x)
    finally:
        if old is None:
            del os.environ["RQSID_SCREEN_VARIANT"]
        else:
            os.environ["RQSID_SCREEN_VARIANT"] = old
    diff = int((a != c).any(1).sum())
    assert diff == 0, f"{diff} rows differ between the default dispatch and the per-tile screens"
    sel = np.unique(np.concatenate([np.linspace(0, BIG - 1, 1024), np.linspace(BIG, N - 1, 1024)]).astype(np.int64))
    assert (sel >= BIG).sum() >= 1000
    xs = x[torch.from_numpy(sel).to(dev)].cpu().numpy()
    ref = O.encode(xs, [cb["c0"], cb["c1"], cb["c2"]], NEED, cb["match"], residual_from_weighted=True, exact=True)
    got = a[torch.from_numpy(sel).to(dev)].cpu().numpy()
    bad = np.nonzero((got != ref).any(1))[0]
    assert len(bad) == 0, f"{len(bad)} of {len(sel)} sampled rows differ from the exact oracle (rows {sel[bad[:5]]})"
    assert enc.error_words() and all(int(w.item()) == 0 for w in enc.error_words())
