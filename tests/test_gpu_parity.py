"""HIP kernels (through the C ABI) vs the CPU oracle and the reference's golden vectors.

Bar: integer IDs bit-identical to the oracle/reference; any row where they differ
must be a certified fp64 near tie (relative gap < 1e-6), and there are none on
these inputs.  Floating outputs: residuals within 1 ulp of the oracle (whose norm
is the correctly rounded one), centroids within 1e-5 relative.
"""
import numpy as np
import pytest
import torch

from generative_ranking_recommender_amd import ops, synth
from generative_ranking_recommender_amd.encode import (HIERARCHICAL_PREDICT_REFERENCE, HIERARCHICAL_TRAIN,
                                                       SIMPLIFIED, LevelSemantics, RQEncoder)
from oracle import rq_oracle as O
from tests import _data

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def gpu(a):
    return torch.from_numpy(np.ascontiguousarray(a)).to(DEV)


def assert_ids_equal_or_near_tie(x, c, got, ref):
    """got must be bit-identical to the oracle's exact argmin; against the fp32 (reference
    arithmetic) oracle every difference must be a certified near tie. Returns #near ties."""
    bad = np.nonzero(got != ref)[0]
    if len(bad):
        nt = O.near_tie(x[bad], c, got[bad], ref[bad])
        assert nt.all(), f"{(~nt).sum()} non-tie mismatches out of {len(got)}"
    return len(bad)


def exact_ids(x, c):
    return O.nearest(x, c, exact=True)


def test_nearest_golden(golden):
    g = golden("assign")
    x, c = _data.assign_inputs(g)
    got = ops.nearest(gpu(x), ops.prepare_centers(gpu(c))).cpu().numpy()
    assert (got == g["ids"]).all()


def test_nearest_ties_lowest_index(golden):
    g = golden("assign")
    x, c = _data.assign_inputs(g)
    x2, c2 = _data.tie_inputs(x, c)
    ws = ops.AssignWorkspace(len(x2), DEV)
    got = ops.nearest(gpu(x2), ops.prepare_centers(gpu(c2)), workspace=ws).cpu().numpy()
    assert (got == g["ids_tie"]).all()
    assert ws.rescored() >= 3  # exact duplicates can only be separated by the fp64 re-score


@pytest.mark.parametrize("n,k,d", [(1, 8, 512), (129, 128, 512), (5000, 100, 256), (20000, 256, 512),
                                   (3000, 1000, 64), (777, 2560, 512)])
def test_nearest_random(n, k, d):
    x = synth.small_mixture(n, d=d, m=50, seed=n + k)
    c = synth.small_mixture(k, d=d, m=50, seed=n + k + 1)
    got = ops.nearest(gpu(x), ops.prepare_centers(gpu(c))).cpu().numpy()
    assert (got == exact_ids(x, c)).all()
    assert_ids_equal_or_near_tie(x, c, got, O.nearest(x, c))


def test_nearest_forced_near_ties():
    """Rows exactly half-way between two centres and centres 1 ulp apart: the bf16 screen cannot
    separate them, the fp64 re-score must, with the lowest index winning exact ties."""
    rng = np.random.default_rng(3)
    c = rng.standard_normal((64, 512), dtype=np.float32)
    c[10] = c[3]
    c[11] = np.nextafter(c[4], np.float32(np.inf))
    x = np.concatenate([(c[3] + c[20]) / 2, (c[4] + c[5]) / 2, c[3], c[4], c[11]]).reshape(5, 512).astype(np.float32)
    x = np.concatenate([x, rng.standard_normal((300, 512), dtype=np.float32)])
    ws = ops.AssignWorkspace(len(x), DEV)
    got = ops.nearest(gpu(x), ops.prepare_centers(gpu(c)), workspace=ws).cpu().numpy()
    d2 = O.exact_d2(x, c)
    exact = d2.argmin(1)  # first index among exact ties
    assert (got == exact).all()
    assert got[2] == 3 and got[3] == 4 and got[4] == 11


@pytest.mark.parametrize("terms", [1, 3])
@pytest.mark.parametrize("xs,cs", [(1e-6, 1.0), (1.0, 1e-6), (1e-7, 1e-7), (3e3, 1.0), (1.0, 2e3)])
def test_nearest_extreme_scales(xs, cs, terms):
    """Rows / centres far from unit scale: their fp16 images are mostly subnormal (flushed: the
    MFMA would otherwise align products to the subnormal's nominal exponent) or near the fp16
    range; the table scale and the measured residuals keep the screen's bound rigorous."""
    rng = np.random.default_rng(int(xs * 1e3 + cs))
    c = (rng.standard_normal((128, 512)) * cs).astype(np.float32)
    c[64:] *= np.float32(1e-3)                   # mixed centre norms in one table
    x = (rng.standard_normal((3000, 512)) * xs).astype(np.float32)
    x[:1000] = c[rng.integers(0, 128, 1000)] + (0.05 * cs * rng.standard_normal((1000, 512))).astype(np.float32)
    got = ops.nearest(gpu(x), ops.prepare_centers(gpu(c)), screen_terms=terms).cpu().numpy()
    assert (got == exact_ids(x, c)).all()


def test_prepare_centers_table_scale():
    """c16 [k][dim/32][hi|lo][32]: hi = fp16(c 2^s) with the largest |hi| in [2^13, 2^14), lo = fp16((c 2^s - hi)
    2^12), no subnormals; meta rows {|c|^2, |c|, |2-term residual|, |1-term residual|}, row k = 2^-s."""
    rng = np.random.default_rng(5)
    c = (rng.standard_normal((300, 256)) * 3e-3).astype(np.float32)
    pc = ops.prepare_centers(gpu(c))
    meta = pc.meta.cpu().numpy()
    assert meta.shape == (301, 4)
    scale = float(meta[300, 0])
    assert np.log2(scale) == np.round(np.log2(scale))
    hl = pc.c16.cpu().numpy().view(np.float16).astype(np.float64)
    assert hl.shape == (300, 256 // 32, 2, 32)
    hi, lo = hl[:, :, 0, :].reshape(300, 256), hl[:, :, 1, :].reshape(300, 256)
    assert 2.0 ** 13 <= np.abs(hi).max() < 2.0 ** 14
    for t in (hi, lo):
        assert ((np.abs(t) >= 2.0 ** -14) | (t == 0)).all()
    c64 = c.astype(np.float64)
    r1 = np.sqrt(((c64 - hi * scale) ** 2).sum(1))
    r2 = np.sqrt(((c64 - (hi + lo * 2.0 ** -12) * scale) ** 2).sum(1))
    assert np.all(meta[:300, 3] >= r1) and np.allclose(meta[:300, 3], r1, rtol=1e-6)
    assert np.all(meta[:300, 2] >= r2) and np.allclose(meta[:300, 2], r2, rtol=1e-6)
    assert (r2 < r1 * 2.0 ** -9).all()
    assert np.allclose(meta[:300, 0], (c64 ** 2).sum(1), rtol=1e-6)


@pytest.mark.parametrize("terms", [1, 3])
@pytest.mark.parametrize("k", [100, 128, 200, 256])
def test_screen_terms_same_ids(terms, k):
    """1- and 3-term screens return the same exact IDs (only the re-scored fraction differs)."""
    x = synth.small_mixture(6000, d=512, m=40, seed=k)
    c = synth.small_mixture(k, d=512, m=40, seed=k + 1)
    ws = ops.AssignWorkspace(len(x), DEV)
    b = ops.single_segment(len(x), DEV)
    cand = ops.Candidates(torch.zeros(1, dtype=torch.int32, device=DEV),
                          torch.full((1,), k, dtype=torch.int32, device=DEV), k)
    got = ops.assign(gpu(x), ops.prepare_centers(gpu(c)), b, cand, workspace=ws, screen_terms=terms)[1]
    assert (got.cpu().numpy() == exact_ids(x, c)).all()


@pytest.mark.parametrize("gd,norm", [([512], True), ([128, 384], True), ([512], False), ([100, 12, 400], True)])
def test_residual(gd, norm):
    x = synth.small_mixture(3000, m=30, seed=4)
    c = synth.small_mixture(64, m=30, seed=5)
    ids = np.random.default_rng(0).integers(0, 64, 3000)
    got = ops.residual(gpu(x), gpu(c), gpu(ids.astype(np.int32)), gd, norm).cpu().numpy()
    ref = O.residual(x, c, ids, gd, norm)
    if not norm:
        assert np.array_equal(got, ref)
    else:
        ulp = np.abs(got.view(np.int32).astype(np.int64) - ref.view(np.int32).astype(np.int64))
        assert ulp.max() <= 1 and (ulp > 0).mean() < 1e-3


def test_residual_golden(golden):
    g = golden("residual")
    x, c = _data.residual_inputs()
    for tag, gd in (("g512", [512]), ("g128_384", [128, 384])):
        got = ops.residual(gpu(x), gpu(c), gpu(g["ids"].astype(np.int32)), gd, True).cpu().numpy()
        np.testing.assert_allclose(got[:256], g[f"res_{tag}_head"], rtol=3e-7, atol=1e-9)
    got = ops.residual(gpu(x), gpu(c), gpu(g["ids"].astype(np.int32)), [512], False).cpu().numpy()
    assert np.array_equal(got[:256], g["res_plain_head"])


# key counts of every bucketing form (csrc/rqsid.hip rqsid_bucket): LDS histograms (300 and 8192 with the count
# matrix off), the count matrix with one slice (128, 300, 8192, 16384), several and a ragged last slice (65536, 70001), and
# device-wide atomics (65536 with the matrix off); row counts below the matrix's chunk count and empty
@pytest.mark.parametrize("S,n,matrix", [(300, 100000, 1), (300, 100000, 0), (128, 3000, 1), (8192, 100000, 1), (8192, 100000, 0), (16384, 300000, 1),
                                        (65536, 1000000, 1), (65536, 1000000, 0), (70001, 500000, 1), (65536, 50, 1),
                                        (65536, 0, 1)])
def test_bucket_is_grouped_permutation(S, n, matrix, monkeypatch):
    monkeypatch.setenv("RQSID_BUCKET_MATRIX", str(matrix))
    keys = np.random.default_rng(S + n).integers(0, S, n).astype(np.int32)
    keys[:n // 20] = 7  # one big segment
    ws = ops.bucket_workspace(S, DEV)
    b = ops.bucket(gpu(keys), S, workspace=ws)
    off = b.seg_row_off.cpu().numpy()
    idx = b.row_index.cpu().numpy()
    assert off[0] == 0 and off[-1] == len(keys)
    assert np.array_equal(np.diff(off), np.bincount(keys, minlength=S))
    assert np.array_equal(np.sort(idx), np.arange(len(keys)))
    assert (keys[idx] == np.repeat(np.arange(S), np.diff(off))).all()
    toff = b.seg_tile_off.cpu().numpy()
    assert np.array_equal(np.diff(toff), (np.diff(off) + 127) // 128)
    assert int(ops.bucket_error_word(ws, S).item()) == 0


def test_segmented_assign_with_match_lists():
    rng = np.random.default_rng(9)
    n, k, groups = 30000, 640, 64
    x = synth.small_mixture(n, m=40, seed=8)
    c = synth.small_mixture(k, m=40, seed=9)
    match = np.zeros((groups, k), dtype=np.uint8)
    for gi in range(groups):
        match[gi, rng.choice(k, 200 if gi % 5 else 256, replace=False)] = 1
    seg = rng.integers(0, groups, n).astype(np.int32)
    cand = ops.match_to_candidates(gpu(match))
    b = ops.bucket(gpu(seg), groups)
    loc, glob = ops.assign(gpu(x), ops.prepare_centers(gpu(c)), b, cand)
    loc, glob = loc.cpu().numpy(), glob.cpu().numpy()
    allowed = O.match_allowed(match)
    assert (glob == O.segmented_nearest(x, c, seg, allowed, exact=True)).all()
    assert_ids_equal_or_near_tie(x, c, glob, O.segmented_nearest(x, c, seg, allowed))
    rank = np.cumsum(match, 1) - 1
    assert (loc == rank[seg, glob]).all()


def test_penalty_segment_matches_reference_rule():
    rng = np.random.default_rng(2)
    x = synth.small_mixture(500, m=10, seed=1)
    c = synth.small_mixture(96, m=10, seed=2)
    match = np.zeros((4, 96), dtype=np.uint8)
    match[0, :32] = 1
    match[2, 40:80] = 1  # groups 1 and 3 are empty -> +10000 everywhere
    seg = rng.integers(0, 4, 500).astype(np.int32)
    cand = ops.match_to_candidates(gpu(match))
    loc, glob = ops.assign(gpu(x), ops.prepare_centers(gpu(c)), ops.bucket(gpu(seg), 4), cand)
    glob = glob.cpu().numpy()
    assert (glob == O.segmented_nearest(x, c, seg, O.match_allowed(match), exact=True)).all()
    assert (loc.cpu().numpy()[np.isin(seg, [1, 3])] == -1).all()


def test_centroid_update_matches_oracle():
    x = synth.small_mixture(50000, m=20, seed=6)
    a = np.random.default_rng(4).integers(0, 96, 50000)
    a[a == 17] = 18  # an empty cluster keeps its previous centre
    prev = synth.small_mixture(96, m=20, seed=7)
    cen, cnt = ops.centroid_update(gpu(x), gpu(a.astype(np.int32)), 96, gpu(prev.copy()))
    cen = cen.cpu().numpy()
    ref = O.centroid_update(x, a, prev, lambda n: 0)
    mask = np.bincount(a, minlength=96) > 0
    np.testing.assert_allclose(cen[mask], ref[mask], rtol=1e-6, atol=1e-7)
    assert np.array_equal(cen[~mask], prev[~mask])
    assert np.array_equal(cnt.cpu().numpy(), np.bincount(a, minlength=96))


def test_pairwise_distance():
    x = synth.small_mixture(3000, m=30, seed=12)
    c = synth.small_mixture(100, m=30, seed=13)
    got = ops.pairwise_distance(gpu(x), gpu(c)).cpu().numpy().astype(np.float64)
    ref = np.sqrt(np.maximum(O.exact_d2(x, c), 0))
    scale = np.sqrt((x.astype(np.float64) ** 2).sum(1)[:, None] + (c.astype(np.float64) ** 2).sum(1)[None, :])
    assert (np.abs(got ** 2 - ref ** 2) <= 4e-6 * scale ** 2).all()


# --- multi-level encoder vs reference goldens ----------------------------------------
def _hier_encoder(g, sem, device=DEV):
    cents = [torch.from_numpy(g[k]) for k in ("c0", "c1", "c2")]
    return RQEncoder(cents, _data.SMALL_CFG["need_clusters"], match=torch.from_numpy(g["match"]), semantics=sem,
                     device=device)


def test_encoder_hierarchical_golden(golden):
    g = golden("hierarchical")
    x, xn = _data.small_rq_inputs(g)
    assert (_hier_encoder(g, HIERARCHICAL_TRAIN).encode(gpu(x)).cpu().numpy() == g["train_ids"]).all()
    assert (_hier_encoder(g, HIERARCHICAL_PREDICT_REFERENCE).encode(gpu(x)).cpu().numpy() == g["pred_bug"]).all()
    fix = LevelSemantics(residual_global_id=False)
    assert (_hier_encoder(g, fix).encode(gpu(x)).cpu().numpy() == g["pred_fix"]).all()
    assert (_hier_encoder(g, HIERARCHICAL_PREDICT_REFERENCE).encode(gpu(xn)).cpu().numpy()
            == g["pred_new_bug"]).all()
    if int(g["new_fix_keyerror"]) >= 0:
        with pytest.raises(KeyError) as e:
            _hier_encoder(g, fix).encode(gpu(xn))
        assert e.value.args[0] == int(g["new_fix_keyerror"])


def test_encoder_simplified_golden(golden):
    g = golden("simplified")
    x, _ = _data.small_rq_inputs(g)
    cents = [torch.from_numpy(g[k]) for k in ("l0_centers", "mid_centers", "final_centers")]
    enc = RQEncoder(cents, _data.SMALL_CFG["need_clusters"], match=torch.from_numpy(g["match"]), semantics=SIMPLIFIED,
                    device=DEV)
    assert (enc.encode(gpu(x)).cpu().numpy() == g["ids"]).all()


def test_encoder_prod_shapes_golden(golden):
    g = golden("encode_prod")
    x, cb = _data.prod_encode_inputs(g)
    cents = [torch.from_numpy(cb[k]) for k in ("c0", "c1", "c2")]
    m = torch.from_numpy(cb["match"])
    modes = {"pred_bug": HIERARCHICAL_PREDICT_REFERENCE, "pred_fix": LevelSemantics(residual_global_id=False),
             "pred_train": HIERARCHICAL_TRAIN}
    for key, sem in modes.items():
        got = RQEncoder(cents, [128, 128, 256], match=m, semantics=sem, device=DEV).encode(gpu(x)).cpu().numpy()
        bad = int((got != g[key]).any(1).sum())
        assert bad == 0, f"{key}: {bad} rows differ from the reference"


def test_encoder_full_size_properties():
    """1M rows at PROD codebook shapes: IDs in range, deterministic, and a 4096-row sample
    identical to the oracle (size-independent checks at the benchmark scale)."""
    cb = synth.encode_codebooks(seed=99)
    enc = RQEncoder([torch.from_numpy(cb[k]) for k in ("c0", "c1", "c2")], [128, 128, 256],
                    match=torch.from_numpy(cb["match"]), semantics=HIERARCHICAL_TRAIN, device=DEV)
    gen = torch.Generator(device=DEV).manual_seed(0)
    means = torch.from_numpy(synth.blob_means()).to(DEV)
    n = 1_000_000
    lab = torch.randint(0, means.shape[0], (n,), device=DEV, generator=gen)
    x = means[lab] + 0.25 * torch.randn((n, 512), device=DEV, generator=gen)
    a = enc.encode(x)
    b = enc.encode(x)
    assert torch.equal(a, b)
    an = a.cpu().numpy()
    assert an.min() >= 0 and (an.max(0) < np.array([128, 128, 256])).all()
    sel = np.random.default_rng(1).choice(n, 4096, replace=False)
    xs = x[torch.from_numpy(sel).to(DEV)].cpu().numpy()
    ref = O.encode(xs, [cb["c0"], cb["c1"], cb["c2"]], [128, 128, 256], cb["match"], residual_from_weighted=True,
                   exact=True)
    assert (an[sel] == ref).all()


@pytest.mark.parametrize("n", [0, 1, 2, 127, 128, 129, 255, 256, 257, 1023, 4097])
def test_encoder_empty_and_ragged_batches(n):
    """Batch sizes around the 128-row (levels 0/1) and 256-row (level 2 ping-pong) tile edges, one row and
    no rows, at PROD codebook shapes: every row's IDs equal the exact oracle's, in both the training and the
    reference-predict semantics; an empty batch gives an empty [0, 3] result."""
    cb = synth.encode_codebooks(seed=99)
    cents = [torch.from_numpy(cb[k]) for k in ("c0", "c1", "c2")]
    x = synth.mixture_rows(5, 5 + n) if n else np.zeros((0, 512), np.float32)
    for sem, weighted in ((HIERARCHICAL_TRAIN, True), (HIERARCHICAL_PREDICT_REFERENCE, None)):
        got = RQEncoder(cents, [128, 128, 256], match=torch.from_numpy(cb["match"]), semantics=sem,
                        device=DEV).encode(gpu(x)).cpu().numpy()
        assert got.shape == (n, 3)
        if not n:
            assert ops.nearest(gpu(x), ops.prepare_centers(gpu(cb["c0"]))).shape == (0,)
        if n and weighted:
            ref = O.encode(x, [cb["c0"], cb["c1"], cb["c2"]], [128, 128, 256], cb["match"],
                           residual_from_weighted=True, exact=True)
            assert (got == ref).all()
        if n:
            full = RQEncoder(cents, [128, 128, 256], match=torch.from_numpy(cb["match"]), semantics=sem,
                             device=DEV).encode(gpu(synth.mixture_rows(5, 5005))).cpu().numpy()
            assert (got == full[:n]).all()  # a row's IDs do not depend on the batch it is encoded in


def test_encoder_xl_shapes_properties():
    """BASELINE configs[4] shapes (need [256,256,512], 5120 last-level candidates, 65536 groups): the
    middle level screens 256 candidates per parent (1-term), the last level 512 per group (multi-pass
    screen).  IDs in range, deterministic, fused == materialised, and a row sample identical to the
    exact oracle."""
    need = (256, 256, 512)
    cb = synth.encode_codebooks(seed=5, need=need, n_cand=5120)
    enc = RQEncoder([torch.from_numpy(cb[k]) for k in ("c0", "c1", "c2")], list(need),
                    match=torch.from_numpy(cb["match"]), semantics=HIERARCHICAL_TRAIN, device=DEV)
    x = gpu(synth.mixture_rows(0, 200000))
    a = enc.encode(x)
    assert torch.equal(a, enc.encode(x))
    an = a.cpu().numpy()
    assert an.min() >= 0 and (an.max(0) < np.array(need)).all()
    enc.force_materialized = True
    assert torch.equal(a, enc.encode(x))
    sel = np.random.default_rng(2).choice(len(an), 2048, replace=False)
    ref = O.encode(x[torch.from_numpy(sel).to(DEV)].cpu().numpy(), [cb["c0"], cb["c1"], cb["c2"]], list(need),
                   cb["match"], residual_from_weighted=True, exact=True)
    assert (an[sel] == ref).all()


@pytest.mark.parametrize("sem_name", ["train", "predict_fix", "simplified"])
def test_fused_residuals_equal_materialized(sem_name):
    """The fused kernels (residual chain rebuilt inside rqsid_assign) must give the same IDs as
    materialised residual matrices + plain assignment.  (The reference-bug predict mode has an
    unconstrained last level and always runs materialised.)"""
    sem = {"train": HIERARCHICAL_TRAIN, "predict_fix": LevelSemantics(residual_global_id=False),
           "simplified": SIMPLIFIED}[sem_name]
    cb = synth.encode_codebooks(seed=99)
    x = gpu(synth.mixture_rows(0, 30000))
    enc = RQEncoder([torch.from_numpy(cb[k]) for k in ("c0", "c1", "c2")], [128, 128, 256],
                    match=torch.from_numpy(cb["match"]), semantics=sem, device=DEV)
    assert enc.fused
    a = enc.encode(x)
    enc.force_materialized = True
    b = enc.encode(x)
    assert torch.equal(a, b)


def test_last_level_group_out_of_range_raises():
    """need[0] > need[1]: the hierarchical before-id l0*need[0] + l1 can pass the need[0]*need[1] match
    rows; the reference raises IndexError at match_matrix_np[before] (hierarchical_rq_kmeans.py:1279-1281),
    and so must both encode paths (bucketing would silently drop the rows)."""
    need = (32, 16, 32)
    cb = synth.encode_codebooks(seed=7, need=need, n_cand=320, pool_rows=8192)
    x = gpu(synth.mixture_rows(0, 8000))
    enc = RQEncoder([torch.from_numpy(cb[k]) for k in ("c0", "c1", "c2")], list(need),
                    match=torch.from_numpy(cb["match"]), semantics=HIERARCHICAL_TRAIN, device=DEV)
    ids0 = O.nearest(synth.mixture_rows(0, 8000), cb["c0"])
    assert ids0.max() * need[0] + need[1] - 1 >= need[0] * need[1]  # the input does reach past the last group
    assert enc.fused
    with pytest.raises(IndexError):
        enc.encode(x)
    enc.force_materialized = True
    with pytest.raises(IndexError):
        enc.encode(x)


def test_multigroup_weighted_encode_vs_oracle():
    """group_dims [128, 384] with the reference's default weights 1/len(groups) (:56-62): the
    materialised path (scale_groups + per-group normalised residuals) vs the oracle."""
    cb = synth.encode_codebooks(seed=5, need=(16, 16, 32), n_cand=320, pool_rows=8192)
    x = synth.mixture_rows(0, 6000)
    gd, w = [128, 384], [[0.5, 0.5]] * 3
    enc = RQEncoder([torch.from_numpy(cb[k]) for k in ("c0", "c1", "c2")], [16, 16, 32],
                    match=torch.from_numpy(cb["match"]), group_dims=gd, weights=w, semantics=HIERARCHICAL_TRAIN,
                    device=DEV)
    assert not enc.fused
    got = enc.encode(gpu(x)).cpu().numpy()
    ref = O.encode(x, [cb["c0"], cb["c1"], cb["c2"]], [16, 16, 32], cb["match"], gd, w, residual_from_weighted=True,
                   exact=True)
    assert (got == ref).all()


def _with_env(env, fn):
    """Run fn with the kernel-selection environment variables in env (read by librqsid per call)."""
    import os
    old = {k: os.environ.get(k) for k in env}
    os.environ.update({k: str(v) for k, v in env.items()})
    try:
        return fn()
    finally:
        for k, v in old.items():
            if v is None:
                del os.environ[k]
            else:
                os.environ[k] = v


PER_TILE = {"RQSID_SCREEN_VARIANT": 1}
# the default dispatch (ping-pong form on 256-candidate levels) and every streamed form, forced
STREAMED = {"default": {"RQSID_SCREEN_VARIANT": 0},
            "s83": {"RQSID_SCREEN_VARIANT": 5, "RQSID_STREAM_SHAPE": 83},
            "s42": {"RQSID_SCREEN_VARIANT": 5, "RQSID_STREAM_SHAPE": 42},
            "pp88": {"RQSID_SCREEN_VARIANT": 5, "RQSID_STREAM_SHAPE": 88},
            "res": {"RQSID_SCREEN_VARIANT": 6},  # the centre-resident screen wherever it applies
            # the row-resident screen (assign_rows.hip) wherever it applies (1-term levels: L0 and L2 here)
            "rows443": {"RQSID_SCREEN_VARIANT": 8, "RQSID_ROWS_SHAPE": 443},
            "rows482": {"RQSID_SCREEN_VARIANT": 8, "RQSID_ROWS_SHAPE": 482},
            "rows883": {"RQSID_SCREEN_VARIANT": 8, "RQSID_ROWS_SHAPE": 883},
            # the producer/consumer screen (assign_pc.hip) on levels 1 and 2: wide (256-row) and 128-row forms
            "pc128": {"RQSID_SCREEN_VARIANT": 9},
            "pcw": {"RQSID_SCREEN_VARIANT": 9, "RQSID_PCW": 1}}


@pytest.mark.parametrize("form", list(STREAMED))
@pytest.mark.parametrize("shape", ["small", "prod"])
@pytest.mark.parametrize("sem_name", ["train", "simplified"])
def test_stream_kernel_equals_tile_kernel(shape, sem_name, form):
    """The persistent streamed screens (assign_stream.hip: 8x3, 4x2 and the ping-pong form) and the
    per-tile screen (assign.hip) return the exact argmin all: identical IDs on every level, with
    partial candidate lists (32 of a 128-wide tile), penalty-free match lists and both semantics;
    the streamed run is also checked row by row against the fp64 oracle on a sample."""
    sem = {"train": HIERARCHICAL_TRAIN, "simplified": SIMPLIFIED}[sem_name]
    if shape == "small":
        need, cb = (16, 16, 32), synth.encode_codebooks(seed=5, need=(16, 16, 32), n_cand=320, pool_rows=8192)
    else:
        need, cb = (128, 128, 256), synth.encode_codebooks(seed=99)
    xn = synth.mixture_rows(0, 40000)
    x = gpu(xn)
    enc = RQEncoder([torch.from_numpy(cb[k]) for k in ("c0", "c1", "c2")], list(need),
                    match=torch.from_numpy(cb["match"]), semantics=sem, device=DEV)
    a = _with_env(STREAMED[form], lambda: enc.encode(x).cpu().numpy())
    b = _with_env(PER_TILE, lambda: enc.encode(x).cpu().numpy())
    assert (a == b).all(), f"{int((a != b).any(1).sum())} rows differ between the streamed and per-tile screens"
    sel = np.arange(0, 40000, 37)
    ref = O.encode(xn[sel], [cb["c0"], cb["c1"], cb["c2"]], list(need), cb["match"],
                   normalize=sem.normalize_residual, remap_last=sem.remap_last,
                   last_group_mult=sem.last_group_mult, residual_from_weighted=True, exact=True) \
        if sem_name == "simplified" else \
        O.encode(xn[sel], [cb["c0"], cb["c1"], cb["c2"]], list(need), cb["match"], residual_from_weighted=True,
                 exact=True)
    assert (a[sel] == ref).all()


@pytest.mark.parametrize("form", ["default", "pc128", "pcw"])
def test_pc_screen_with_duplicate_centres(form):
    """Deduplicated candidate lists (ops.dedup_candidates: bitwise-identical centres of one list keep the first,
    the kept entries report their original local ids through cand_lid) through the producer/consumer screens:
    duplicated children inside level-1 parent blocks and duplicated level-2 centres.  IDs equal the per-tile
    screen's on every row and the exact oracle's on a sample (the reference's argmin takes the first equal
    centre, which is what the local ids must report)."""
    need, cb = (128, 128, 256), dict(synth.encode_codebooks(seed=99))
    c1, c2 = cb["c1"].copy(), cb["c2"].copy()
    for par in range(0, 128, 3):  # child 2 := child 9, child 40 := child 41 in every third parent
        c1[par * 128 + 2] = c1[par * 128 + 9]
        c1[par * 128 + 40] = c1[par * 128 + 41]
    c2[1:2560:5] = c2[0:2560:5]
    cb["c1"], cb["c2"] = c1, c2
    xn = synth.mixture_rows(7, 40000)
    x = gpu(xn)
    enc = RQEncoder([torch.from_numpy(cb[k]) for k in ("c0", "c1", "c2")], list(need),
                    match=torch.from_numpy(cb["match"]), semantics=HIERARCHICAL_TRAIN, device=DEV)
    assert all(c is not None and c.lid is not None for c in enc.cands[1:]), "the lists were not deduplicated"
    a = _with_env(STREAMED[form], lambda: enc.encode(x).cpu().numpy())
    b = _with_env(PER_TILE, lambda: enc.encode(x).cpu().numpy())
    assert (a == b).all(), f"{int((a != b).any(1).sum())} rows differ between the {form} and per-tile screens"
    sel = np.arange(0, 40000, 41)
    ref = O.encode(xn[sel], [cb["c0"], c1, c2], list(need), cb["match"], residual_from_weighted=True, exact=True)
    assert (a[sel] == ref).all()


@pytest.mark.parametrize("form", ["default", "s83", "pp88", "res", "rows443", "rows883"])
@pytest.mark.parametrize("k", [100, 128, 200, 256])
def test_stream_nearest_partial_tiles(k, form):
    """Single-segment nearest with k < NT*32 candidates (padding lanes masked) on the streamed path."""
    rng = np.random.default_rng(k)
    c = rng.standard_normal((k, 512)).astype(np.float32)
    x = (c[rng.integers(0, k, 30000)] + 0.3 * rng.standard_normal((30000, 512))).astype(np.float32)
    pc = ops.prepare_centers(gpu(c))
    got = _with_env(STREAMED[form], lambda: ops.nearest(gpu(x), pc).cpu().numpy())
    tile = _with_env(PER_TILE, lambda: ops.nearest(gpu(x), pc).cpu().numpy())
    assert (got == tile).all()
    sel = np.arange(0, 30000, 29)
    assert (got[sel] == exact_ids(x[sel], c)).all()


def test_integration_md_binding_runs():
    """The ctypes stub INTEGRATION.md shows a maintainer (KMeans.predict's argmin through the C ABI)
    runs against the built library and returns the exact argmin."""
    import re
    from pathlib import Path
    from generative_ranking_recommender_amd import _lib
    text = (Path(__file__).resolve().parent.parent / "INTEGRATION.md").read_text()
    code = re.search(r"```python\n(# balancekmeans/_rqsid.py.*?)```", text, re.S).group(1)
    code = code.replace('"/path/to/generative_ranking_recommender_amd/librqsid.so"', repr(str(_lib.LIB_PATH)))
    ns = {}
    exec(compile(code, "INTEGRATION.md", "exec"), ns)
    x = synth.small_mixture(3000, d=512, m=50, seed=5)
    c = synth.small_mixture(128, d=512, m=50, seed=6)
    got = ns["nearest_center"](torch.from_numpy(x), torch.from_numpy(c)).numpy()
    assert (got == exact_ids(x, c)).all()


def test_resident_spin_cap_fails_loudly():
    """a capped role wait of the centre-resident screen must not return wrong IDs
    silently.  RQSID_TEST_FORCE_SPIN_CAP gives the screen's final wait a zero cap (every other wait
    runs normally, so the forced path reads nothing out of order): the device error word is set and
    rqsid_assign fails with RQSID_E_LAUNCH -> RuntimeError.  Without it the same call succeeds."""
    rng = np.random.default_rng(3)
    c = rng.standard_normal((200, 512)).astype(np.float32)
    x = (c[rng.integers(0, 200, 30000)] + 0.3 * rng.standard_normal((30000, 512))).astype(np.float32)
    pc = ops.prepare_centers(gpu(c))
    with pytest.raises(RuntimeError, match="spin cap"):
        _with_env({"RQSID_SCREEN_VARIANT": 6, "RQSID_TEST_FORCE_SPIN_CAP": 1}, lambda: ops.nearest(gpu(x), pc))
    got = _with_env({"RQSID_SCREEN_VARIANT": 6, "RQSID_TEST_FORCE_SPIN_CAP": 0},
                    lambda: ops.nearest(gpu(x), pc).cpu().numpy())
    sel = np.arange(0, 30000, 29)
    assert (got[sel] == exact_ids(x[sel], c)).all()


MULTI_PASS = {"RQSID_SCREEN_VARIANT": 7}  # the multi-pass per-tile screen, no candidate split


@pytest.mark.parametrize("k,terms", [(257, 1), (384, 1), (512, 1), (129, 3), (200, 3), (256, 3)])
def test_candidate_split_nearest(k, terms):
    """Candidate-split single-pass screen (CW = 2: 512 1-term / 256 3-term candidates per segment):
    identical to the multi-pass screen and to the exact oracle, including partly padded candidate
    groups and duplicated centres (exact ties: lowest index)."""
    rng = np.random.default_rng(1000 + k + terms)
    c = rng.standard_normal((k, 512)).astype(np.float32)
    c[k - 1] = c[3]  # a duplicate in the second group: ties across the groups resolve to the lower index
    x = (c[rng.integers(0, k, 20000)] + 0.3 * rng.standard_normal((20000, 512))).astype(np.float32)
    x[:64] = c[3]    # rows sitting exactly on the duplicated centre
    pc = ops.prepare_centers(gpu(c))
    got = ops.nearest(gpu(x), pc, screen_terms=terms).cpu().numpy()
    multi = _with_env(MULTI_PASS, lambda: ops.nearest(gpu(x), pc, screen_terms=terms).cpu().numpy())
    assert (got == multi).all(), f"{int((got != multi).sum())} rows differ from the multi-pass screen"
    assert (got[:64] == 3).all()
    if terms == 1:  # the row-resident screen (candidate blocks with a running bound) on the same input
        for form in ("rows443", "rows883"):
            rows = _with_env(STREAMED[form], lambda: ops.nearest(gpu(x), pc, screen_terms=terms).cpu().numpy())
            assert (rows == got).all(), f"{form}: {int((rows != got).sum())} rows differ"
    sel = np.arange(0, 20000, 13)
    assert (got[sel] == exact_ids(x[sel], c)).all()


def test_candidate_split_xl_levels_equal_multi_pass():
    """XL shapes (need [256,256,512]): the middle level (256 3-term candidates per parent) and the last
    level (512 per group) take the candidate-split screen; every level's IDs equal the multi-pass
    screen's, and a sample equals the exact oracle."""
    need = (256, 256, 512)
    cb = synth.encode_codebooks(seed=5, need=need, n_cand=5120)
    enc = RQEncoder([torch.from_numpy(cb[k]) for k in ("c0", "c1", "c2")], list(need),
                    match=torch.from_numpy(cb["match"]), semantics=HIERARCHICAL_TRAIN, device=DEV)
    xn = synth.mixture_rows(3, 120000)
    x = gpu(xn)
    a = enc.encode(x).cpu().numpy()
    b = _with_env(MULTI_PASS, lambda: enc.encode(x).cpu().numpy())
    assert (a == b).all(), f"{int((a != b).any(1).sum())} rows differ between the split and multi-pass screens"
    for form in ("rows443", "rows883"):  # the row-resident screen at the 512-candidate last level
        c = _with_env(STREAMED[form], lambda: enc.encode(x).cpu().numpy())
        assert (c == a).all(), f"{form}: {int((c != a).any(1).sum())} rows differ"
    sel = np.arange(0, 120000, 97)
    ref = O.encode(xn[sel], [cb["c0"], cb["c1"], cb["c2"]], list(need), cb["match"], residual_from_weighted=True,
                   exact=True)
    assert (a[sel] == ref).all()


@pytest.mark.parametrize("k,dim", [(300, 512), (64, 256), (200, 1024)])
def test_rescore_two_rows_per_wave_equals_one(k, dim):
    """The two-rows-per-wave re-score (rows of <= 512 dims) and the one-row form return the same IDs on
    near-isotropic rows against many close centres (most rows listed, many overflowing to 'every
    candidate'), an odd number of work items included; both equal the exact oracle."""
    rng = np.random.default_rng(k + dim)
    c = (rng.standard_normal((k, dim)) * 0.05 + 1.0).astype(np.float32)
    x = (rng.standard_normal((4097, dim)) * 0.05 + 1.0).astype(np.float32)
    pc = ops.prepare_centers(gpu(c))
    ws = ops.AssignWorkspace(len(x), DEV)
    a = ops.nearest(gpu(x), pc, workspace=ws, screen_terms=1).cpu().numpy()
    assert ws.rescored() > 100
    b = _with_env({"RQSID_RESCORE_FULL": 1}, lambda: ops.nearest(gpu(x), pc, screen_terms=1).cpu().numpy())
    assert (a == b).all()
    sel = np.arange(0, len(x), 7)
    assert (a[sel] == exact_ids(x[sel], c)).all()


@pytest.mark.parametrize("k,dups", [(2560, 0), (1280, 0), (2560, 12)])
def test_rescreen_of_overflowing_rows_keeps_exact_ids(k, dups, monkeypatch):
    """The fp32 re-screen (assign.hip assign_rescreen_kernel, VERDICT r3 "re-score cliff"): diffuse unit
    rows against K = 1280 / 2560 unit centres (the training-time nearest of residual codebooks) leave most
    rows with more than 8 candidates inside the fp16 screen's bound.  With the re-screen those rows get an
    fp32 list first; the IDs equal the all-candidate fp64 pass (RQSID_NO_RESCREEN=1) and the exact oracle,
    also when 12 exact duplicates of one centre keep a true > 8-way tie overflowing (fp64 fallback, lowest
    index).  Times both forms (printed)."""
    import time
    rng = np.random.default_rng(k + dups)
    x = rng.standard_normal((30000, 512), dtype=np.float32)
    x /= np.linalg.norm(x, axis=1, keepdims=True)
    c = rng.standard_normal((k, 512), dtype=np.float32)
    c /= np.linalg.norm(c, axis=1, keepdims=True)
    if dups:
        c[100:100 + dups] = c[7]
        x[:500] = c[7] + np.float32(0.01) * rng.standard_normal((500, 512), dtype=np.float32)
    pc = ops.prepare_centers(gpu(c))
    xg = gpu(x)
    out = {}
    for mode in ("0", "1"):
        monkeypatch.setenv("RQSID_NO_RESCREEN", mode)
        ops.nearest(xg, pc)
        torch.cuda.synchronize()
        t = time.perf_counter()
        out[mode] = ops.nearest(xg, pc).cpu().numpy()
        torch.cuda.synchronize()
        print(f"k={k} dups={dups} rescreen={'off' if mode == '1' else 'on'}: {(time.perf_counter() - t) * 1e3:.2f} ms")
    assert np.array_equal(out["0"], out["1"])
    smp = np.arange(0, len(x), 7)
    assert np.array_equal(out["0"][smp], exact_ids(x[smp], c))
    if dups:
        assert (out["0"][:500] == 7).all()

def test_nearest_with_many_duplicate_centres():
    """K-Means centres initialised from rows that are exactly equal (here: zero rows, as a normalised
    residual of a one-member cluster is) make every row nearest to them an exact many-way tie.  nearest()
    drops the later copies (only the first can be the argmin), so the screen lists those rows instead of
    re-scoring all K candidates; the IDs equal the exact oracle's, ties to the lowest index."""
    rng = np.random.default_rng(77)
    k, n = 2560, 20000
    c = rng.standard_normal((k, 512)).astype(np.float32)
    c /= np.linalg.norm(c, axis=1, keepdims=True)
    dup = rng.choice(k, 300, replace=False)
    c[dup] = 0.0                       # 300 identical (zero) centres
    x = rng.standard_normal((n, 512)).astype(np.float32)
    x /= np.linalg.norm(x, axis=1, keepdims=True)
    x[:500] = 0.0                      # rows on the duplicated centre
    pc = ops.prepare_centers(gpu(c))
    ws = ops.AssignWorkspace(n, DEV)
    got = ops.nearest(gpu(x), pc, workspace=ws).cpu().numpy()
    assert pc.nearest_cand.count_max == k - 299
    assert (got[:500] == dup.min()).all()
    sel = np.arange(0, n, 7)
    assert (got[sel] == exact_ids(x[sel], c)).all()


@pytest.mark.parametrize("form", ["default", "pp88", "rows443"])
@pytest.mark.parametrize("shape", ["prod", "xl"])
def test_hi_only_centre_table_equals_interleaved(shape, form):
    """The 1-term streamed screens gather their centre pieces from the hi-only table (rqsid_prepare_centers_hi)
    by default; the interleaved table gives the same IDs on every level (ping-pong and row-resident forms, the
    PROD and XL codebook shapes), and the hi table is the interleaved table's hi halves."""
    need = (128, 128, 256) if shape == "prod" else (256, 256, 512)
    cb = synth.encode_codebooks(seed=99, need=need, n_cand=2560 if shape == "prod" else 5120)
    x = gpu(synth.mixture_rows(0, 60000))
    enc = RQEncoder([torch.from_numpy(cb[k]) for k in ("c0", "c1", "c2")], list(need),
                    match=torch.from_numpy(cb["match"]), semantics=HIERARCHICAL_TRAIN, device=DEV)
    env = {"default": {}, "pp88": STREAMED.get("pp88", {}), "rows443": {"RQSID_SCREEN_VARIANT": "8",
                                                                          "RQSID_ROWS_SHAPE": "443"}}[form]
    assert all(pc.c16h is not None for pc in enc.pcs)
    c16 = enc.pcs[2].c16.view(enc.pcs[2].k, -1, 2, 32)
    assert torch.equal(enc.pcs[2].c16h.view(enc.pcs[2].k, -1, 32), c16[:, :, 0, :])
    a = _with_env(env, lambda: enc.encode(x).cpu().numpy())
    for pc in enc.pcs:
        pc.c16h = None
    b = _with_env(env, lambda: enc.encode(x).cpu().numpy())
    assert (a == b).all(), f"{int((a != b).any(1).sum())} rows differ between the hi-only and interleaved tables"
