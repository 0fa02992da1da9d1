"""Pin the CPU oracle (oracle/rq_oracle.py) against golden vectors captured from the reference.

These run without a GPU.  Where the reference's fp32 arithmetic and the oracle's
could order two nearly tied centres differently, the mismatch must be a certified
near tie (fp64 relative gap < 1e-6) — none occur on these inputs.
"""
import numpy as np
import pytest
import torch

from oracle import rq_oracle as O
from tests import _data

F32 = np.float32


def test_assign_matches_reference(golden):
    g = golden("assign")
    x, c = _data.assign_inputs(g)
    ids = O.nearest(x, c)
    assert (ids == g["ids"]).all()
    # the mm expansion cancels |x|^2 + |c|^2 - 2x.c in fp32: compare d^2 on that scale
    d = O.cdist_f32(x, c).astype(np.float64)
    scale = (x.astype(np.float64) ** 2).sum(1)[:, None] + (c.astype(np.float64) ** 2).sum(1)[None, :]
    tol = 4e-6 * scale
    assert (np.abs(d.min(1) ** 2 - g["dmin"].astype(np.float64) ** 2) <= tol[np.arange(len(x)), ids]).all()
    assert (np.abs(d[:64] ** 2 - g["dist_head"].astype(np.float64) ** 2) <= tol[:64]).all()


def test_assign_ties_take_lowest_index(golden):
    g = golden("assign")
    x, c = _data.assign_inputs(g)
    x2, c2 = _data.tie_inputs(x, c)
    ids = O.nearest(x2, c2)
    assert (ids == g["ids_tie"]).all()
    assert ids[0] == 5 and ids[1] == 3 and ids[2] == 0


@pytest.mark.parametrize("tag,gd,norm", [("g512", [512], True), ("g128_384", [128, 384], True),
                                         ("plain", [512], False)])
def test_residual_matches_reference(golden, tag, gd, norm):
    g = golden("residual")
    x, c = _data.residual_inputs()
    r = O.residual(x, c, g["ids"], gd, normalize=norm)
    ref = g[f"res_{tag}_head"]
    if not norm:
        assert np.array_equal(r[:256], ref)  # plain fp32 subtraction is exact
    else:
        # torch.norm's fp32 reduction can differ from the correctly rounded norm by 1 ulp
        np.testing.assert_allclose(r[:256], ref, rtol=3e-7, atol=1e-9)


@pytest.mark.parametrize("s", [0, 1, 2, 3])
def test_lloyd_update_with_empty_clusters(golden, s):
    g = golden("update")
    x = _data.update_inputs(g)
    gen = torch.Generator().manual_seed(100 + s)
    rng = O.LegacyRNG(100 + s, lambda n: torch.randint(n, (1,), generator=gen).item())
    c, a = O.kmeans_fit(x, 24, rng, iter_limit=1, balanced=False)
    assert (a == g[f"assign_{s}"]).all()
    np.testing.assert_allclose(c, g[f"centers_{s}"], rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("tag", ["n64k8", "n67k8", "n1000k16", "n5k8", "n96k8"])
def test_auction_matches_reference(golden, tag):
    g = golden("auction")
    dist, out = _data.auction_case(g, tag)
    got = O.auction_lap_half(-dist)
    assert (got == out).all()


@pytest.mark.parametrize("tag", ["n64k8", "n67k8", "n1000k16", "n5k8", "n96k8"])
@pytest.mark.parametrize("tie_rule", ["torch", "stable"])
def test_auction_full_matches_reference(golden, tag, tie_rule):
    """oracle auction_lap_full (fp32) == the reference's auction_lap_full outputs (tests/golden)."""
    g = golden("auction_full")
    dist, out = _data.auction_case(g, tag)
    assert (O.auction_lap_full(-dist, tie_rule=tie_rule) == out).all()


def test_kmeans_drivers_match_reference(golden):
    g = golden("fit")
    x = _data.fit_inputs(g)

    def rng(seed):
        gen = torch.Generator().manual_seed(seed)
        return O.LegacyRNG(seed, lambda n: torch.randint(n, (1,), generator=gen).item())

    c, _ = O.kmeans_fit(x, 8, rng(3), iter_limit=12, balanced=True, min_loss_target=64)
    np.testing.assert_allclose(c, g["fbml_centers"], rtol=1e-5, atol=1e-5)
    c, a = O.kmeans_fit(x, 8, rng(4), iter_limit=5, balanced=True)
    assert (a == g["fit_bal_assign"]).all()
    np.testing.assert_allclose(c, g["fit_bal_centers"], rtol=1e-5, atol=1e-5)
    c, a = O.kmeans_fit(x, 8, rng(5), iter_limit=0, balanced=False)
    assert (a == g["fit_unbal_assign"]).all()
    np.testing.assert_allclose(c, g["fit_unbal_centers"], rtol=1e-5, atol=1e-5)


def test_hierarchical_predict_modes(golden):
    g = golden("hierarchical")
    x, xn = _data.small_rq_inputs(g)
    cents = [g["c0"], g["c1"], g["c2"]]
    need = _data.SMALL_CFG["need_clusters"]
    bug = O.encode(x, cents, need, g["match"], match_lookup=False, residual_global_id=False)
    assert (bug == g["pred_bug"]).all()
    fix = O.encode(x, cents, need, g["match"], match_lookup=True, residual_global_id=False)
    assert (fix == g["pred_fix"]).all()
    train = O.encode(x, cents, need, g["match"], residual_from_weighted=True)
    assert (train == g["train_ids"]).all()
    newbug = O.encode(xn, cents, need, g["match"], match_lookup=False, residual_global_id=False)
    assert (newbug == g["pred_new_bug"]).all()
    if int(g["new_fix_keyerror"]) >= 0:
        with pytest.raises(KeyError) as e:
            O.encode(xn, cents, need, g["match"], match_lookup=True, residual_global_id=False)
        assert e.value.args[0] == int(g["new_fix_keyerror"])


def test_simplified_encode_matches_reference(golden):
    g = golden("simplified")
    x, _ = _data.small_rq_inputs(g)
    cents = [g["l0_centers"], g["mid_centers"], g["final_centers"]]
    ids = O.encode(x, cents, _data.SMALL_CFG["need_clusters"], g["match"], normalize=False,
                   remap_last=False, last_group_mult="need_minus_2")
    assert (ids == g["ids"]).all()


def test_jsonl_bytes(golden):
    g = golden("simplified")
    sids = [f"s{i:05d}" for i in range(len(g["ids"]))]
    raw = O.jsonl_lines(sids, g["ids"])
    head = bytes(g["jsonl_head"])
    assert raw[:len(head)] == head
    from generative_ranking_recommender_amd import synth
    assert synth.sha256(np.frombuffer(raw, dtype=np.uint8)) == str(g["jsonl_sha"])


@pytest.mark.slow
def test_prod_shape_encode_matches_reference(golden):
    g = golden("encode_prod")
    x, cb = _data.prod_encode_inputs(g)
    cents = [cb["c0"], cb["c1"], cb["c2"]]
    need = [128, 128, 256]
    res = {
        "pred_bug": dict(match_lookup=False, residual_global_id=False),
        "pred_fix": dict(match_lookup=True, residual_global_id=False),
        "pred_train": dict(residual_from_weighted=True),
    }
    for key, kw in res.items():
        if key not in g:
            continue
        ids = O.encode(x, cents, need, cb["match"], **kw)
        bad = np.nonzero((ids != g[key]).any(1))[0]
        assert len(bad) == 0, f"{key}: {len(bad)} rows differ"


def _half_case(g, which):
    from tests import _data
    x, c, x2, c2 = _data.half_inputs(g)
    return (x, c, g["d"]) if which == 1 else (x2, c2, g["d2"])


@pytest.mark.parametrize("which", [1, 2])
def test_cdist_half_matches_reference(golden, which):
    """pairwise_distance_half (balancekmeans/__init__.py:536-574; the input of every auction at K >= 512):
    the oracle's restatement of torch's fp16 cdist vs the reference's own output.  A mismatch is allowed
    only where the fp32 accumulation order (torch's kernels vs numpy's) can legitimately change the fp16
    result: both values inside O.half_dist_interval."""
    x, c, d_ref = _half_case(golden("dist_half"), which)
    ref = d_ref.view(np.float16)
    got = O.cdist_half(x, c)
    lo, hi = O.half_dist_interval(x, c)
    assert not O.uncertified(got, ref, lo, hi).any()
    assert ((ref >= lo) & (ref <= hi)).all()
    assert (got != ref).mean() < 1e-3
    if which == 1:
        # equal operands: fp16 cancellation leaves d^2 = 0 (-> the clamp at 1e-5) or a few fp16 ulps
        diag = ref[np.arange(5), np.arange(5)]
        assert (diag == np.float16(1e-5)).any() and (diag < np.float16(1e-2)).all()


def test_trainer_side_files_match_reference(golden):
    """train_semantic_ids.py:239-365: training_config.json, training_statistics.json and the jsonl written
    by the reference's SemanticIDTrainer, byte for byte, from the same IDs / config."""
    from generative_ranking_recommender_amd import io as rq_io, synth
    from generative_ranking_recommender_amd.hierarchical_rq_kmeans import HierarchicalRQKMeansConfig
    g = golden("trainer")
    cfg = HierarchicalRQKMeansConfig(**_data.SMALL_CFG)
    assert rq_io.json_bytes(rq_io.training_config(cfg, True)) == bytes(g["config_json"])
    sids = [f"s{i:05d}" for i in range(len(g["ids"]))]
    semantic = {s: [int(v) for v in row] for s, row in zip(sids, g["ids"])}
    assert rq_io.json_bytes(rq_io.semantic_id_statistics(semantic, cfg.need_clusters)) == bytes(g["stats_json"])
    raw = O.jsonl_lines(sids, g["ids"])
    assert synth.sha256(np.frombuffer(raw, dtype=np.uint8)) == str(g["jsonl_sha"])
    assert (g["ids"] == golden("hierarchical")["train_ids"]).all()  # the driver trains what G3 trained


@pytest.mark.parametrize("reader", ["oracle", "native"])
def test_csv_loader_matches_reference(golden, tmp_path, reader):
    """simplified_semantic_id_generator.py:38-76: the reference loader's own output on a file exercising
    its skip rules (too few fields, non-numeric, wrong dimension, duplicate ids, padded numbers) and the
    fp16 rule (any layer_clusters > 512), for the CSV restatement and the native reader."""
    from oracle import csv_oracle
    from generative_ranking_recommender_amd import io as rq_io
    g = golden("csv")
    p = tmp_path / "v.csv"
    p.write_bytes(bytes(g["text"]))
    def load(path, dim, lc):
        out = (csv_oracle.load_song_vectors if reader == "oracle" else rq_io.load_song_vectors)(path, dim, lc)
        return out[0], out[1]
    ids, x = load(str(p), 4, [2])
    assert ids == [str(s) for s in g["sids"]]
    assert x.dtype == np.float32 and np.array_equal(x, g["emb"])
    ids_h, x_h = load(str(p), 4, [600])
    assert str(g["emb_half_dtype"]) == "torch.float16" and x_h.dtype == np.float16
    assert np.array_equal(x_h.view(np.uint16), g["emb_half"].view(np.uint16))


# ----------------------------------------------------------------- match-matrix builders (§8f row 2)
@pytest.mark.parametrize("variant", ["hier", "simp"])
def test_match_builders_match_reference(golden, variant):
    """The oracle's restatements of _assign_last_match_matrix (:968-1053) and _get_dynamic_match_matrix
    (simplified…:247-303), replaying the reference's recorded sub-K-Means results, give the reference's
    match matrix, the reference's greedy operands and leave both generators where the reference did."""
    g = golden("match")
    x, l1, l2, cand = _data.match_inputs(g)
    need = _data.MATCH_NEED
    sizes = _data.MATCH_SIZES
    subs = []
    if variant == "hier":
        np.random.seed(71)
        torch.manual_seed(71)
        fits = [g["hier_fitted"][g["hier_fitted_off"][i]:g["hier_fitted_off"][i + 1]]
                for i in range(len(g["hier_fitted_off"]) - 1)]
        got = O.assign_last_match_matrix(x, l1, l2, cand, need[0], need[1], need[2], 2 * need[2],
                                         O.recorded_fits(fits, need[2]), subs_out=subs)
        want_sub, want_off = g["hier_sub"], g["hier_sub_off"]
    else:
        np.random.seed(72)
        torch.manual_seed(72)
        off = g["simp_sub_off"]
        fits = [g["simp_sub"][off[gi]:off[gi + 1]] for gi, n in enumerate(sizes) if n > need[2]]
        got = O.dynamic_match_matrix(x, l1, l2, cand, need[0], need[1], need[2],
                                     O.recorded_fits(fits, need[2]), subs_out=subs)
        want_sub, want_off = g["simp_sub"], g["simp_sub_off"]
    np_after = np.random.randint(1 << 30, size=4)
    torch_after = torch.randint(1 << 30, (4,)).numpy()
    assert len(subs) == len(want_off) - 1
    for i, s in enumerate(subs):
        assert np.array_equal(s, want_sub[want_off[i]:want_off[i + 1]])
    assert np.array_equal(got, g[f"{variant}_match"])
    assert np.array_equal(np_after, g[f"{variant}_np_after"])
    assert np.array_equal(torch_after, g[f"{variant}_torch_after"])
    assert (got.sum(1)[np.asarray(sizes) > 0] == need[2]).all() if variant == "hier" else (got.sum(1) == need[2]).all()


def test_greedy_certificate_on_reference_operands(golden):
    """On the reference's own greedy operands the certificate's determined columns are in the reference's
    row, and at an undetermined step (an fp32 near tie under the any-order bound, or the duplicated
    candidate pair 5 / 63) the reference took one of the tied columns: the certificate the GPU parity
    test relies on is consistent with the reference."""
    g = golden("match")
    x, l1, l2, cand = _data.match_inputs(g)
    need = _data.MATCH_NEED[2]
    off = g["hier_sub_off"]
    rows = [gi for gi, n in enumerate(_data.MATCH_SIZES) if n > 0]
    for k, gi in enumerate(rows):
        sub = g["hier_sub"][off[k]:off[k + 1]]
        cert = O.greedy_certificate(sub, cand, min(len(sub), need))
        row = g["hier_match"][gi]
        assert row[cert["taken"]].all()
        if not cert["determined"]:
            assert row[cert["tied"]].any(), cert


@pytest.mark.parametrize("tag", sorted(_data.CONFIG0_CASES))
def test_config0_single_level_matches_reference(golden, tag):
    """BASELINE configs[0] (SimplifiedHierarchicalRQ with one level, simplified…:193-202): the oracle's
    fit_by_min_loss with target_nodes_num = np.prod([]) = 1.0 and the reference's seeds reproduces the
    reference's centres and per-song IDs (tests/golden/config0.npz).  The distances are the reference's
    own torch.cdist call (O.torch_cdist_batched): with numpy's summation order instead, an fp16 score
    rounds the other way somewhere in the K = 128 run and 12 of 128 centres part (a legitimate
    order effect, certified on the GPU side by tests/_certify.py)."""
    g = golden("config0")
    x, k, it = _data.config0_inputs(tag, g)
    target = np.prod([])
    assert target == 1.0
    torch.manual_seed(42)
    rng = O.LegacyRNG(42, lambda n: torch.randint(n, (1,)).item())
    c, _ = O.kmeans_fit(x, k, rng, iter_limit=it, balanced=True, min_loss_target=target,
                        dist_fn=O.torch_cdist_batched)
    np.testing.assert_allclose(c, g[f"{tag}_centers"], rtol=1e-5, atol=1e-5)
    assert np.array_equal(O.torch_cdist_batched(x, c).argmin(1), g[f"{tag}_ids"][:, 0])


@pytest.mark.parametrize("tag", ["k8", "k128"])
def test_config0_exact_fixture_matches_reference_with_either_tie_rule(golden, tag):
    """tests/golden/exact.npz (the tree-mixture rows on which the reference's fits take no tie-born step):
    the oracle's fit_by_min_loss reproduces the reference's centres and IDs with the reference's own
    torch.topk tie choice AND with the lowest-index rule of the HIP kernels, and with numpy's summation
    order as well as torch's -- the fixture pins the trainer, not an implementation detail."""
    g = golden("exact")
    x = _data.exact_rows(tag, g[f"{tag}_labels"], g)
    spec = _data.EXACT_CASES[tag]
    for dist in (O.torch_cdist_batched, O.cdist_f32):
        torch.manual_seed(42)
        rng = O.LegacyRNG(42, lambda n: torch.randint(n, (1,)).item())
        c, _ = O.kmeans_fit(x, spec["k"], rng, iter_limit=spec["iter_limit"], balanced=True, min_loss_target=1.0,
                            dist_fn=dist)
        np.testing.assert_allclose(c, g[f"{tag}_c0"], rtol=1e-5, atol=1e-5)
        assert np.array_equal(O.nearest(x, c, exact=True), g[f"{tag}_ids"][:, 0])


def test_exact_fixture_reference_auctions_are_tie_free(golden):
    """Every balanced auction of the exact fixtures settles without a tie-rule dependence: on the
    level-0 scores of the hier case (the reference's first fit, its initial centres = the rows its seed
    draws), torch's tie rule and the lowest-index rule give the same assignment, which is the blob labels."""
    g = golden("exact")
    lab = g["hier_labels"].astype(np.int64)
    x = _data.exact_rows("hier", lab, g)
    np.random.seed(42)
    idx = np.random.choice(len(x), 8, replace=False)
    s = -O.torch_cdist_batched(x, x[idx])
    cert = O.auction_tie_certificate(s)
    assert np.array_equal(cert["torch"], cert["stable"])
    assert np.array_equal(cert["stable"], lab[:, 0])


def test_pairwise_cosine_and_cosine_kmeans_match_reference(golden):
    """pairwise_cosine (balancekmeans/__init__.py:625-655) and KMeans(distance='cosine') fits / predict
    (:279-280, 511-512) restated by the oracle against the reference's outputs (tests/golden/cosine.npz)."""
    g = golden("cosine")
    x, c = _data.cosine_inputs(g)
    np.testing.assert_allclose(O.pairwise_cosine(x, c), g["d"], rtol=0, atol=2e-6)

    def rng(seed):
        gen = torch.Generator().manual_seed(seed)
        np.random.seed(seed)
        return O.LegacyRNG(seed, lambda n: torch.randint(n, (1,), generator=gen).item())

    c1, a1 = O.kmeans_fit(x, 8, rng(31), iter_limit=4, balanced=True, dist_fn=O.pairwise_cosine)
    assert np.array_equal(a1, g["fit_bal_assign"])
    np.testing.assert_allclose(c1, g["fit_bal_centers"], rtol=1e-5, atol=1e-5)
    assert np.array_equal(O.pairwise_cosine(x, c1).argmin(1), g["pred"])
    c2, a2 = O.kmeans_fit(x, 8, rng(32), iter_limit=3, balanced=False, dist_fn=O.pairwise_cosine)
    assert np.array_equal(a2, g["fit_unbal_assign"])
    np.testing.assert_allclose(c2, g["fit_unbal_centers"], rtol=1e-5, atol=1e-5)
    c3, _ = O.kmeans_fit(x, 8, rng(33), iter_limit=4, balanced=True, min_loss_target=64, dist_fn=O.pairwise_cosine)
    np.testing.assert_allclose(c3, g["fbml_centers"], rtol=1e-5, atol=1e-5)
