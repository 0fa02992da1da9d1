"""Lockstep (segmented) sub-K-Means on the GPU: the segmented score kernel and the segmented auction
against the single-segment kernels (each already pinned bit for bit to the oracle's stable-tie auction
in test_gpu_training.py) and against the oracle directly, and balancekmeans.batched_fit against the
reference-order sequential KMeans.fit / fit_by_min_loss run segment by segment with the same draws
(hierarchical_rq_kmeans.py:703-725, 1010-1019)."""
import numpy as np
import pytest
import torch

from generative_ranking_recommender_amd import ops, synth
from generative_ranking_recommender_amd.balancekmeans import KMeans, batched_fit, init_indices
from generative_ranking_recommender_amd.hierarchical_rq_kmeans import HierarchicalRQKMeans, HierarchicalRQKMeansConfig
from oracle import rq_oracle as O

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def _blocks(w_flat, k, off):
    w = w_flat.cpu()
    return [w[k * off[s]:k * off[s + 1]].view(k, off[s + 1] - off[s]) for s in range(len(off) - 1)]


@pytest.mark.parametrize("half", [False, True])
def test_seg_scores_equal_per_segment_scores(half):
    k = 24
    sizes = np.array([70, 0, 5, 64, 200, 1], dtype=np.int64)
    x = torch.from_numpy(synth.small_mixture(int(sizes.sum()), m=12, seed=3)).to(DEV)
    c = torch.randn(len(sizes) * k, 512, device=DEV)
    lay = ops.SegmentLayout(sizes, DEV)
    w = ops.seg_auction_scores(x, c, k, lay, half=half)
    for s, blk in enumerate(_blocks(w, k, lay.off)):
        if sizes[s] == 0:
            continue
        ref = ops.auction_scores(x[lay.off[s]:lay.off[s + 1]].contiguous(), c[s * k:(s + 1) * k], half=half).cpu()
        assert torch.equal(blk.view(torch.int16), ref.view(torch.int16)), s


def _random_scores(rng, k, n, levels):
    """-distance-like fp16 scores with many exact ties (few distinct levels)."""
    v = -rng.integers(1, levels + 1, size=(k, n)).astype(np.float32) * np.float32(0.37)
    return v.astype(np.float16)


@pytest.mark.parametrize("k,levels", [(8, 5), (16, 2000), (128, 40)])
def test_seg_auction_equals_single_auction(k, levels):
    rng = np.random.default_rng(k + levels)
    # empty, fewer jobs than workers (farthest fallback), N % K == 0 (few rounds), ragged (1002 rounds),
    # two and three chunks (global histograms), one chunk exactly full
    ch = int(ops.lib().rqsid_seg_auction_chunk_jobs())
    sizes = np.array([0, k - 1, 4 * k, 3 * k + 5, ch + 7, 2 * ch + 300, ch, 2 * k + 1], dtype=np.int64)
    blocks = [_random_scores(rng, k, int(n), levels) for n in sizes]
    flat = np.concatenate([b.reshape(-1) for b in blocks])
    lay = ops.SegmentLayout(sizes, DEV)
    a, rounds = ops.seg_auction(torch.from_numpy(flat).to(DEV), k, lay)
    a = a.cpu().numpy()
    rounds = rounds.cpu().numpy()
    for s, b in enumerate(blocks):
        if sizes[s] == 0:
            assert rounds[s] == 0
            continue
        ref, r_ref = ops.auction(torch.from_numpy(np.ascontiguousarray(b)).to(DEV))
        got = a[lay.off[s]:lay.off[s + 1]]
        assert np.array_equal(got, ref.cpu().numpy()), s
        assert rounds[s] == r_ref, (s, rounds[s], r_ref)


def test_seg_auction_against_oracle_and_active_mask():
    k = 8
    rng = np.random.default_rng(5)
    sizes = np.array([67, 64, 120, 2100], dtype=np.int64)  # the last spans three chunks
    blocks = [_random_scores(rng, k, int(n), 7) for n in sizes]
    flat = torch.from_numpy(np.concatenate([b.reshape(-1) for b in blocks])).to(DEV)
    lay = ops.SegmentLayout(sizes, DEV)
    out = torch.full((int(sizes.sum()),), -7, dtype=torch.int32, device=DEV)
    a, rounds = ops.seg_auction(flat, k, lay, active=torch.tensor([1, 0, 1, 1], dtype=torch.uint8, device=DEV), out=out)
    a = a.cpu().numpy()
    assert (a[64 + 3:64 + 3 + 64] == -7).all() and rounds.cpu().numpy()[1] == 0  # skipped segment untouched
    for s in (0, 2, 3):
        want = O.auction_lap_half(blocks[s].T.astype(np.float32), tie_rule="stable")
        assert np.array_equal(a[lay.off[s]:lay.off[s + 1]], np.asarray(want, dtype=np.int64)), s


@pytest.mark.parametrize("levels", [6, 3000])
def test_seg_auction_small_groups_against_oracle(levels):
    """The last layer's group shape (one-chunk segments with 2 or 3 jobs per worker: the block's top-4
    merge selection whenever the guessed window misses), heavily tied and nearly tie-free; K=128 keeps
    the oracle's 1002 rounds to seconds (the PROD groups have K=256, jpw=2)."""
    k = 128
    rng = np.random.default_rng(levels)
    sizes = np.array([300, 3 * k + 1, 2 * k + 1], dtype=np.int64)
    blocks = [_random_scores(rng, k, int(n), levels) for n in sizes]
    flat = torch.from_numpy(np.concatenate([b.reshape(-1) for b in blocks])).to(DEV)
    lay = ops.SegmentLayout(sizes, DEV)
    a, rounds = ops.seg_auction(flat, k, lay)
    a = a.cpu().numpy()
    for s in range(len(sizes)):
        want = O.auction_lap_half(blocks[s].T.astype(np.float32), tie_rule="stable")
        assert np.array_equal(a[lay.off[s]:lay.off[s + 1]], np.asarray(want, dtype=np.int64)), s


def test_seg_auction_repeat_calls_with_rewritten_scores():
    """Repeated auctions over one score buffer rewritten in place between calls (the K-Means iterations' pattern):
    the round blocks instantiated by one call are replayed by the next when the buffers and shapes agree, so
    each call must still read the new scores (every result against the oracle)."""
    k = 8
    sizes = np.array([67, 2100, 130], dtype=np.int64)
    flat = torch.empty(int(sizes.sum()) * k, dtype=torch.float16, device=DEV)
    lay = ops.SegmentLayout(sizes, DEV)
    for it in range(3):
        rng = np.random.default_rng(100 + it)
        blocks = [_random_scores(rng, k, int(n), 7 + 500 * it) for n in sizes]
        flat.copy_(torch.from_numpy(np.concatenate([b.reshape(-1) for b in blocks])))
        a, _ = ops.seg_auction(flat, k, lay)
        a = a.cpu().numpy()
        for s in range(len(sizes)):
            want = O.auction_lap_half(blocks[s].T.astype(np.float32), tie_rule="stable")
            assert np.array_equal(a[lay.off[s]:lay.off[s + 1]], np.asarray(want, dtype=np.int64)), (it, s)


def _segments(sizes, seed):
    x = synth.small_mixture(int(np.sum(sizes)), m=24, seed=seed)
    return torch.from_numpy(x).to(DEV), ops.SegmentLayout(np.asarray(sizes, dtype=np.int64), DEV)


@pytest.mark.parametrize("balanced", [True, False])
def test_batched_fit_equals_sequential_fits(balanced):
    k = 16
    # unbalanced fits meet empty clusters, whose torch RNG draws come in another order across segments
    # in lockstep: one segment there (same order), every segment shape for the balanced fits
    sizes = [300, 40, 16, 257, 1100] if balanced else [1100]
    x, lay = _segments(sizes, 11)
    limits = [4, 3, 2, 5, 4][:len(sizes)]
    np.random.seed(5)
    inits = [[init_indices(n, k)] for n in sizes]
    torch.manual_seed(3)
    centers, a = batched_fit(x, lay, k, limits, inits, tol=0.0, balanced=balanced)
    torch.manual_seed(3)
    for s, n in enumerate(sizes):
        xs = x[lay.off[s]:lay.off[s + 1]]
        km = KMeans(n_clusters=k, cluster_centers=xs[torch.from_numpy(inits[s][0]).to(DEV)].clone(), device=DEV,
                    balanced=balanced)
        a_ref = km.fit(xs, tol=0.0, iter_limit=limits[s], online=True, iter_k=1)
        assert (a[lay.off[s]:lay.off[s + 1]].cpu() == a_ref.int()).all(), s
        torch.testing.assert_close(centers[s * k:(s + 1) * k], km.cluster_centers, rtol=1e-6, atol=1e-6)


def test_batched_min_loss_equals_sequential_fits():
    k = 8
    sizes = [400, 90, 333]
    x, lay = _segments(sizes, 12)
    limits = [23, 12, 15]
    target = 40
    inits = []
    for s, n in enumerate(sizes):
        np.random.seed(100 + s)
        inits.append([init_indices(n, k) for _ in range(1 + (limits[s] - 1) // 10)])
    centers, _ = batched_fit(x, lay, k, limits, inits, target_nodes_num=target, tol=0.0)
    for s, n in enumerate(sizes):
        np.random.seed(100 + s)  # the sequential fit draws the same start and re-initialisations
        km = KMeans(n_clusters=k, device=DEV, balanced=True)
        km.fit_by_min_loss(x[lay.off[s]:lay.off[s + 1]], target_nodes_num=target, tol=0.0, iter_limit=limits[s])
        torch.testing.assert_close(centers[s * k:(s + 1) * k], km.cluster_centers, rtol=1e-6, atol=1e-6)


def test_hierarchical_batched_match_matrix_equals_sequential():
    """The last layer's match-matrix builder: lockstep group fits give the sequential builder's matrix
    (``fit`` draws only its start from numpy, so the reference's RNG order is kept exactly)."""
    cfg = HierarchicalRQKMeansConfig(layer_clusters=[4, 8, 16], need_clusters=[4, 4, 8], embedding_dim=512,
                                     iter_limit=3)
    n = 3000
    x = torch.from_numpy(synth.small_mixture(n, m=32, seed=8)).to(DEV)
    rng = np.random.default_rng(0)
    # uneven groups: empty, short (< need), exactly need, mid (< 2 need), large
    l1 = torch.from_numpy(rng.choice(4, n, p=[0.55, 0.3, 0.149, 0.001])).to(DEV)
    l2 = torch.from_numpy(rng.choice(4, n, p=[0.7, 0.2, 0.098, 0.002])).to(DEV)
    cand = torch.randn(32, 512, device=DEV)
    out = []
    for batched in (True, False):
        m = HierarchicalRQKMeans(cfg, device=DEV)
        m.batched_sub_fits = batched
        np.random.seed(9)
        torch.manual_seed(9)
        out.append(m._assign_last_match_matrix(cand, 32, x, 4, 4, l1, l2, 8, 16, 2))
    assert np.array_equal(out[0], out[1])
    assert (out[0].sum(1)[np.bincount((l1 * 4 + l2).cpu().numpy(), minlength=16) > 0] == 8).all()


def test_simplified_batched_equals_sequential():
    """The simplified generator's middle-layer sub-fits and dynamic match matrix (simplified…:98-140,
    247-303): lockstep and sequential runs draw the same numbers and give the same centres / matrix."""
    from generative_ranking_recommender_amd.simplified_semantic_id_generator import SimplifiedHierarchicalRQ
    cfg = HierarchicalRQKMeansConfig(layer_clusters=[4, 8, 16], need_clusters=[4, 4, 8], embedding_dim=512,
                                     iter_limit=3)
    n = 2500
    x = torch.from_numpy(synth.small_mixture(n, m=32, seed=9)).to(DEV)
    rng = np.random.default_rng(1)
    p1 = torch.from_numpy(rng.choice(4, n, p=[0.6, 0.3, 0.098, 0.002])).to(DEV)
    l2 = torch.from_numpy(rng.choice(4, n, p=[0.7, 0.2, 0.098, 0.002])).to(DEV)
    cand = torch.randn(32, 512, device=DEV)
    res = []
    for batched in (True, False):
        m = SimplifiedHierarchicalRQ(cfg, device=DEV)
        m.batched_sub_fits = batched
        np.random.seed(4)
        torch.manual_seed(4)
        ids, _ = m._train_middle_layer(x, p1, 1)
        mm = m._get_dynamic_match_matrix(x, p1, l2, cand)
        res.append((ids.cpu(), m.middle_layer_centers.cpu(), mm))
    assert torch.equal(res[0][0], res[1][0])
    torch.testing.assert_close(res[0][1], res[1][1], rtol=1e-6, atol=1e-6)
    assert torch.equal(res[0][2], res[1][2])


def _rng_state_equal(a, b):
    return a[0] == b[0] and np.array_equal(a[1], b[1]) and a[2:] == b[2:]


def test_middle_layer_batched_equals_sequential_with_early_convergence():
    """a parent that converges before its last re-initialisation, and parents with fewer rows
    than centres (argmin fallback, empty clusters refilled from the torch RNG in several segments).  The
    lockstep middle layer must give the sequential loop's centres AND leave both generators in the
    sequential loop's state (hierarchical_rq_kmeans.py:703-731, balancekmeans/__init__.py:305-306, 321-322)."""
    cfg = HierarchicalRQKMeansConfig(layer_clusters=[4, 8, 16], need_clusters=[4, 8, 8], embedding_dim=512,
                                     iter_limit=100)
    pts = synth.small_mixture(8, m=8, seed=31)
    parts = [np.repeat(pts, 20, axis=0),                              # 8 distinct rows x 20: converges at once
             synth.small_mixture(5, m=4, seed=32),                    # 5 rows < 8 centres
             synth.small_mixture(6, m=4, seed=33),                    # 6 rows < 8 centres
             synth.small_mixture(300, m=16, seed=34)]
    x = torch.from_numpy(np.concatenate(parts)).to(DEV)
    prev = torch.from_numpy(np.concatenate([np.full(len(p), i) for i, p in enumerate(parts)])).to(DEV)
    perm = torch.from_numpy(np.random.default_rng(2).permutation(len(x))).to(DEV)
    x, prev = x[perm].contiguous(), prev[perm]
    res = []
    for batched in (True, False):
        m = HierarchicalRQKMeans(cfg, device=DEV)
        m.batched_sub_fits = batched
        m.result_cluster_ids = [prev]
        np.random.seed(77)
        torch.manual_seed(77)
        c, ids, r = m._train_middle_layer(x, 1)
        res.append((c.cpu(), ids.cpu(), np.random.get_state(), torch.get_rng_state()))
    torch.testing.assert_close(res[0][0], res[1][0], rtol=1e-6, atol=1e-6)
    assert torch.equal(res[0][1], res[1][1])
    assert _rng_state_equal(res[0][2], res[1][2]), "numpy RNG state differs from the sequential loop's"
    assert torch.equal(res[0][3], res[1][3]), "torch RNG state differs from the sequential loop's"


def test_fit_segments_restores_torch_draw_order():
    """Unbalanced lockstep fits with empty clusters in several segments: fit_segments gives the
    one-after-another result and torch state (the lockstep loop alone draws in another order)."""
    k = 16
    sizes = [10, 1100, 12, 700]  # fewer rows than centres: argmin fallback, empty clusters every iteration
    x, lay = _segments(sizes, 13)
    limits = [4, 3, 5, 4]
    np.random.seed(6)
    inits = [[init_indices(n, k)] for n in sizes]
    torch.manual_seed(8)
    from generative_ranking_recommender_amd.balancekmeans import fit_segments
    centers, a = fit_segments(x, sizes, k, limits, inits, tol=0.0)
    st = torch.get_rng_state()
    torch.manual_seed(8)
    for s, n in enumerate(sizes):
        xs = x[lay.off[s]:lay.off[s + 1]]
        km = KMeans(n_clusters=k, cluster_centers=xs[torch.from_numpy(inits[s][0]).to(DEV)].clone(), device=DEV,
                    balanced=True)
        a_ref = km.fit(xs, tol=0.0, iter_limit=limits[s], online=True, iter_k=1)
        assert (a[lay.off[s]:lay.off[s + 1]].cpu() == a_ref.int()).all(), s
        torch.testing.assert_close(centers[s * k:(s + 1) * k], km.cluster_centers, rtol=1e-6, atol=1e-6)
    assert torch.equal(st, torch.get_rng_state())
