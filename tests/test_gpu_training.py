"""Training path on the GPU: the auction kernels bit for bit against the oracle (stable tie rule),
K-Means fits against the oracle, and the hierarchical / simplified trainers end to end (invariants
and train/encode consistency; the reference's balanced fits are pinned by invariants only because
torch.topk's tie order is implementation-defined, SURVEY.md §7 hard part 3)."""
import numpy as np
import pytest
import torch

from generative_ranking_recommender_amd import ops, synth
from generative_ranking_recommender_amd import io as rq_io
from generative_ranking_recommender_amd.balancekmeans import (KMeans, auction_lap_half, pairwise_distance_full,
                                                              pairwise_distance_half)
from generative_ranking_recommender_amd.hierarchical_rq_kmeans import HierarchicalRQKMeans, HierarchicalRQKMeansConfig
from generative_ranking_recommender_amd.simplified_semantic_id_generator import SimplifiedHierarchicalRQ
from oracle import rq_oracle as O
from tests import _data

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def gpu_auction(neg_dist_f16: np.ndarray):
    w = torch.from_numpy(np.ascontiguousarray(neg_dist_f16.T)).to(DEV)
    a, rounds = ops.auction(w)
    return a.cpu().numpy().astype(np.int64), rounds


@pytest.mark.parametrize("tag", ["n64k8", "n67k8", "n1000k16", "n5k8", "n96k8"])
def test_auction_golden_inputs_match_oracle(golden, tag):
    g = golden("auction")
    dist, _ = _data.auction_case(g, tag)
    scores = (-dist).astype(np.float16)
    got, rounds = gpu_auction(scores)
    ref = O.auction_lap_half(scores.astype(np.float32), tie_rule="stable")
    assert (got == ref).all()


# N % 4 == 0 takes the 8-byte-load sweeps (4 jobs per lane, ranks in lane-major job order); 4100 and 2048
# add heavily tied multi-chunk cases of that path (tie ranks across lanes, waves and chunks)
@pytest.mark.parametrize("n,k,levels", [(200, 8, 0), (256, 8, 0), (999, 16, 7), (3000, 16, 0), (513, 32, 3),
                                        (4100, 16, 5), (2048, 8, 3), (3001, 16, 5),
                                        # K = 256 (BASELINE configs[4]'s level 0 / middle level)
                                        (5120, 256, 7), (5120, 256, 0), (601, 256, 5)])
def test_auction_random_and_tied_match_oracle(n, k, levels):
    rng = np.random.default_rng(n * k)
    d = rng.random((n, k), dtype=np.float32) * 4
    if levels:
        d = np.round(d * levels) / levels  # heavy ties at every top-k boundary
    scores = (-d).astype(np.float16)
    got, rounds = gpu_auction(scores)
    ref = O.auction_lap_half(scores.astype(np.float32), tie_rule="stable")
    assert (got == ref).all()
    if n % k:
        assert rounds == 1002  # the leftover rule ends it (Appendix A item 6)


# the last layer's candidate-fit widths (hierarchical_rq_kmeans.py:792-801: K = 1280 PROD, 2560 XL), with
# N % K == 0 and != 0 (1002 rounds, on the 2-byte-load path: N % 4 != 0) and heavily tied levels
@pytest.mark.parametrize("n,k,levels", [(2560, 1280, 0), (2560, 1280, 5), (1501, 1280, 0), (5120, 2560, 0),
                                        (5120, 2560, 7)])
def test_auction_candidate_fit_widths_match_oracle(n, k, levels):
    rng = np.random.default_rng(n * k + 7)
    d = rng.random((n, k), dtype=np.float32) * 4
    if levels:
        d = np.round(d * levels) / levels
    scores = (-d).astype(np.float16)
    got, rounds = gpu_auction(scores)
    ref = O.auction_lap_half(scores.astype(np.float32), tie_rule="stable")
    assert (got == ref).all()
    if n % k:
        assert rounds == 1002


def test_auction_half_scores_k1280_match_oracle():
    """fp16 pairwise_distance_half scores (the candidate fits' input, :546-574 via balancekmeans.py) of
    unit-norm rows: values crowd into few fp16 levels, so the topk boundary is full of equal values."""
    x = synth.small_mixture(2560, m=200, seed=31)
    x /= np.linalg.norm(x, axis=1, keepdims=True)
    c = x[np.random.default_rng(3).choice(2560, 1280, replace=False)] + np.float32(0.01)
    w = ops.auction_scores(torch.from_numpy(x.astype(np.float32)).to(DEV), torch.from_numpy(c.astype(np.float32)).to(DEV),
                           half=True)
    a, rounds = ops.auction(w)
    s16 = w.cpu().numpy().T
    ref = O.auction_lap_half(s16.astype(np.float32), tie_rule="stable")
    assert (a.cpu().numpy().astype(np.int64) == ref).all()
    assert len(np.unique(s16)) < s16.size // 100  # heavily tied


@pytest.mark.parametrize("tag", ["n64k8", "n67k8", "n1000k16", "n5k8", "n96k8"])
def test_auction_full_golden_inputs_match_reference(golden, tag):
    """fp32 auction (auction_lap_full, A6) on the reference's own outputs (tests/golden/auction_full.npz,
    captured by running the reference: 1002-round leftover case n67k8, N < K case n5k8)."""
    g = golden("auction_full")
    dist, want = _data.auction_case(g, tag)
    got, _ = ops.auction_full(torch.from_numpy(np.ascontiguousarray(-dist.T)).to(DEV))
    assert (got.cpu().numpy() == want).all()


@pytest.mark.parametrize("n,k,levels", [(300, 8, 0), (2050, 16, 5), (999, 16, 7), (40, 32, 3)])
def test_auction_full_random_and_tied_match_oracle(n, k, levels):
    rng = np.random.default_rng(n * k + 1)
    d = rng.random((n, k), dtype=np.float32) * 4
    if levels:
        d = np.round(d * levels) / levels  # heavy ties at every top-k boundary
    s = -d
    got, rounds = ops.auction_full(torch.from_numpy(np.ascontiguousarray(s.T)).to(DEV))
    assert (got.cpu().numpy() == O.auction_lap_full(s, tie_rule="stable")).all()
    if n % k:
        assert rounds == 1002


def test_kmeans_predict_balanced_uses_fp32_auction():
    x = torch.from_numpy(synth.small_mixture(512, m=8, seed=4)).to(DEV)
    km = KMeans(n_clusters=8, cluster_centers=x[:8].clone(), device=DEV)
    got = km.predict(x, balanced=True).numpy()
    d = pairwise_distance_full(x, x[:8].clone()).cpu().numpy()
    assert (got == O.auction_lap_full(-d, tie_rule="stable")).all()
    assert np.bincount(got, minlength=8).max() <= 512 // 8


def test_auction_fewer_jobs_than_workers_is_farthest():
    rng = np.random.default_rng(0)
    d = rng.random((5, 8), dtype=np.float32)
    s16 = (-d).astype(np.float16)
    got, _ = gpu_auction(s16)
    assert (got == O.auction_lap_half(s16.astype(np.float32))).all()  # argmin(-D): the farthest centre


def test_auction_lap_half_api_and_balance():
    x = torch.from_numpy(synth.small_mixture(4096, m=16, seed=3)).to(DEV)
    c = x[:64].clone()
    d = pairwise_distance_half(x, c)
    a = auction_lap_half(-d.float())
    assert a.shape == (4096,) and a.dtype == torch.int64
    cnt = torch.bincount(a, minlength=64).cpu().numpy()
    assert cnt.sum() == 4096 and cnt.max() <= 4096 // 64 + 1 and cnt.min() >= 4096 // 64 - 1


def seeded(seed):
    np.random.seed(seed)
    torch.manual_seed(seed)


def test_kmeans_fit_unbalanced_matches_oracle(golden):
    g = golden("fit")
    x = _data.fit_inputs(g)
    seeded(5)
    km = KMeans(n_clusters=8, device=DEV, balanced=False)
    a = km.fit(torch.from_numpy(x), iter_limit=0).numpy()
    gen = torch.Generator().manual_seed(5)
    rng = O.LegacyRNG(5, lambda n: torch.randint(n, (1,), generator=gen).item())
    c_ref, a_ref = O.kmeans_fit(x, 8, rng, iter_limit=0, balanced=False)
    assert (a == a_ref).all()
    np.testing.assert_allclose(km.cluster_centers.cpu().numpy(), c_ref, rtol=1e-5, atol=1e-5)
    # the reference's own golden (same seeds, torch's arithmetic)
    assert (a == g["fit_unbal_assign"]).all()
    np.testing.assert_allclose(km.cluster_centers.cpu().numpy(), g["fit_unbal_centers"], rtol=1e-5, atol=1e-5)


def test_kmeans_empty_cluster_takes_random_row():
    x = synth.small_mixture(300, m=3, seed=9)
    seeded(1)
    km = KMeans(n_clusters=40, device=DEV, balanced=False)
    km.fit(torch.from_numpy(x), iter_limit=2)
    gen = torch.Generator().manual_seed(1)
    rng = O.LegacyRNG(1, lambda n: torch.randint(n, (1,), generator=gen).item())
    c_ref, a_ref = O.kmeans_fit(x, 40, rng, iter_limit=2, balanced=False)
    np.testing.assert_allclose(km.cluster_centers.cpu().numpy(), c_ref, rtol=1e-5, atol=1e-5)


def test_kmeans_balanced_fit_invariants():
    x = torch.from_numpy(synth.small_mixture(2048, m=16, seed=4))
    seeded(7)
    km = KMeans(n_clusters=16, device=DEV, balanced=True)
    a = km.fit(x, iter_limit=4)
    cnt = np.bincount(a.numpy(), minlength=16)
    assert cnt.sum() == 2048 and cnt.max() <= 2048 // 16 + 1
    seeded(7)
    km2 = KMeans(n_clusters=16, device=DEV, balanced=True)
    a2 = km2.fit(x, iter_limit=4)
    assert torch.equal(a, a2) and torch.equal(km.cluster_centers, km2.cluster_centers)  # deterministic
    seeded(8)
    km3 = KMeans(n_clusters=16, device=DEV, balanced=True)
    km3.fit_by_min_loss(x, target_nodes_num=64, iter_limit=12)
    assert km3.cluster_centers.shape == (16, 512) and torch.isfinite(km3.cluster_centers).all()
    assert len(km3.last_auction_rounds) == 12


SMALL = dict(layer_clusters=[8, 16, 16], need_clusters=[8, 8, 8], embedding_dim=512, iter_limit=5)


def test_hierarchical_train_predict_save_load(tmp_path):
    x = synth.small_mixture(2048, m=64, seed=21)
    seeded(42)
    model = HierarchicalRQKMeans(HierarchicalRQKMeansConfig(**SMALL), checkpoint_dir=str(tmp_path / "ck"), device=DEV)
    res = model.train(x)
    ids = np.stack([t.cpu().numpy() for t in res["cluster_ids"]], 1)
    assert ids.shape == (2048, 3)
    assert (ids >= 0).all() and (ids.max(0) < np.array(SMALL["need_clusters"])).all()
    m = np.asarray(model.match_matrices[0])
    assert m.shape == (64, 32) and (m.sum(1)[np.unique(ids[:, 0] * 8 + ids[:, 1])] == 8).all()
    # the training-consistent encode of the training rows reproduces the training ids
    assert (model.predict(x, reference_quirks=False) == ids).all()
    # the reference's predict: modulo residuals + unconstrained last layer (raw ids < 2*lc)
    quirky = model.predict(x)
    assert (quirky[:, :2] == ids[:, :2]).all() and quirky[:, 2].max() < 32
    # save / load round trip
    model.save_model(str(tmp_path / "model"))
    m2 = HierarchicalRQKMeans(HierarchicalRQKMeansConfig(**SMALL), device=DEV)
    m2.load_model(str(tmp_path / "model"))
    assert (m2.predict(x, reference_quirks=False) == ids).all()
    assert model.get_training_status()["last_completed_layer"] == 2
    # resume: drop the last layer's checkpoint, retrain only that layer
    (tmp_path / "ck" / "layer_2_checkpoint.npz").unlink()
    seeded(43)
    m3 = HierarchicalRQKMeans(HierarchicalRQKMeansConfig(**SMALL), checkpoint_dir=str(tmp_path / "ck"), device=DEV)
    r3 = m3.train(x, resume=True)
    assert (r3["cluster_ids"][0].cpu().numpy() == ids[:, 0]).all()
    assert (r3["cluster_ids"][1].cpu().numpy() == ids[:, 1]).all()


def test_hierarchical_errors():
    model = HierarchicalRQKMeans(HierarchicalRQKMeansConfig(**SMALL), device=DEV)
    with pytest.raises(RuntimeError):
        model.predict(np.zeros((4, 512), np.float32))
    with pytest.raises(ValueError):
        model.train(np.zeros((4, 100), np.float32))


def test_simplified_train_jsonl(tmp_path):
    x = synth.small_mixture(1500, m=64, seed=21)
    sids = [f"s{i:05d}" for i in range(len(x))]
    csv_path = tmp_path / "vec.csv"
    rq_io.write_song_vectors(str(csv_path), sids, x)
    seeded(42)
    model = SimplifiedHierarchicalRQ(HierarchicalRQKMeansConfig(**SMALL), device=DEV)
    model.train(str(csv_path))
    ids = np.array([model.semantic_ids[s] for s in sids])
    assert ids.shape == (1500, 3) and ids[:, 0].max() < 8 and ids[:, 1].max() < 8 and ids[:, 2].max() < 32
    out = tmp_path / "ids.jsonl"
    model.save_semantic_ids(str(out))
    assert out.read_bytes() == rq_io.semantic_id_lines(sids, ids)
    model.save_model(str(tmp_path / "m.npz"))
    m2 = SimplifiedHierarchicalRQ.load_model(str(tmp_path / "m.npz"), device=DEV)
    assert torch.equal(m2.final_layer_centers.cpu(), model.final_layer_centers.cpu())


def test_sharded_lloyd_on_gpu_world1(tmp_path):
    """The default (GPU kernel) local steps of the row-sharded fit, one rank over RCCL, against the
    single-process GPU KMeans with the same seeds."""
    import torch.distributed as dist
    from generative_ranking_recommender_amd.distributed import ShardedLloyd
    if not dist.is_initialized():
        dist.init_process_group("nccl", init_method=f"file://{tmp_path}/pg", rank=0, world_size=1)
    try:
        x = torch.from_numpy(synth.small_mixture(5000, m=20, seed=2)).to(DEV)
        seeded(3)
        sl = ShardedLloyd(24, x, len(x))
        a = sl.fit(iter_limit=5)
        seeded(3)
        km = KMeans(n_clusters=24, device=DEV, balanced=False)
        a_ref = km.fit(x, iter_limit=5)
        assert (a.cpu() == a_ref).all()
        torch.testing.assert_close(sl.cluster_centers, km.cluster_centers, rtol=1e-6, atol=1e-6)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("n_cand", [300, 65536])
def test_greedy_match_matches_numpy(n_cand):
    """rqsid_greedy_match (the match-matrix builders' greedy unique-nearest step) against a numpy
    restatement of _assign_last_match_matrix :1022-1038, up to the largest accepted column count
    (65536 columns = 64 KiB of dynamic LDS per group)."""
    rng = np.random.default_rng(n_cand)
    sizes = [5, 0, 9, 3]
    sub_off = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int32)
    dist = rng.random((int(sub_off[-1]), n_cand), dtype=np.float32)
    dist[2, :] = dist[1, :]  # duplicate rows: the second takes the next-nearest free column
    max_take = 4
    got, nsel = ops.greedy_match(torch.from_numpy(dist).cuda(), torch.from_numpy(sub_off).cuda(), max_take)
    got = got.cpu().numpy()
    want = np.zeros((len(sizes), n_cand), dtype=np.uint8)
    for g in range(len(sizes)):
        used = np.zeros(n_cand, bool)
        for r in range(sub_off[g], sub_off[g] + min(sizes[g], max_take)):
            d = np.where(used, np.inf, dist[r])
            c = int(np.argmin(d))
            used[c] = True
            want[g, c] = 1
    assert (got == want).all()
    assert (nsel.cpu().numpy() == want.sum(1)).all()


def _gpu_sharded_auction_worker(rank, world, port, w16, out):
    import os
    import torch.distributed as dist
    from generative_ranking_recommender_amd.distributed import GpuAuctionPasses, ShardedAuction, shard_bounds
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    n = w16.shape[1]
    s, e = shard_bounds(n, rank, world)
    try:
        w = torch.from_numpy(np.ascontiguousarray(w16[:, s:e])).to(DEV)
        a, rounds = ShardedAuction().run(GpuAuctionPasses(w, n), n, w16.shape[0], max_rounds=2500)
        out.put((rank, a.cpu().numpy().astype(np.int64), rounds))
    except Exception as exc:  # report instead of leaving the parent waiting
        out.put((rank, None, repr(exc)))
    dist.destroy_process_group()


# per-rank shares of a multiple of 4 jobs take the 8-byte-load passes; 3002 (1501 per rank) the 2-byte ones;
# N % K != 0 runs 1002 rounds, so the list phase (from round 32; 16 at K >= 1024) carries most of them
@pytest.mark.parametrize("dlist", ["1", "0"])
@pytest.mark.parametrize("n,k,levels", [(3000, 16, 7), (640, 64, 1000), (3002, 16, 7), (40001, 128, 0),
                                        (24002, 1024, 0)])
def test_sharded_auction_gpu_passes_two_ranks(n, k, levels, dlist, monkeypatch):
    """Two ranks on one GPU (gloo collectives over device tensors), each running the rqsid_dauction_*
    passes on its row block: the concatenation equals the single-process GPU auction (pinned to the
    oracle above), ties across the shard boundary included, with the row-sharded bid lists (dlist "1":
    list rounds from per-rank lists, void slots re-run as sweeps) and without them (every round sweeps).
    levels 0: fp16 distances of unit rows to centres (the training scores), otherwise heavily tied levels."""
    import socket
    import torch.multiprocessing as mp
    monkeypatch.setenv("RQSID_DAUCTION_LIST", dlist)
    rng = np.random.default_rng(n)
    if levels:
        w16 = (-rng.integers(1, levels + 1, size=(k, n)).astype(np.float32) * np.float32(0.37)).astype(np.float16)
    else:
        x = synth.small_mixture(n, m=max(64, k), seed=n)
        x /= np.linalg.norm(x, axis=1, keepdims=True)
        c = x[rng.choice(n, k, replace=False)] * np.float32(0.9)
        d = np.sqrt(np.maximum(((x[:, None, :] - c[None]) ** 2).sum(-1), 0)) if n * k <= 4_000_000 else None
        if d is None:
            d = np.sqrt(np.maximum((x ** 2).sum(1)[:, None] + (c ** 2).sum(1)[None] - 2 * x @ c.T, 0))
        w16 = np.ascontiguousarray((-d.T).astype(np.float16))
    sock = socket.socket()
    sock.bind(("127.0.0.1", 0))
    port = sock.getsockname()[1]
    sock.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_gpu_sharded_auction_worker, args=(r, 2, port, w16, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=150) for _ in range(2)], key=lambda r: r[0])
    for p in procs:
        p.join(60)
    assert all(r[1] is not None for r in res), res
    got = np.concatenate([r[1] for r in res])
    want, r_want = ops.auction(torch.from_numpy(w16).to(DEV))
    assert np.array_equal(got, want.cpu().numpy())
    assert res[0][2] == res[1][2] == r_want


def test_sharded_balanced_fit_world1(tmp_path):
    """ShardedLloyd(balanced=True) over RCCL with one rank == KMeans(balanced=True).fit (same draws)."""
    import torch.distributed as dist
    from generative_ranking_recommender_amd.distributed import ShardedLloyd
    if not dist.is_initialized():
        dist.init_process_group("nccl", init_method=f"file://{tmp_path}/pg", rank=0, world_size=1)
    try:
        x = torch.from_numpy(synth.small_mixture(3000, m=20, seed=2)).to(DEV)
        seeded(5)
        sl = ShardedLloyd(24, x, len(x), balanced=True)
        a = sl.fit(iter_limit=3)
        seeded(5)
        km = KMeans(n_clusters=24, device=DEV, balanced=True)
        a_ref = km.fit(x, iter_limit=3)
        assert (a.cpu() == a_ref).all()
        torch.testing.assert_close(sl.cluster_centers, km.cluster_centers, rtol=1e-6, atol=1e-6)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("n,k,half", [(200_000, 128, False), (100_000, 1280, True), (60_001, 1280, True),
                                      (800_001, 128, True), (1_100_001, 128, False)])
def test_auction_bid_list_equals_sweep(n, k, half, monkeypatch):
    """List rounds (auction_seg.hip sa_list_round_kernel: a worker's threshold, tie ranks and bids from the jobs a
    sweep round listed, keys >= its threshold - 64, while the threshold stays above that base) give the sweep's
    assignment and round count (RQSID_AUCTION_LIST=0) on the level-0 (K = 128) and candidate-fit (K = 1280,
    fp16 cdist) shapes, with the retention (round < 100) and leftover (round > 1000, N % K != 0) rules; above
    8192 jobs per worker (one segment) the default is the multi-block form (sa_mlist_*), checked against the
    sweep and the one-block form (RQSID_AUCTION_LIST=2); lists are built from round 32 on; the list rounds gather a
    packed {winner, cost} word per listed job (RQSID_LIST_JS=0, mode "1s": the two arrays); times all (printed)."""
    import time
    x = synth.small_mixture(n, m=3000, seed=k)
    x /= np.linalg.norm(x, axis=1, keepdims=True)
    xg = torch.from_numpy(x.astype(np.float32)).to(DEV)
    c = xg[torch.from_numpy(np.random.default_rng(k).choice(n, k, replace=False)).to(DEV)] * 0.9
    w = ops.auction_scores(xg, c, half=half)
    out = {}
    for mode in ("1", "1s", "0", "2"):
        monkeypatch.setenv("RQSID_AUCTION_LIST", mode[0])
        monkeypatch.setenv("RQSID_LIST_JS", "0" if mode == "1s" else "1")  # 1s: winner and cost gathered separately
        ops.auction(w)
        torch.cuda.synchronize()
        t = time.perf_counter()
        a, rounds = ops.auction(w)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t
        out[mode] = (a.cpu().numpy(), rounds)
        print(f"n={n} k={k} list={mode}: {rounds} rounds, {dt * 1e3 / rounds:.3f} ms/round")
    assert np.array_equal(out["1"][0], out["0"][0]) and out["1"][1] == out["0"][1]
    assert np.array_equal(out["1s"][0], out["0"][0]) and out["1s"][1] == out["0"][1]
    assert np.array_equal(out["2"][0], out["0"][0]) and out["2"][1] == out["0"][1]
    if n % k:
        assert out["1"][1] == 1002


def test_group_fits_k512_certified():
    """configs[4]'s match-matrix group fits (hierarchical_rq_kmeans.py:1011-1018 with need[2] = 512: groups of
    >= 1024 rows fit KMeans(512, balanced).fit, half=False) through the lockstep path (fit_segments), every
    iteration of both segments certified against the oracle (tests/_certify.py)."""
    from generative_ranking_recommender_amd import balancekmeans as bk
    from tests import _certify
    x = synth.small_mixture(2560, m=300, seed=77)
    x /= np.linalg.norm(x, axis=1, keepdims=True)
    sizes = [1024, 1536]
    seeded(5)
    inits = [[bk.init_indices(n, 512)] for n in sizes]
    rec = _certify.Recorder()
    bk.TRACE = rec
    try:
        c, a = bk.fit_segments(torch.from_numpy(x.astype(np.float32)).to(DEV), sizes, 512, [3, 3], inits, half=False)
    finally:
        bk.TRACE = None
    st = _certify.certify_trace(rec.events)
    assert st["auctions"] == st["steps"] and 2 <= st["steps"] <= 6
    a = a.cpu().numpy()
    for s0, s1 in ((0, 1024), (1024, 2560)):
        assert np.bincount(a[s0:s1], minlength=512).max() == (s1 - s0) // 512  # N % K == 0: exactly balanced
