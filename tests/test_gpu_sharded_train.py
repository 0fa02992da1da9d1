"""Multi-GPU training path: the row-/segment-sharded HierarchicalRQKMeans
training, the sharded predict and the SemanticIDTrainer driver, run by two ranks (gloo collectives;
both ranks share the box's one GPU) against the single-process run with the same seeds.  They must be
the same model: IDs, match matrix and jsonl bytes identical, centres within 1e-6."""
import os
import socket
import types

import numpy as np
import pytest
import torch

from generative_ranking_recommender_amd import io as rq_io
from generative_ranking_recommender_amd import synth
from generative_ranking_recommender_amd.hierarchical_rq_kmeans import HierarchicalRQKMeans, HierarchicalRQKMeansConfig
from generative_ranking_recommender_amd.train_semantic_ids import SemanticIDTrainer

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)
CFG = dict(layer_clusters=[8, 16, 16], need_clusters=[8, 8, 8], embedding_dim=512, iter_limit=5)


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _seeded(seed):
    np.random.seed(seed)
    torch.manual_seed(seed)


def _train_worker(rank, world, port, x, seed, out):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        _seeded(seed)
        m = HierarchicalRQKMeans(HierarchicalRQKMeansConfig(**CFG), device=DEV, group=dist.group.WORLD)
        res = m.train(x, resume=False)
        ids = np.stack([t.cpu().numpy() for t in res["cluster_ids"]], 1)
        pred = m.predict(x, reference_quirks=False)
        quirky = m.predict(x)
        out.put((rank, ids, [c.cpu().numpy() for c in m.cluster_centers_list], np.asarray(m.match_matrices[0]),
                 pred, quirky, np.random.get_state()[1].copy(), torch.get_rng_state().numpy().copy()))
    except Exception as exc:  # report instead of leaving the parent waiting
        import traceback
        out.put((rank, None, traceback.format_exc()))
    dist.destroy_process_group()


def _run(target, world, args):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=target, args=(r, world, port) + args + (q,)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=240) for _ in range(world)], key=lambda r: r[0])
    for p in procs:
        p.join(60)
    for r in res:
        assert r[1] is not None, r[2]
    return res


def test_sharded_train_and_predict_equal_single_process():
    x = synth.small_mixture(2500, m=64, seed=21)
    seed = 42
    _seeded(seed)
    ref = HierarchicalRQKMeans(HierarchicalRQKMeansConfig(**CFG), device=DEV)
    rr = ref.train(x, resume=False)
    ids_ref = np.stack([t.cpu().numpy() for t in rr["cluster_ids"]], 1)
    np_state, t_state = np.random.get_state()[1].copy(), torch.get_rng_state().numpy().copy()
    pred_ref = ref.predict(x, reference_quirks=False)
    quirky_ref = ref.predict(x)
    for rank, ids, cents, match, pred, quirky, nps, ts in _run(_train_worker, 2, (x, seed)):
        assert np.array_equal(ids, ids_ref), f"rank {rank}: IDs differ"
        for c, cr in zip(cents, ref.cluster_centers_list):
            np.testing.assert_allclose(c, cr.cpu().numpy(), rtol=1e-6, atol=1e-6)
        assert np.array_equal(match, np.asarray(ref.match_matrices[0]))
        assert np.array_equal(pred, pred_ref) and np.array_equal(pred, ids_ref)
        assert np.array_equal(quirky, quirky_ref)
        assert np.array_equal(nps, np_state) and np.array_equal(ts, t_state), "RNG state differs"


def _trainer_cfg(root, csv_path):
    return types.SimpleNamespace(
        output_dir=os.path.join(root, "outputs"), model_dir=os.path.join(root, "models"),
        h_rqkmeans_test=HierarchicalRQKMeansConfig(**CFG), h_rqkmeans=None,
        data=types.SimpleNamespace(song_vectors_file=csv_path,
                                   semantic_ids_file=os.path.join(root, "outputs", "semantic_id",
                                                                  "song_semantic_ids.jsonl")))


def _trainer_worker(rank, world, port, root, csv_path, seed, out):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        _seeded(seed)
        SemanticIDTrainer(_trainer_cfg(root, csv_path), use_test_config=True, device=DEV,
                          group=dist.group.WORLD).train(resume=False)
        out.put((rank, True, None))
    except Exception:
        import traceback
        out.put((rank, None, traceback.format_exc()))
    dist.destroy_process_group()


def test_sharded_semantic_id_trainer_writes_the_single_process_files(tmp_path):
    """train_semantic_ids.py:133-365 over two ranks: rank 0 writes song_semantic_ids.jsonl,
    training_config.json and training_statistics.json byte-identical to the single-process driver's."""
    x = synth.small_mixture(1800, m=64, seed=5)
    sids = [f"song{i}" for i in range(len(x))]
    csv_path = str(tmp_path / "vec.csv")
    rq_io.write_song_vectors(csv_path, sids, x)
    one, two = str(tmp_path / "one"), str(tmp_path / "two")
    _seeded(7)
    SemanticIDTrainer(_trainer_cfg(one, csv_path), use_test_config=True, device=DEV).train(resume=False)
    _run(_trainer_worker, 2, (two, csv_path, 7))
    for rel in ("outputs/semantic_id/song_semantic_ids.jsonl", "outputs/semantic_id/training_config.json",
                "outputs/semantic_id/training_statistics.json"):
        a = open(os.path.join(one, rel), "rb").read()
        b = open(os.path.join(two, rel), "rb").read()
        assert a == b, rel


def _ckpt_worker(rank, world, port, x, seed, ck, np_state, t_state, resume, out):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        _seeded(seed)
        if np_state is not None:
            np.random.set_state(np_state)
            torch.set_rng_state(t_state)
        m = HierarchicalRQKMeans(HierarchicalRQKMeansConfig(**CFG), checkpoint_dir=ck, device=DEV,
                                 group=dist.group.WORLD)
        res = m.train(x, resume=resume)
        out.put((rank, np.stack([t.cpu().numpy() for t in res["cluster_ids"]], 1),
                 [c.cpu().numpy() for c in m.cluster_centers_list], np.asarray(m.match_matrices[0])))
    except Exception:
        import traceback
        out.put((rank, None, traceback.format_exc()))
    dist.destroy_process_group()


def test_resume_from_sharded_checkpoints_equals_uninterrupted_run(tmp_path, monkeypatch):
    """a sharded run's checkpoints (rank 0 writes them, without residual data) resumed after the
    last layer's checkpoint is lost -- by two ranks and by a single process, both rebuilding the residual
    chain from ids and centres (_residual_chain) -- give the uninterrupted run's IDs, centres and match
    matrix.  The generators are put where the uninterrupted run had them when its last layer started."""
    import shutil
    x = synth.small_mixture(2500, m=64, seed=21)
    state = {}
    orig = HierarchicalRQKMeans._train_last_layer

    def recording(self, X, layer):
        state["np"], state["torch"] = np.random.get_state(), torch.get_rng_state()
        return orig(self, X, layer)
    monkeypatch.setattr(HierarchicalRQKMeans, "_train_last_layer", recording)
    _seeded(42)
    ref = HierarchicalRQKMeans(HierarchicalRQKMeansConfig(**CFG), device=DEV)
    rr = ref.train(x, resume=False)
    monkeypatch.setattr(HierarchicalRQKMeans, "_train_last_layer", orig)
    ids_ref = np.stack([t.cpu().numpy() for t in rr["cluster_ids"]], 1)
    cents_ref = [c.cpu().numpy() for c in ref.cluster_centers_list]
    match_ref = np.asarray(ref.match_matrices[0])

    def same(ids, cents, match):
        assert np.array_equal(ids, ids_ref)
        for c, cr in zip(cents, cents_ref):
            np.testing.assert_allclose(c, cr, rtol=1e-6, atol=1e-6)
        assert np.array_equal(match, match_ref)

    ck = str(tmp_path / "ck")
    for r in _run(_ckpt_worker, 2, (x, 42, ck, None, None, False)):
        same(*r[1:])
    os.remove(os.path.join(ck, "layer_2_checkpoint.npz"))
    ck2 = str(tmp_path / "ck2")
    shutil.copytree(ck, ck2)
    for r in _run(_ckpt_worker, 2, (x, 42, ck, state["np"], state["torch"], True)):
        same(*r[1:])
    np.random.set_state(state["np"])
    torch.set_rng_state(state["torch"])
    m = HierarchicalRQKMeans(HierarchicalRQKMeansConfig(**CFG), checkpoint_dir=ck2, device=DEV)
    res = m.train(x, resume=True)
    same(np.stack([t.cpu().numpy() for t in res["cluster_ids"]], 1), [c.cpu().numpy() for c in m.cluster_centers_list],
         np.asarray(m.match_matrices[0]))


def test_encoder_cache_follows_codebook_changes():
    """the cached fused encoder is rebuilt when a codebook is replaced or edited in place."""
    x = synth.small_mixture(2500, m=64, seed=21)
    _seeded(42)
    m = HierarchicalRQKMeans(HierarchicalRQKMeansConfig(**CFG), device=DEV)
    m.train(x, resume=False)
    a = m.predict(x[:300], reference_quirks=False)
    c0 = m.cluster_centers_list[0]
    c0[[0, 1]] = c0[[1, 0]].clone()  # in place: ids 0 and 1 of level 0 swap
    b = m.predict(x[:300], reference_quirks=False)
    assert np.array_equal(np.where(a[:, 0] == 0, 1, np.where(a[:, 0] == 1, 0, a[:, 0])), b[:, 0])
    restored = c0.clone()
    restored[[0, 1]] = c0[[1, 0]]
    m.cluster_centers_list = [restored] + m.cluster_centers_list[1:]  # replaced by a new tensor: the original
    assert np.array_equal(m.predict(x[:300], reference_quirks=False), a)
