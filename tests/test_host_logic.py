"""Host-side logic that needs no GPU: config validation, the adaptive iteration budget, checkpoint
files, the CSV reader and the jsonl writer (byte-exact against the reference's golden)."""
import json

import numpy as np
import pytest

from generative_ranking_recommender_amd import io as rq_io
from generative_ranking_recommender_amd.hierarchical_rq_kmeans import (CheckpointManager, HierarchicalRQKMeansConfig,
                                                                      adaptive_iter_limit)
from oracle import rq_oracle as O


def test_config_defaults_and_validation():
    c = HierarchicalRQKMeansConfig(layer_clusters=[4, 8, 8], need_clusters=[4, 4, 4], embedding_dim=16)
    assert c.group_dims == [16] and c.hierarchical_weights == [[1.0]] * 3
    c = HierarchicalRQKMeansConfig(layer_clusters=[4], need_clusters=[4], embedding_dim=16, group_dims=[8, 8],
                                   hierarchical_weights=0.3)
    assert c.hierarchical_weights == [[0.5, 0.5]]
    with pytest.raises(ValueError):
        HierarchicalRQKMeansConfig(layer_clusters=[4], need_clusters=[4], embedding_dim=16, group_dims=[8, 4])
    with pytest.raises(ValueError):
        HierarchicalRQKMeansConfig(layer_clusters=[4, 4], need_clusters=[4, 4], embedding_dim=16,
                                   hierarchical_weights=[[1.0]])
    with pytest.raises(ValueError):
        HierarchicalRQKMeansConfig(layer_clusters=[4], need_clusters=[4], embedding_dim=16, group_dims=[8, 8],
                                   hierarchical_weights=[[1.0]])


def test_adaptive_iter_limit_matches_oracle():
    for n in (100, 4999, 5000, 9999, 20000, 60000, 100000, 600000, 2_000_000, 10_000_000):
        for k in (32, 128, 300, 600, 1280):
            for layer in (0, 1, 2):
                for sub in (False, True):
                    assert adaptive_iter_limit(n, k, layer, 100, sub) == O.adaptive_iter_limit(n, k, layer, 100, sub)
    # the survey's measured points
    assert adaptive_iter_limit(100_000, 128, 0) == 100 and adaptive_iter_limit(1_000_000, 128, 0) == 150
    assert [adaptive_iter_limit(n, 128, 1, is_sub_cluster=True) for n in (100_000, 1_000_000, 10_000_000)] == [36, 36, 36]


def test_checkpoint_manager_roundtrip(tmp_path):
    cm = CheckpointManager(str(tmp_path))
    ids = np.arange(10)
    cen = np.ones((4, 3), np.float32)
    cm.save_layer_checkpoint(0, ids, np.zeros((10, 3), np.float32), cen)
    cm.save_layer_checkpoint(1, ids, np.zeros((10, 3), np.float32), cen, match_matrix=[[1, 0], [0, 1]])
    assert cm.get_last_completed_layer() == 1
    assert not list(tmp_path.glob("*.tmp*"))
    cm.save_metadata({"num_layers": 3})
    assert cm.load_metadata() == {"num_layers": 3}
    cm.clear_checkpoints()
    assert cm.get_last_completed_layer() == -1 and cm.load_metadata() is None


def test_csv_reader_rules(tmp_path):
    p = tmp_path / "v.csv"
    good = np.random.default_rng(0).standard_normal((3, 4)).astype(np.float32)
    lines = [f"a,{','.join(repr(float(v)) for v in good[0])}",
             "short",                       # < 2 fields: skipped
             "b,1,2,x,4",                   # non-numeric: skipped
             "c,1,2,3",                     # wrong dimension: skipped
             f"d,{','.join(repr(float(v)) for v in good[1])}",
             f"e,{','.join(repr(float(v)) for v in good[2])}"]
    p.write_text("\n".join(lines) + "\n")
    ids, x = rq_io.load_song_vectors(str(p), 4)
    assert ids == ["a", "d", "e"] and x.dtype == np.float32 and np.array_equal(x, good)
    ids, x = rq_io.load_song_vectors(str(p), 4, layer_clusters=[128, 1280])
    assert x.dtype == np.float16 and np.array_equal(x, good.astype(np.float16))
    ids, _ = rq_io.load_song_vectors(str(p), 4, limit=2)
    assert ids == ["a"]
    with pytest.raises(ValueError):
        rq_io.load_song_vectors(str(p), 7)
    with pytest.raises(FileNotFoundError):
        rq_io.load_song_vectors(str(tmp_path / "missing.csv"), 4)


def test_jsonl_writer_matches_reference_bytes(golden, tmp_path):
    g = golden("simplified")
    sids = [f"s{i:05d}" for i in range(len(g["ids"]))]
    raw = rq_io.semantic_id_lines(sids, g["ids"])
    assert raw[:len(bytes(g["jsonl_head"]))] == bytes(g["jsonl_head"])
    out = tmp_path / "x.jsonl"
    n_unique = rq_io.write_semantic_ids(str(out), {s: [int(v) for v in r] for s, r in zip(sids, g["ids"])})
    assert out.read_bytes() == raw and n_unique == len({tuple(r) for r in g["ids"]})


def test_statistics_side_file():
    sem = {"a": [0, 1, 2], "b": [0, 1, 3], "c": [1, 0, 2]}
    st = rq_io.semantic_id_statistics(sem, [2, 2, 4])
    assert st["total_songs"] == 3 and st["unique_semantic_ids"] == 3
    l0 = st["layer_statistics"][0]
    assert l0["unique_clusters"] == 2 and l0["cluster_distribution"]["max"] == 2
    json.dumps(st)


def test_random_fill_blocks_equal_the_reference_loop():
    """hierarchical :1041-1048 / simplified :294-297 one draw at a time vs the block-drawn restatement:
    same row, same numpy generator state afterwards."""
    import numpy as np
    from generative_ranking_recommender_amd.hierarchical_rq_kmeans import random_fill

    def loop(row, need):
        have = int(row.sum())
        while have < need:
            r = np.random.randint(row.shape[0])
            if not row[r]:
                row[r] = 1
                have += 1

    rng = np.random.default_rng(0)
    for n_cand, need, pre in [(2560, 256, 3), (32, 8, 0), (300, 299, 10), (64, 64, 63), (5120, 512, 500), (16, 4, 4)]:
        base = np.zeros(n_cand, np.uint8)
        base[rng.choice(n_cand, pre, replace=False)] = 1
        a, b = base.copy(), base.copy()
        np.random.seed(n_cand + need)
        loop(a, need)
        sa = np.random.get_state()
        np.random.seed(n_cand + need)
        random_fill(b, need)
        sb = np.random.get_state()
        assert np.array_equal(a, b)
        assert np.array_equal(sa[1], sb[1]) and sa[2] == sb[2]
