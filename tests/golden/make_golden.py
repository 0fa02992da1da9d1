"""Capture golden vectors by running the REFERENCE implementation in this container.

Run ONLY in the build container (``/root/reference`` does not exist on the GPU
box)::

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py

It imports the read-only reference with the harness of SURVEY.md Appendix B:

* a ``numba`` stub in ``sys.modules`` (``balancekmeans/__init__.py:6`` imports
  ``soft_dtw_cuda``, which imports numba; soft-DTW itself is never executed);
* ``HierarchicalRQKMeans._calculate_safe_batch_size`` patched to a constant
  (``hierarchical_rq_kmeans.py:252`` calls ``torch.cuda.mem_get_info``
  unconditionally, which raises on a CPU-only host; batch size only changes
  chunking, not arithmetic).

Outputs are small ``.npz`` fixtures next to this script. Inputs are regenerated
from seeds by ``generative_ranking_recommender_amd.synth`` in the tests and
checked against the sha256 stored here, so the fixtures stay small. Nothing in
the package imports this file.
"""
from __future__ import annotations

import csv
import io
import json
import os
import sys
import tempfile
import types
from pathlib import Path

import numpy as np
import torch

HERE = Path(__file__).resolve().parent
REPO = HERE.parent.parent
sys.path.insert(0, str(REPO))
from generative_ranking_recommender_amd import synth  # noqa: E402

# --- reference harness --------------------------------
nb, cu = types.ModuleType("numba"), types.ModuleType("numba.cuda")


def _d(*a, **k):
    return a[0] if a and callable(a[0]) and not k else (lambda f: f)


nb.jit = cu.jit = _d
nb.cuda = cu
sys.modules.update({"numba": nb, "numba.cuda": cu})
sys.path.insert(0, "/root/reference")
from src.semantic_id_generator import balancekmeans as ref_bk  # noqa: E402
from src.semantic_id_generator import hierarchical_rq_kmeans as ref_h  # noqa: E402
from src.semantic_id_generator import simplified_semantic_id_generator as ref_s  # noqa: E402

ref_h.HierarchicalRQKMeans._calculate_safe_batch_size = staticmethod(
    lambda X, n, d, initial_batch_size=200000: 200000)
torch.set_num_threads(8)


def seed_all(s):
    np.random.seed(s)
    torch.manual_seed(s)


def save(name, **arrays):
    np.savez_compressed(HERE / f"{name}.npz", **arrays)
    print("wrote", name, {k: getattr(v, "shape", v) for k, v in arrays.items()})


# --- G1: fp32 assignment (pairwise_distance_full + argmin) -------------------
def g_assign():
    X = synth.small_mixture(4096, m=64, seed=11)
    cidx = np.random.default_rng(5).choice(4096, 128, replace=False)
    C = X[cidx].copy()
    dist = ref_bk.pairwise_distance_full(torch.from_numpy(X), torch.from_numpy(C))
    ids = torch.argmin(dist, dim=1).numpy()
    km = ref_bk.KMeans(n_clusters=128, cluster_centers=torch.from_numpy(C))
    ids_pred = km.predict(torch.from_numpy(X)).numpy()
    assert (ids == ids_pred).all()
    # tie case: duplicated centres and rows sitting exactly on centres
    C2 = C.copy()
    C2[77] = C2[5]
    C2[100] = C2[3]
    C2[127] = C2[0]
    X2 = X[:512].copy()
    X2[0], X2[1], X2[2] = C2[5], C2[3], C2[0]
    ids_tie = ref_bk.KMeans(n_clusters=128, cluster_centers=torch.from_numpy(C2)).predict(
        torch.from_numpy(X2)).numpy()
    save("assign", x_sha=np.array(synth.sha256(X)), cidx=cidx, ids=ids.astype(np.int64),
         dmin=dist.min(dim=1).values.numpy(), dist_head=dist[:64].numpy(),
         ids_tie=ids_tie.astype(np.int64))


# --- G-residual: _compute_residuals_with_centers (hier.) / _get_residuals (simplified)
def g_residual():
    X = synth.small_mixture(4096, m=64, seed=11)
    C = X[np.random.default_rng(5).choice(4096, 128, replace=False)].copy()
    ids = torch.argmin(ref_bk.pairwise_distance_full(torch.from_numpy(X), torch.from_numpy(C)), 1)
    out = {}
    for tag, gd in (("g512", [512]), ("g128_384", [128, 384])):
        cfg = ref_h.HierarchicalRQKMeansConfig(layer_clusters=[128], need_clusters=[128],
                                               embedding_dim=512, group_dims=gd)
        m = ref_h.HierarchicalRQKMeans(cfg, device=torch.device("cpu"))
        r = m._compute_residuals_with_centers(torch.from_numpy(X), ids, torch.from_numpy(C)).numpy()
        out[f"res_{tag}_head"] = r[:256]
        out[f"res_{tag}_sha"] = np.array(synth.sha256(r))
    km = ref_bk.KMeans(n_clusters=128, cluster_centers=torch.from_numpy(C))
    s = ref_s.SimplifiedHierarchicalRQ.__new__(ref_s.SimplifiedHierarchicalRQ)
    s.device = torch.device("cpu")
    rs = s._get_residuals(torch.from_numpy(X), km).numpy()
    out["res_plain_head"] = rs[:256]
    out["res_plain_sha"] = np.array(synth.sha256(rs))
    save("residual", ids=ids.numpy().astype(np.int64), **out)


# --- G4: Lloyd update incl. an empty cluster (fit, balanced=False, 1 iteration)
def g_update():
    base = synth.small_mixture(256, m=8, seed=13)
    X = np.concatenate([base, base[:64]], 0)  # exact duplicate rows -> tied centres
    res = {}
    for s in (0, 1, 2, 3):
        seed_all(100 + s)
        km = ref_bk.KMeans(n_clusters=24, balanced=False)
        a = km.fit(torch.from_numpy(X), iter_limit=1, tqdm_flag=False)
        res[f"assign_{s}"] = a.numpy().astype(np.int64)
        res[f"centers_{s}"] = km.cluster_centers.numpy()
    save("update", x_sha=np.array(synth.sha256(X)), **res)


# --- G5: auction_lap_half ----------------------------------------------------
def g_auction():
    res = {}
    cases = {"n64k8": (64, 8, 17), "n67k8": (67, 8, 18), "n1000k16": (1000, 16, 19),
             "n5k8": (5, 8, 20), "n96k8": (96, 8, 21)}
    for tag, (n, k, seed) in cases.items():
        X = synth.small_mixture(n, d=32, m=6, seed=seed)
        C = synth.small_mixture(k, d=32, m=6, seed=seed + 100)
        dist = ref_bk.pairwise_distance_full(torch.from_numpy(X), torch.from_numpy(C))
        out = ref_bk.auction_lap_half(-dist)
        res[f"dist_{tag}"] = dist.numpy()
        res[f"out_{tag}"] = out.numpy().astype(np.int64)
    save("auction", **res)


# --- G5b: auction_lap_full (fp32; only predict(balanced=True) reaches it) -------
def g_auction_full():
    res = {}
    cases = {"n64k8": (64, 8, 17), "n67k8": (67, 8, 18), "n1000k16": (1000, 16, 19),
             "n5k8": (5, 8, 20), "n96k8": (96, 8, 21)}
    for tag, (n, k, seed) in cases.items():
        X = synth.small_mixture(n, d=32, m=6, seed=seed)
        C = synth.small_mixture(k, d=32, m=6, seed=seed + 100)
        dist = ref_bk.pairwise_distance_full(torch.from_numpy(X), torch.from_numpy(C))
        out = ref_bk.auction_lap_full(-dist)
        res[f"dist_{tag}"] = dist.numpy()
        res[f"out_{tag}"] = out.numpy().astype(np.int64)
    save("auction_full", **res)


# --- G-half: pairwise_distance_half (fp16 cdist + clamp at 1e-5, the K >= 512 auction input) ---
def half_inputs():
    """normalised-residual-like rows (unit norm) and 520 centres, five of them equal to rows (zero
    distance -> the clamp at 1e-5); a second, unnormalised set at another scale"""
    x = synth.small_mixture(640, m=32, seed=41)
    x /= np.linalg.norm(x, axis=1, keepdims=True)
    c = synth.small_mixture(520, m=32, seed=42)
    c /= np.linalg.norm(c, axis=1, keepdims=True)
    c[:5] = x[:5]
    x2 = synth.small_mixture(300, m=16, seed=43) * np.float32(3.0)
    c2 = synth.small_mixture(600, m=16, seed=44) * np.float32(3.0)
    return x.astype(np.float32), c.astype(np.float32), x2.astype(np.float32), c2.astype(np.float32)


def g_dist_half():
    """The reference's CPU branch of pairwise_distance_half computes ``int(free_mem / ...)`` with
    ``free_mem = float('inf')`` (:552-553), which raises OverflowError: the function only runs on CUDA
    as written.  Like the batch-size patch above, the harness makes that batch size finite: the module's
    global name ``float`` is shadowed so ``float('inf')`` gives 1e18 (only the chunking of the loop at
    :563-569 depends on it; the arithmetic is the reference's own torch.cdist + clamp on fp16 tensors)."""
    ref_bk.float = lambda v: 1e18 if v == "inf" else float(v)
    x, c, x2, c2 = half_inputs()
    d = ref_bk.pairwise_distance_half(torch.from_numpy(x), torch.from_numpy(c))
    d2 = ref_bk.pairwise_distance_half(torch.from_numpy(x2), torch.from_numpy(c2))
    assert d.dtype == torch.float16
    del ref_bk.float
    save("dist_half", x_sha=np.array(synth.sha256(x)), c_sha=np.array(synth.sha256(c)),
         x2_sha=np.array(synth.sha256(x2)), c2_sha=np.array(synth.sha256(c2)),
         d=d.numpy().view(np.uint16), d2=d2.numpy().view(np.uint16))


# --- G6: fit_by_min_loss / fit (balanced) trajectories ----------------------
def g_fit():
    X = synth.small_mixture(512, m=16, seed=23)
    seed_all(3)
    km = ref_bk.KMeans(n_clusters=8, balanced=True)
    km.fit_by_min_loss(torch.from_numpy(X), target_nodes_num=64, iter_limit=12, tqdm_flag=False)
    c_fbml = km.cluster_centers.numpy()
    seed_all(4)
    km2 = ref_bk.KMeans(n_clusters=8, balanced=True)
    a2 = km2.fit(torch.from_numpy(X), iter_limit=5, tqdm_flag=False)
    seed_all(5)
    km3 = ref_bk.KMeans(n_clusters=8, balanced=False)
    a3 = km3.fit(torch.from_numpy(X), iter_limit=0, tqdm_flag=False)
    save("fit", x_sha=np.array(synth.sha256(X)), fbml_centers=c_fbml,
         fit_bal_assign=a2.numpy().astype(np.int64), fit_bal_centers=km2.cluster_centers.numpy(),
         fit_unbal_assign=a3.numpy().astype(np.int64), fit_unbal_centers=km3.cluster_centers.numpy())


SMALL_CFG = dict(layer_clusters=[8, 16, 16], need_clusters=[8, 8, 8], embedding_dim=512, iter_limit=5)


def write_csv(path, ids, X):
    with open(path, "w", newline="") as f:
        w = csv.writer(f)
        for sid, row in zip(ids, X):
            w.writerow([sid] + [repr(float(v)) for v in row])


# --- G2: SimplifiedHierarchicalRQ end to end + jsonl bytes --------------------
def g_simplified():
    X = synth.small_mixture(2048, m=64, seed=21)
    sids = [f"s{i:05d}" for i in range(len(X))]
    with tempfile.TemporaryDirectory() as td:
        p = os.path.join(td, "vec.csv")
        write_csv(p, sids, X)
        seed_all(42)
        model = ref_s.SimplifiedHierarchicalRQ(ref_h.HierarchicalRQKMeansConfig(**SMALL_CFG))
        model.train(p)
        out = os.path.join(td, "ids.jsonl")
        model.save_semantic_ids(out)
        raw = Path(out).read_bytes()
    ids = np.array([model.semantic_ids[s] for s in sids], dtype=np.int64)
    save("simplified", x_sha=np.array(synth.sha256(X)),
         l0_centers=model.trained_kmeans_models[0].cluster_centers.numpy(),
         mid_centers=model.middle_layer_centers.numpy(),
         final_centers=model.final_layer_centers.numpy(),
         match=model.dynamic_match_matrix.numpy(), ids=ids,
         jsonl_head=np.frombuffer(b"".join(raw.splitlines(True)[:5]), dtype=np.uint8),
         jsonl_sha=np.array(synth.sha256(np.frombuffer(raw, dtype=np.uint8))))


# --- G3: HierarchicalRQKMeans train + predict (bug-compatible and fixed) ------
def g_hierarchical():
    X = synth.small_mixture(2048, m=64, seed=21)
    Xn = synth.small_mixture(512, m=64, seed=22)
    seed_all(42)
    m = ref_h.HierarchicalRQKMeans(ref_h.HierarchicalRQKMeansConfig(**SMALL_CFG),
                                   device=torch.device("cpu"))
    tr = m.train(X, resume=False)
    pred_bug = m.predict(X)
    pred_new_bug = m.predict(Xn)
    mm = m.match_matrices[0]
    m.match_matrices = [mm, mm]  # makes predict's lookup at :1248 find the matrix
    pred_fix = m.predict(X)
    # new rows can land in an (l1,l2) group that was empty in training: its match row is
    # all zero, the +10000 mask admits every candidate and the remap at :1084 raises KeyError
    try:
        pred_new_fix = m.predict(Xn)
        new_fix_err = -1
    except KeyError as e:
        pred_new_fix = np.zeros((len(Xn), 3), dtype=np.int64)
        new_fix_err = int(e.args[0])
    save("hierarchical", x_sha=np.array(synth.sha256(X)), xn_sha=np.array(synth.sha256(Xn)),
         c0=m.cluster_centers_list[0].numpy(), c1=m.cluster_centers_list[1].numpy(),
         c2=m.cluster_centers_list[2].numpy(), match=np.array(mm, dtype=np.uint8),
         train_ids=np.stack([t.cpu().numpy() for t in tr["cluster_ids"]], 1).astype(np.int64),
         pred_bug=pred_bug.astype(np.int64), pred_fix=pred_fix.astype(np.int64),
         pred_new_bug=pred_new_bug.astype(np.int64), pred_new_fix=pred_new_fix.astype(np.int64),
         new_fix_keyerror=np.array(new_fix_err))


# --- G-trainer: the reference's driver SemanticIDTrainer (train_semantic_ids.py:35-365) end to end ---
def g_trainer():
    """train_semantic_ids.SemanticIDTrainer(config, use_test_config=True).train(resume=False) on a small
    CSV: the side files training_config.json / training_statistics.json and the jsonl, as bytes."""
    from src.semantic_id_generator import train_semantic_ids as ref_t
    X = synth.small_mixture(2048, m=64, seed=21)
    sids = [f"s{i:05d}" for i in range(len(X))]
    with tempfile.TemporaryDirectory() as td:
        csv_path = os.path.join(td, "vec.csv")
        write_csv(csv_path, sids, X)
        cfg = types.SimpleNamespace(
            output_dir=os.path.join(td, "outputs"), model_dir=os.path.join(td, "models"),
            h_rqkmeans_test=ref_h.HierarchicalRQKMeansConfig(**SMALL_CFG), h_rqkmeans=None,
            data=types.SimpleNamespace(song_vectors_file=csv_path,
                                       semantic_ids_file=os.path.join(td, "outputs", "semantic_id",
                                                                      "song_semantic_ids.jsonl")))
        seed_all(42)
        trainer = ref_t.SemanticIDTrainer(cfg, use_test_config=True)
        res = trainer.train(resume=False)
        out = Path(td) / "outputs" / "semantic_id"
        cfg_bytes = (out / "training_config.json").read_bytes()
        stats_bytes = (out / "training_statistics.json").read_bytes()
        jsonl = (out / "song_semantic_ids.jsonl").read_bytes()
    ids = np.array([res["semantic_ids"][s] for s in sids], dtype=np.int64)
    save("trainer", x_sha=np.array(synth.sha256(X)), ids=ids,
         config_json=np.frombuffer(cfg_bytes, dtype=np.uint8), stats_json=np.frombuffer(stats_bytes, dtype=np.uint8),
         jsonl_sha=np.array(synth.sha256(np.frombuffer(jsonl, dtype=np.uint8))))


# --- G-encode: predict at PROD codebook shapes [128,1280,1280]/[128,128,256] --
def g_encode_prod():
    cb = synth.encode_codebooks(seed=99)
    X = synth.mixture_rows(0, 2000)
    cfg = ref_h.HierarchicalRQKMeansConfig(layer_clusters=[128, 1280, 1280],
                                           need_clusters=[128, 128, 256], embedding_dim=512)
    m = ref_h.HierarchicalRQKMeans(cfg, device=torch.device("cpu"))
    m.cluster_centers_list = [torch.from_numpy(cb["c0"]), torch.from_numpy(cb["c1"]),
                              torch.from_numpy(cb["c2"])]
    mm_list = cb["match"].astype(np.int64).tolist()
    m.match_matrices = [mm_list]
    m.is_trained = True
    pred_bug = m.predict(X)
    m.match_matrices = [mm_list, mm_list]
    pred_fix = m.predict(X)
    # training-time semantics (raw block ids for residuals, match-constrained last level), run
    # through the reference's own reassignment methods (:839-966, :1055-1086)
    Xt = torch.from_numpy(X)
    c0, c1, c2 = m.cluster_centers_list
    ids0 = m._predict_layer_0(Xt, 0)
    r1 = m._compute_residuals_with_centers(Xt, ids0, c0)
    m.result_cluster_ids = [ids0]
    raw1, r2 = m._reassign_clusters_middle_layer_with_residuals(r1, c1, ids0, 1)
    ids1 = raw1 % 128
    before = ids0.numpy() * 128 + ids1.numpy()
    raw2, _ = m._reassign_clusters_last_layer_with_residuals(r2, c2, before, mm_list, 2)
    ids2 = m._merge_match_matrix_cluster_ids(mm_list, raw2, before)
    pred_train = np.stack([ids0.numpy(), ids1.numpy(), ids2.numpy()], 1)
    save("encode_prod", x_sha=np.array(synth.sha256(X)), cb_sha=np.array(synth.codebooks_sha(cb)),
         pred_bug=pred_bug.astype(np.int64), pred_fix=pred_fix.astype(np.int64),
         pred_train=pred_train.astype(np.int64))


# --- G-match: the last layer's match-matrix builders, called directly ----------
def _rng_after():
    """the next draws of both global generators (pins the RNG state the builder leaves behind)"""
    return np.random.randint(1 << 30, size=4).astype(np.int64), torch.randint(1 << 30, (4,)).numpy().astype(np.int64)


def g_match():
    """HierarchicalRQKMeans._assign_last_match_matrix (:968-1053) and
    SimplifiedHierarchicalRQ._get_dynamic_match_matrix (simplified…:247-303) on fixed inputs
    (tests/_data.match_inputs: 16 groups of every kind).  Besides each returned matrix the capture
    records every group's sub-centres exactly as the reference computed them (the operand of its greedy
    step), the fitted sub-K-Means centres, and the next draws of the numpy / torch generators."""
    from tests import _data
    x, l1, l2, cand = _data.match_inputs()
    need = _data.MATCH_NEED
    cfg = ref_h.HierarchicalRQKMeansConfig(layer_clusters=[4, 16, 32], need_clusters=list(need), embedding_dim=512)
    cand_t = torch.from_numpy(cand)
    fitted = []

    class RecKMeans(ref_bk.KMeans):
        def fit(self, *a, **kw):
            out = super().fit(*a, **kw)
            fitted.append(self.cluster_centers.detach().cpu().numpy().copy())
            return out

    # hierarchical: the greedy operand is the first argument of torch.cdist(sub_centers, candidates) (:1027)
    subs_h = []
    orig_cdist = torch.cdist

    def cdist_rec(a, b, *args, **kw):
        if b.data_ptr() == cand_t.data_ptr():
            subs_h.append(a.detach().numpy().copy())
        return orig_cdist(a, b, *args, **kw)

    m = ref_h.HierarchicalRQKMeans(cfg, device=torch.device("cpu"))
    seed_all(71)
    ref_h.KMeans, torch.cdist = RecKMeans, cdist_rec
    try:
        match_h = m._assign_last_match_matrix(cand_t, 2 * 32, torch.from_numpy(x), need[0], need[1], l1, l2,
                                              need[2], 2 * need[2], 2)
    finally:
        ref_h.KMeans, torch.cdist = ref_bk.KMeans, orig_cdist
    h_np, h_torch = _rng_after()
    fitted_h, fitted[:] = list(fitted), []
    # simplified: the greedy operand is rebuilt from the recorded draws (empty group -> its candidate
    # sample, :268; <= need rows -> the rows, :270; else the fitted centres, :276)
    choices = []
    orig_choice = np.random.choice

    def choice_rec(*a, **kw):
        r = orig_choice(*a, **kw)
        choices.append(np.asarray(r).copy())
        return r

    s = ref_s.SimplifiedHierarchicalRQ.__new__(ref_s.SimplifiedHierarchicalRQ)
    s.config, s.device = cfg, torch.device("cpu")
    seed_all(72)
    ref_s.KMeans, np.random.choice = RecKMeans, choice_rec
    try:
        match_s = s._get_dynamic_match_matrix(torch.from_numpy(x), torch.from_numpy(l1), torch.from_numpy(l2), cand_t)
    finally:
        ref_s.KMeans, np.random.choice = ref_bk.KMeans, orig_choice
    s_np, s_torch = _rng_after()
    gid = l1 * need[1] + l2
    subs_s, ci, fi = [], 0, 0
    for g in range(need[0] * need[1]):
        rows = np.nonzero(gid == g)[0]
        if len(rows) == 0:
            subs_s.append(cand[choices[ci]])
            ci += 1
        elif len(rows) <= need[2]:
            subs_s.append(x[rows])
        else:
            subs_s.append(fitted[fi])
            ci += 1  # the fit's KMeans.initialize draw
            fi += 1
    assert ci == len(choices) and fi == len(fitted)

    def cat(parts):
        return (np.concatenate(parts, 0).astype(np.float32),
                np.concatenate([[0], np.cumsum([len(p) for p in parts])]).astype(np.int64))
    sh, sh_off = cat(subs_h)
    ss, ss_off = cat(subs_s)
    fh, fh_off = cat(fitted_h) if fitted_h else (np.zeros((0, 512), np.float32), np.zeros(1, np.int64))
    save("match", x_sha=np.array(synth.sha256(x)), cand_sha=np.array(synth.sha256(cand)),
         hier_match=np.array(match_h, dtype=np.uint8), hier_sub=sh, hier_sub_off=sh_off,
         hier_fitted=fh, hier_fitted_off=fh_off, hier_np_after=h_np, hier_torch_after=h_torch,
         simp_match=match_s.numpy().astype(np.uint8), simp_sub=ss, simp_sub_off=ss_off,
         simp_np_after=s_np, simp_torch_after=s_torch)


# --- G-config0: BASELINE configs[0], the single-level simplified run (L = 1) -----
def g_config0():
    """SimplifiedHierarchicalRQ.train with layer_clusters = need_clusters = [K] (simplified…:176-245):
    one balanced fit_by_min_loss with target_nodes_num = np.prod([]) = 1.0 (:197), then predict.  Two
    golden-size cases (tests/_data.CONFIG0_CASES): K = 8 with N % K != 0 (1002-round auctions) and the
    configs[0] K = 128."""
    from tests import _data
    out = {}
    for tag in _data.CONFIG0_CASES:
        x, k, it = _data.config0_inputs(tag)
        sids = [f"s{i:05d}" for i in range(len(x))]
        with tempfile.TemporaryDirectory() as td:
            p = os.path.join(td, "vec.csv")
            write_csv(p, sids, x)
            seed_all(42)
            model = ref_s.SimplifiedHierarchicalRQ(ref_h.HierarchicalRQKMeansConfig(
                layer_clusters=[k], need_clusters=[k], embedding_dim=512, iter_limit=it))
            model.train(p)
            o = os.path.join(td, "ids.jsonl")
            model.save_semantic_ids(o)
            raw = Path(o).read_bytes()
        out[f"{tag}_x_sha"] = np.array(synth.sha256(x))
        out[f"{tag}_ids"] = np.array([model.semantic_ids[s] for s in sids], dtype=np.int64)
        out[f"{tag}_centers"] = model.trained_kmeans_models[0].cluster_centers.numpy()
        out[f"{tag}_jsonl_sha"] = np.array(synth.sha256(np.frombuffer(raw, dtype=np.uint8)))
    save("config0", **out)


# --- G-exact: trainer runs on which the reference's own fits take no tie-born step -------
def _exact_labels(run, n, shape_fn, tries=4):
    """labels at the fixed point of (record the reference's initialisation draws -> place the labels)"""
    import exact_fixture as E
    lab = shape_fn(None)
    for _ in range(tries):
        with E.DrawRecorder() as dr:
            run(lab)
        new = shape_fn(dr.draws)
        if np.array_equal(new, lab):
            return lab
        lab = new
    raise RuntimeError("draws did not reach a fixed point")


def g_exact():
    """tests/_data.EXACT_CASES: the SMALL_CFG hierarchical and simplified trainers and the single-level
    configs[0] runs on tree-mixture rows whose every fit is clean (tests/golden/precertify.py: no auction
    whose two tie rules give different results, no fp16 rounding flip that changes one).  Stores the
    labels (the tests regenerate the rows with synth.tree_mixture) and the reference's outputs."""
    import exact_fixture as E
    import precertify as PC
    from tests import _data
    out = {}
    for tag, spec in _data.EXACT_CASES.items():
        n, kind = spec["n"], spec["kind"]
        if kind == "single":
            k = spec["k"]
            cfg = dict(layer_clusters=[k], need_clusters=[k], embedding_dim=512, iter_limit=spec["iter_limit"])
        else:
            cfg = dict(SMALL_CFG)

        def shape_fn(draws):
            if draws is None:  # placeholder: balanced random labels
                return _data.exact_placeholder(tag)
            if kind == "single":
                lab = E.single_labels(draws[0][2], n, spec["k"], seed=spec["label_seed"])
                return np.stack([lab, np.zeros_like(lab), np.zeros_like(lab)], 1)
            return E.hier_labels(draws, n, 8, 8, 16, 8, seed=spec["label_seed"])

        def run(lab):
            x = _data.exact_rows(tag, lab)
            return (PC.run_hierarchical if kind == "hier" else PC.run_simplified)(x, cfg)

        lab = _exact_labels(run, n, shape_fn)
        x = _data.exact_rows(tag, lab)
        m, ids, fits = run(lab)
        bad = [f for f in fits if not f["clean"]]
        assert not bad, PC.summary(fits)
        out[f"{tag}_labels"] = lab.astype(np.int16)
        out[f"{tag}_x_sha"] = np.array(synth.sha256(x))
        out[f"{tag}_ids"] = ids
        out[f"{tag}_fits"] = np.array(len(fits))
        if kind == "hier":
            for l in range(3):
                out[f"{tag}_c{l}"] = m.cluster_centers_list[l].numpy()
            out[f"{tag}_match"] = np.array(m.match_matrices[0], dtype=np.uint8)
        else:
            out[f"{tag}_c0"] = m.trained_kmeans_models[0].cluster_centers.numpy()
            if kind == "simp":
                out[f"{tag}_c1"] = m.middle_layer_centers.numpy()
                out[f"{tag}_c2"] = m.final_layer_centers.numpy()
                out[f"{tag}_match"] = m.dynamic_match_matrix.numpy().astype(np.uint8)
            sids = [f"s{i:05d}" for i in range(n)]
            with tempfile.TemporaryDirectory() as td:
                o = os.path.join(td, "ids.jsonl")
                m.save_semantic_ids(o)
                raw = Path(o).read_bytes()
            out[f"{tag}_jsonl_sha"] = np.array(synth.sha256(np.frombuffer(raw, dtype=np.uint8)))
        print(tag, "clean fits:", len(fits))
    save("exact", **out)


# --- G-cosine: KMeans(distance='cosine') (:279-280, 511-512, pairwise_cosine :625-655) ------------------
def g_cosine():
    """pairwise_cosine on fixed rows; KMeans(balanced=True).fit / fit_by_min_loss and the unbalanced fit with
    distance='cosine' (seeded); predict(distance='cosine')."""
    from tests import _data
    x, c = _data.cosine_inputs()
    d = ref_bk.pairwise_cosine(torch.from_numpy(x), torch.from_numpy(c))
    out = {"x_sha": np.array(synth.sha256(x)), "d": d.numpy()}
    seed_all(31)
    km = ref_bk.KMeans(n_clusters=8, balanced=True)
    a = km.fit(torch.from_numpy(x), distance="cosine", iter_limit=4, tqdm_flag=False)
    out.update(fit_bal_assign=a.numpy().astype(np.int64), fit_bal_centers=km.cluster_centers.numpy())
    out["pred"] = km.predict(torch.from_numpy(x), distance="cosine").numpy().astype(np.int64)
    seed_all(32)
    km2 = ref_bk.KMeans(n_clusters=8, balanced=False)
    a2 = km2.fit(torch.from_numpy(x), distance="cosine", iter_limit=3, tqdm_flag=False)
    out.update(fit_unbal_assign=a2.numpy().astype(np.int64), fit_unbal_centers=km2.cluster_centers.numpy())
    seed_all(33)
    km3 = ref_bk.KMeans(n_clusters=8, balanced=True)
    km3.fit_by_min_loss(torch.from_numpy(x), target_nodes_num=64, distance="cosine", iter_limit=4, tqdm_flag=False)
    out["fbml_centers"] = km3.cluster_centers.numpy()
    save("cosine", **out)


# --- G-csv: loader skip rules (simplified :38-76) ----------------------------
def g_csv():
    rows = [["a", "1", "2", "3", "4"], ["b"], ["c", "1", "x", "3", "4"], ["d", "1", "2", "3"],
            ["e", "0.5", "-1.25", "3e-3", "4"], [], ["a", "9", "9", "9", "9"], ["f", " 1", "2 ", "3", "4"]]
    buf = io.StringIO()
    csv.writer(buf).writerows(rows)
    text = buf.getvalue()
    with tempfile.TemporaryDirectory() as td:
        p = os.path.join(td, "v.csv")
        Path(p).write_text(text)
        s = ref_s.SimplifiedHierarchicalRQ.__new__(ref_s.SimplifiedHierarchicalRQ)
        s.config = ref_h.HierarchicalRQKMeansConfig(layer_clusters=[2], need_clusters=[2], embedding_dim=4)
        sids, emb = s._load_data(p)
        s.config = ref_h.HierarchicalRQKMeansConfig(layer_clusters=[600], need_clusters=[2], embedding_dim=4)
        sids_h, emb_h = s._load_data(p)
    save("csv", text=np.frombuffer(text.encode(), dtype=np.uint8), sids=np.array(sids),
         emb=emb.numpy(), emb_half=emb_h.numpy(), emb_half_dtype=np.array(str(emb_h.dtype)))


if __name__ == "__main__":
    which = sys.argv[1:] or ["assign", "residual", "update", "auction", "fit", "simplified",
                             "hierarchical", "encode_prod", "csv", "dist_half", "trainer", "match", "config0", "exact", "cosine"]
    for w in which:
        globals()[f"g_{w}"]()
