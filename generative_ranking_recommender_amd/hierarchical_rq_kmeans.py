"""Hierarchical residual-quantisation balanced K-Means on MI355X — the drop-in for
src/semantic_id_generator/hierarchical_rq_kmeans.py.

Same classes, constructor arguments, method names, return values and error types as the reference:
``HierarchicalRQKMeansConfig``, ``CheckpointManager``, ``HierarchicalRQKMeans`` (``train``,
``predict``, ``save_model``, ``load_model``, ``get_training_status``).  The per-level strategy
(:438-475), the ID semantics (modulo ids in middle layers, rank-remapped last-layer ids, the
``l1 * need[l-2] + l2`` group id of :824) and the numpy / torch RNG call order are the reference's.
Every distance, argmin, auction, centroid update and residual runs in ``librqsid.so``:

* K-Means fits            -> balancekmeans.KMeans (rqsid_assign / rqsid_auction_* / rqsid_centroid_*)
* masked reassignment     -> rqsid_assign on rows bucketed by parent / (l1,l2) group, the allowed
                             centres as candidate lists (no dense N x K distance matrix, no +10000 mask)
* residual normalisation  -> rqsid_residual
* match-matrix greedy     -> rqsid_greedy_match (batched over groups)

Deliberate, documented differences: model and checkpoint files are ``.npz`` / JSON, never pickle;
``predict(X)`` reproduces the reference's predict-time quirks by default (the missing last-layer match
lookup of :1248 and the modulo-id residual of :1143) — ``predict(X, reference_quirks=False)`` gives
the training-consistent encode.
"""
from __future__ import annotations

import json
import logging
import os
import time
from dataclasses import asdict, dataclass
from pathlib import Path
from typing import Dict, List, Optional, Union

import numpy as np
import torch

from . import ops
from .balancekmeans import KMeans, _device, fit_segments, init_indices

logger = logging.getLogger(__name__)


@dataclass
class HierarchicalRQKMeansConfig:
    """hierarchical_rq_kmeans.py:32-82 (same fields, defaults and validation)."""
    layer_clusters: List[int]
    need_clusters: List[int]
    embedding_dim: int
    group_dims: Union[int, List[int]] = None
    hierarchical_weights: Union[float, List[List[float]]] = None
    iter_limit: int = 100

    def __post_init__(self):
        if self.group_dims is None or (isinstance(self.group_dims, list) and len(self.group_dims) == 0):
            self.group_dims = [self.embedding_dim]
        elif isinstance(self.group_dims, int):
            self.group_dims = [self.group_dims]
        if sum(self.group_dims) != self.embedding_dim:
            raise ValueError(
                f"Sum of group_dims {sum(self.group_dims)} must equal embedding_dim {self.embedding_dim}")
        if self.hierarchical_weights is None or (
                isinstance(self.hierarchical_weights, list) and len(self.hierarchical_weights) == 0):
            self.hierarchical_weights = [[1.0 / len(self.group_dims)] * len(self.group_dims)
                                         for _ in range(len(self.layer_clusters))]
        elif isinstance(self.hierarchical_weights, (int, float)):
            self.hierarchical_weights = [[1.0 / len(self.group_dims)] * len(self.group_dims)
                                         for _ in range(len(self.layer_clusters))]
        if len(self.hierarchical_weights) != len(self.layer_clusters):
            raise ValueError(
                f"Length of hierarchical_weights {len(self.hierarchical_weights)} "
                f"must equal length of layer_clusters {len(self.layer_clusters)}")
        for i, weights in enumerate(self.hierarchical_weights):
            if len(weights) != len(self.group_dims):
                raise ValueError(
                    f"Length of hierarchical_weights[{i}] {len(weights)} "
                    f"must equal length of group_dims {len(self.group_dims)}")


def _np(t):
    if isinstance(t, torch.Tensor):
        return t.detach().cpu().numpy()
    return None if t is None else np.asarray(t)


class CheckpointManager:
    """hierarchical_rq_kmeans.py:85-184 — per-layer checkpoints written to a temporary file,
    re-read and validated, then atomically renamed.  Format: ``layer_{i}_checkpoint.npz``."""

    def __init__(self, checkpoint_dir: str):
        self.checkpoint_dir = Path(checkpoint_dir)
        self.checkpoint_dir.mkdir(parents=True, exist_ok=True)
        self.metadata_file = self.checkpoint_dir / "checkpoint_metadata.json"

    def _file(self, layer: int) -> Path:
        return self.checkpoint_dir / f"layer_{layer}_checkpoint.npz"

    def save_layer_checkpoint(self, layer: int, cluster_ids, residual_data, cluster_centers=None,
                              match_matrix=None):
        arrays = {"layer": np.int64(layer), "cluster_ids": _np(cluster_ids), "residual_data": _np(residual_data),
                  "cluster_centers": _np(cluster_centers)}
        if match_matrix is not None:
            arrays["match_matrix"] = np.asarray(_np(match_matrix), dtype=np.uint8)
        arrays = {k: v for k, v in arrays.items() if v is not None}
        final = self._file(layer)
        tmp = self.checkpoint_dir / f"layer_{layer}_checkpoint.tmp.npz"
        try:
            np.savez(tmp, **arrays)
            with np.load(tmp, allow_pickle=False) as z:
                for key in ("cluster_ids", "cluster_centers"):
                    if key not in z.files:
                        raise ValueError(f"Checkpoint validation failed: missing or None key '{key}'")
            os.replace(tmp, final)
        except Exception as e:
            if tmp.exists():
                try:
                    tmp.unlink()
                except OSError:
                    pass
            logger.error("Failed to save checkpoint for layer %d: %s", layer, e)
            raise

    def load_layer_checkpoint(self, layer: int, device: torch.device) -> Optional[Dict]:
        f = self._file(layer)
        if not f.exists():
            return None
        with np.load(f, allow_pickle=False) as z:
            ck = {k: z[k] for k in z.files}
        for key in ("cluster_ids", "residual_data", "cluster_centers"):
            if key in ck:
                ck[key] = torch.from_numpy(ck[key]).to(device)
        if "match_matrix" in ck:
            ck["match_matrix"] = ck["match_matrix"]
        return ck

    def get_last_completed_layer(self) -> int:
        done = -1
        for i in range(100):
            if self._file(i).exists():
                done = i
            else:
                break
        return done

    def save_metadata(self, metadata: Dict):
        with open(self.metadata_file, "w") as f:
            json.dump(metadata, f, indent=2, default=str)

    def load_metadata(self) -> Optional[Dict]:
        if not self.metadata_file.exists():
            return None
        with open(self.metadata_file) as f:
            return json.load(f)

    def clear_checkpoints(self):
        for f in self.checkpoint_dir.glob("layer_*_checkpoint.npz"):
            f.unlink()
        if self.metadata_file.exists():
            self.metadata_file.unlink()


def adaptive_iter_limit(num_samples: int, n_clusters: int, layer: int, base_iter_limit: int = 100,
                        is_sub_cluster: bool = False) -> int:
    """_calculate_adaptive_iter_limit, hierarchical_rq_kmeans.py:288-366."""
    spc = num_samples / max(n_clusters, 1)
    if is_sub_cluster:
        it = 15 if num_samples < 5000 else 20 if num_samples < 10000 else 25 if num_samples < 20000 else 30
        if spc < 50:
            it = max(10, int(it * 0.8))
        elif spc > 200:
            it = int(it * 1.2)
        return max(10, it)
    if num_samples < 5000:
        it = max(10, int(base_iter_limit * 0.2))
    elif num_samples < 10000:
        it = max(15, int(base_iter_limit * 0.3))
    elif num_samples < 50000:
        it = max(30, int(base_iter_limit * 0.5))
    elif num_samples < 100000:
        it = max(50, int(base_iter_limit * 0.7))
    elif num_samples < 500000:
        it = base_iter_limit
    elif num_samples < 1000000:
        it = int(base_iter_limit * 1.2)
    else:
        it = int(base_iter_limit * 1.5)
    if n_clusters > 512:
        it = int(it * 1.3)
    elif n_clusters > 256:
        it = int(it * 1.15)
    if layer > 1:
        it = max(10, int(it * 0.9))
    if spc < 50:
        it = int(it * 1.2)
    return max(10, it)


def group_rows(keys: torch.Tensor, n_groups: int):
    """Rows of every group in ascending row order (``torch.where(ids == g)`` for all g at once):
    returns (order i64[N], offsets i64[G+1])."""
    order = torch.sort(keys.long(), stable=True)[1]
    counts = torch.bincount(keys.long(), minlength=n_groups)
    off = torch.zeros(n_groups + 1, dtype=torch.int64, device=keys.device)
    off[1:] = torch.cumsum(counts, 0)
    return order, off.cpu().numpy()


def random_fill(row: np.ndarray, need: int) -> None:
    """The reference's fill-up loop (hierarchical :1041-1048 / simplified :294-297):
    ``while have < need: r = np.random.randint(n_cand); if not row[r]: row[r] = 1; have += 1``.

    Drawn in blocks: the legacy MT19937 ``randint(n, size=m)`` yields exactly the values (and the
    generator state) of m single calls, so a block is drawn, scanned in draw order for the first
    occurrences of unset columns, and when the block holds the last needed column the generator is
    rewound and advanced by exactly the draws the loop would have consumed."""
    n_cand = row.shape[0]
    have = int(row.sum())
    while have < need:
        state = np.random.get_state()
        m = max(64, 2 * (need - have))
        draws = np.random.randint(n_cand, size=m)
        vals, first = np.unique(draws, return_index=True)
        fresh = row[vals] == 0
        pos = np.sort(first[fresh])
        missing = need - have
        if len(pos) >= missing:
            k = int(pos[missing - 1])
            np.random.set_state(state)
            np.random.randint(n_cand, size=k + 1)
            row[draws[pos[:missing]]] = 1
            return
        row[draws[pos]] = 1
        have += len(pos)


def masked_assign(x: torch.Tensor, centers: torch.Tensor, seg: torch.Tensor, cand: ops.Candidates, n_segments: int):
    """The +10000 / +inf masked argmin over each row's allowed centres.  Returns (local i32, global i32)."""
    return ops.assign(x, ops.prepare_centers(centers), ops.bucket(seg, n_segments), cand)


class HierarchicalRQKMeans:
    """hierarchical_rq_kmeans.py:187-1409."""

    def __init__(self, config: HierarchicalRQKMeansConfig, checkpoint_dir: Optional[str] = None,
                 device: Optional[torch.device] = None, group=None):
        self.config = config
        self.group = group  # torch.distributed group: row-sharded training / encode
        self.device = _device(device)
        self.checkpoint_manager = CheckpointManager(checkpoint_dir) if checkpoint_dir else None
        self.is_trained = False
        self.cluster_centers_list: List[torch.Tensor] = []
        self.match_matrices: List[np.ndarray] = []
        self.result_cluster_ids: List[torch.Tensor] = []
        # Sub-K-Means of the middle layer and of the last-layer match matrix: True runs them in lockstep
        # (balancekmeans.fit_segments: one segmented auction per iteration for all parents / groups);
        # False runs them one after another as the reference does.  Both consume the numpy and torch
        # random numbers exactly as the reference's loop does.
        self.batched_sub_fits = True

    @staticmethod
    def _get_device() -> torch.device:
        return _device(None)

    @staticmethod
    def _calculate_safe_batch_size(X, num_centers, device, initial_batch_size: int = 200000) -> int:
        """Kept for API compatibility: the kernels stream rows and need no N x K buffer."""
        return max(1, min(initial_batch_size, len(X)))

    @staticmethod
    def _calculate_adaptive_iter_limit(num_samples, n_clusters, layer, base_iter_limit=100, is_sub_cluster=False):
        return adaptive_iter_limit(num_samples, n_clusters, layer, base_iter_limit, is_sub_cluster)

    # ------------------------------------------------------------------------------------ training
    def train(self, X: np.ndarray, resume: bool = True) -> Dict:
        """:368-537.  With a process group (``group=``) the rows are sharded across the ranks: see
        ``_train_sharded``."""
        self.invalidate_encoder()
        if self.group is not None:
            return self._train_sharded(X, resume)
        cfg = self.config
        if X.shape[1] != cfg.embedding_dim:
            raise ValueError(f"Input dimension {X.shape[1]} does not match config embedding_dim {cfg.embedding_dim}")
        t_total = time.time()
        L = len(cfg.layer_clusters)
        start_layer = 0
        if resume and self.checkpoint_manager:
            start_layer = self.checkpoint_manager.get_last_completed_layer() + 1
            if start_layer > 0:
                logger.info("[RESUME] Resuming training from layer %d", start_layer)
                self._load_previous_checkpoints(start_layer)
        current = torch.from_numpy(np.ascontiguousarray(X, dtype=np.float32)).to(self.device)
        if start_layer > 0 and self.checkpoint_manager:
            ck = self.checkpoint_manager.load_layer_checkpoint(start_layer - 1, self.device)
            if ck and "residual_data" in ck:
                current = ck["residual_data"].float().contiguous()
            else:  # a sharded run's checkpoints hold no residuals: rebuild the chain from ids + centres
                current = self._residual_chain(current, [t.to(self.device).long() for t in self.result_cluster_ids],
                                               start_layer)
        for layer in range(start_layer, L):
            t0 = time.time()
            n_clusters, need = cfg.layer_clusters[layer], cfg.need_clusters[layer]
            weighted = self._apply_weights(current, layer)
            match = None
            residual = None
            if n_clusters == need:
                centers, ids, residual = self._train_layer_0(weighted, layer)
            elif layer == L - 1:
                centers, ids, residual = self._train_last_layer(weighted, layer)
                if self.match_matrices:
                    match = self.match_matrices[-1]
            else:
                centers, ids, residual = self._train_middle_layer(weighted, layer)
            self.cluster_centers_list.append(centers)
            self.result_cluster_ids.append(ids)
            if self.checkpoint_manager:
                ck_res = residual if layer < L - 1 else current
                self.checkpoint_manager.save_layer_checkpoint(layer, ids, ck_res, centers, match)
            if layer < L - 1:
                current = residual
            logger.info("[LAYER %d] completed in %.2fs", layer + 1, time.time() - t0)
        self.is_trained = True
        if self.checkpoint_manager:
            self.checkpoint_manager.save_metadata({
                "num_layers": L, "embedding_dim": cfg.embedding_dim, "group_dims": cfg.group_dims,
                "hierarchical_weights": cfg.hierarchical_weights, "num_samples": len(X)})
        logger.info("[TRAINING COMPLETE] Total time: %.2fs", time.time() - t_total)
        return {"cluster_ids": self.result_cluster_ids, "cluster_centers": self.cluster_centers_list}

    def _apply_weights(self, data: torch.Tensor, layer: int) -> torch.Tensor:
        """:583-604 (identity weights skip the multiply: x * 1.0 is x exactly)."""
        w = self.config.hierarchical_weights[layer]
        if all(float(v) == 1.0 for v in w):
            return data
        return ops.scale_groups(data.contiguous(), self.config.group_dims, [float(v) for v in w])

    def _compute_residuals_with_centers(self, X, cluster_ids, cluster_centers) -> torch.Tensor:
        """:1088-1128: r = x - c[id], every dimension group divided by (||r_g|| + 1e-8)."""
        return ops.residual(X.contiguous(), cluster_centers.float().contiguous().to(X.device),
                            cluster_ids.to(X.device).to(torch.int32), self.config.group_dims, True)

    def _compute_residuals(self, X, cluster_ids, layer) -> torch.Tensor:
        return self._compute_residuals_with_centers(X, cluster_ids, self.cluster_centers_list[layer])

    def _train_layer_0(self, X: torch.Tensor, layer: int):
        """:606-669."""
        cfg = self.config
        n_clusters = cfg.layer_clusters[layer]
        target = 1
        for idx, v in enumerate(cfg.need_clusters):
            if idx != layer:
                target *= v
        iters = adaptive_iter_limit(len(X), n_clusters, layer, cfg.iter_limit)
        km = KMeans(n_clusters=n_clusters, device=self.device, balanced=True)
        km.fit_by_min_loss(X=X, target_nodes_num=target, distance="euclidean", iter_limit=iters, tqdm_flag=True,
                           half=n_clusters >= 512, online=False)
        centers = km.cluster_centers.detach()
        ids = ops.nearest(X.contiguous(), ops.prepare_centers(centers)).long()
        residual = self._compute_residuals_with_centers(X, ids, centers)
        return centers, ids, residual

    def _train_middle_layer(self, X: torch.Tensor, layer: int):
        """:671-752: one balanced sub-K-Means per parent cluster, masked reassignment, residual on the raw id."""
        cfg = self.config
        cur_need, pre_need = cfg.need_clusters[layer], cfg.need_clusters[layer - 1]
        if layer - 1 >= len(self.result_cluster_ids):
            raise RuntimeError(
                f"Previous layer {layer - 1} cluster IDs not found. "
                f"Expected at least {layer} layers but only have {len(self.result_cluster_ids)} layers.")
        prev = self.result_cluster_ids[layer - 1].to(self.device)
        target = 1
        for idx, v in enumerate(cfg.need_clusters):
            if idx > layer:
                target *= v
        order, off = group_rows(prev, pre_need)
        if self.batched_sub_fits:
            t0 = time.time()
            centers = self._batched_middle_fits(X, order, off, cur_need, layer, target)
            logger.info("[LAYER %d] %d lockstep sub-fits %.2fs", layer + 1, pre_need, time.time() - t0)
            raw, residual = self._reassign_clusters_middle_layer_with_residuals(X, centers, prev, layer)
            return centers, raw % cur_need, residual
        sub_centers = []
        for i in range(pre_need):
            idx = order[off[i]:off[i + 1]]
            sub = X[idx]
            iters = adaptive_iter_limit(len(idx), cur_need, layer, cfg.iter_limit, is_sub_cluster=True)
            km = KMeans(n_clusters=cur_need, device=self.device, balanced=True)
            km.fit_by_min_loss(X=sub, target_nodes_num=target, distance="euclidean", iter_limit=iters,
                               tqdm_flag=True, half=cur_need >= 512, online=False)
            sub_centers.append(km.cluster_centers.detach())
        centers = torch.cat(sub_centers, 0).contiguous()
        raw, residual = self._reassign_clusters_middle_layer_with_residuals(X, centers, prev, layer)
        return centers, raw % cur_need, residual

    def _batched_middle_fits(self, X, order, off, cur_need, layer, target):
        """The per-parent balanced fit_by_min_loss runs of :703-725 in lockstep, drawing numpy and torch
        random numbers exactly as the one-after-another loop does (balancekmeans.fit_segments)."""
        cfg = self.config
        sizes = np.diff(off).astype(np.int64)
        limits = [adaptive_iter_limit(int(n_i), cur_need, layer, cfg.iter_limit, is_sub_cluster=True) for n_i in sizes]
        centers, _ = fit_segments(X[order].contiguous(), sizes, cur_need, limits, target_nodes_num=target,
                                  half=cur_need >= 512)
        return centers.contiguous()

    def _reassign_clusters_middle_layer_with_residuals(self, X, kmeans_centers, prev_cluster_ids, layer):
        """:839-904: each row may take only its parent's block of need[l] centres."""
        pre_need, cur_need = self.config.need_clusters[layer - 1], self.config.need_clusters[layer]
        cand = ops.contiguous_candidates(pre_need, cur_need, self.device)
        _, glob = masked_assign(X.contiguous(), kmeans_centers, prev_cluster_ids.to(self.device), cand, pre_need)
        raw = glob.long()
        return raw, self._compute_residuals_with_centers(X, raw, kmeans_centers)

    def _train_last_layer(self, X: torch.Tensor, layer: int):
        """:754-837: two balanced K-Means give 2 * layer_clusters candidates; the match matrix allows
        need[l] of them per (l1, l2) group; ids are the rank of the chosen column in its row."""
        cfg = self.config
        n_clusters, need = cfg.layer_clusters[layer], cfg.need_clusters[layer]
        if len(self.result_cluster_ids) < 2:
            raise RuntimeError(
                f"Previous layers cluster IDs not found. "
                f"Expected at least 2 layers but only have {len(self.result_cluster_ids)} layers.")
        t0 = time.time()
        parts = []
        for _ in range(2):
            km = KMeans(n_clusters=n_clusters, device=self.device, balanced=True)
            km.fit(X=X, distance="euclidean", iter_limit=20, tqdm_flag=True, half=n_clusters >= 512, online=False)
            parts.append(km.cluster_centers.detach())
        cand_centers = torch.cat(parts, 0).contiguous()
        logger.info("[LAYER %d] candidate fits (2 x %d centres) %.2fs", layer + 1, n_clusters, time.time() - t0)
        t0 = time.time()
        l1 = self.result_cluster_ids[-2].to(self.device).long()
        l2 = self.result_cluster_ids[-1].to(self.device).long()
        pp_need = cfg.need_clusters[layer - 2]
        match = self._assign_last_match_matrix(cand_centers, 2 * n_clusters, X, pp_need, cfg.need_clusters[layer - 1],
                                               l1, l2, need, 2 * need, layer)
        self.match_matrices.append(match)
        logger.info("[LAYER %d] match matrix %.2fs", layer + 1, time.time() - t0)
        before = l1 * pp_need + l2
        raw, residual = self._reassign_clusters_last_layer_with_residuals(X, cand_centers, before, match, layer)
        ids = self._merge_match_matrix_cluster_ids(match, raw, before)
        return cand_centers, ids, residual

    def _reassign_clusters_last_layer_with_residuals(self, X, kmeans_centers, before_cluster_ids, match_matrix, layer):
        """:906-966: rows of group g may take only the columns of match row g (an all-zero row: the
        +10000 penalty makes every centre equal, argmin over all)."""
        m = torch.as_tensor(np.asarray(match_matrix, dtype=np.uint8)).to(self.device)
        before = torch.as_tensor(before_cluster_ids).to(self.device).long()
        if before.numel() and int(before.max().item()) >= m.shape[0]:
            raise IndexError(f"index {int(before.max().item())} is out of bounds for axis 0 with size {m.shape[0]}")
        cand = ops.match_to_candidates(m)
        local, glob = masked_assign(X.contiguous(), kmeans_centers, before, cand, m.shape[0])
        raw = glob.long()
        self._last_local = local
        return raw, self._compute_residuals_with_centers(X, raw, kmeans_centers)

    def _merge_match_matrix_cluster_ids(self, match_matrix, cluster_ids, before_cluster_ids) -> torch.Tensor:
        """:1055-1086: rank of the raw column among the row's allowed columns (KeyError when the column
        is not allowed, as the reference's dict lookup)."""
        m = np.asarray(match_matrix) == 1
        raw = _np(cluster_ids).astype(np.int64)
        before = _np(before_cluster_ids).astype(np.int64)
        ok = m[before, raw]
        if not ok.all():
            raise KeyError(int(raw[np.nonzero(~ok)[0][0]]))
        rank = np.cumsum(m, axis=1) - 1
        return torch.from_numpy(rank[before, raw].astype(np.int64)).to(self.device)

    def _assign_last_match_matrix(self, cur_kmeans_centers, cur_n_cluster, X, prev_prev_need_cluster,
                                  prev_need_cluster, prev_prev_cluster_ids, prev_cluster_ids, cur_need_cluster,
                                  cur_trunct_cluster, layer) -> np.ndarray:
        """:968-1053.  Per (l1, l2) group, in the reference's order: no rows -> all-zero row; <= need rows ->
        the rows themselves; < 2*need rows -> need random rows (np.random.choice); else a balanced
        sub-K-Means.  Each group's centres greedily take their nearest unused candidate column
        (rqsid_greedy_match, batched over groups); groups left short draw random columns."""
        need = cur_need_cluster
        G = prev_prev_need_cluster * prev_need_cluster
        gid = torch.as_tensor(prev_prev_cluster_ids).to(self.device).long() * prev_need_cluster + \
            torch.as_tensor(prev_cluster_ids).to(self.device).long()
        order, off = group_rows(gid, G)
        cand = cur_kmeans_centers.float().contiguous()
        match = np.zeros((G, cur_n_cluster), dtype=np.uint8)
        deferred_groups, deferred_centers = [], []

        def greedy(groups, centers_list):
            sizes = [len(c) for c in centers_list]
            sub_off = torch.tensor(np.concatenate([[0], np.cumsum(sizes)]), dtype=torch.int32, device=self.device)
            sc = torch.cat(centers_list, 0).float()
            dist = ops.pairwise_distance(sc.contiguous(), cand) if len(sc) else sc.new_zeros((0, len(cand)))
            rows, _ = ops.greedy_match(dist, sub_off, need)
            return rows.cpu().numpy()

        if self.batched_sub_fits:
            return self._batched_match_matrix(cand, X, order, off, G, need, cur_trunct_cluster, layer, greedy, match)
        for g in range(G):
            n_g = int(off[g + 1] - off[g])
            if n_g == 0:
                continue
            sub = X[order[off[g]:off[g + 1]]]
            if n_g <= need:
                centers = sub
            elif n_g < cur_trunct_cluster:
                centers = sub[torch.from_numpy(np.random.choice(n_g, need, replace=False)).to(self.device)]
            else:
                km = KMeans(n_clusters=need, device=self.device, balanced=True)
                iters = adaptive_iter_limit(n_g, need, layer, base_iter_limit=20)
                km.fit(X=sub, distance="euclidean", iter_limit=iters, tqdm_flag=True, half=False, online=False)
                centers = km.cluster_centers.detach()
            if min(len(centers), need) < need:
                # the random fill draws from the RNG right after this group's greedy step
                match[g] = greedy([g], [centers])[0]
                random_fill(match[g], need)
            else:
                deferred_groups.append(g)
                deferred_centers.append(centers)
        if deferred_groups:
            match[np.asarray(deferred_groups)] = greedy(deferred_groups, deferred_centers)
        return match

    def _batched_match_matrix(self, cand, X, order, off, G, need, trunc, layer, greedy, match):
        """:968-1053 with the groups' sub-K-Means in lockstep (balancekmeans.batched_fit).  Every random
        draw of the reference happens in its group order: a short group's random fill right after its
        greedy step (its centres are its own rows, so the greedy step can run first), a mid-size group's
        row sample, a large group's initialisation (``fit`` draws nothing else from numpy).  Rows are
        gathered once for all groups (16384 groups at PROD shape)."""
        sizes = np.diff(off).astype(np.int64)

        def rows_of(groups, picks=None):
            """positions in ``order`` of each group's rows (or of its picked rows), concatenated"""
            parts = [off[g] + (np.arange(sizes[g]) if picks is None else picks[i]) for i, g in enumerate(groups)]
            return torch.from_numpy(np.concatenate(parts).astype(np.int64)).to(self.device)

        def greedy_cat(sc, counts):
            sub_off = torch.tensor(np.concatenate([[0], np.cumsum(counts)]), dtype=torch.int32, device=self.device)
            rows, _ = ops.greedy_match(ops.pairwise_distance(sc.float().contiguous(), cand), sub_off, need)
            return rows.cpu().numpy()

        short = [g for g in range(G) if 0 < sizes[g] < need]
        if short:
            match[np.asarray(short)] = greedy_cat(X[order[rows_of(short)]], sizes[short])
        small, small_picks, big, big_inits = [], [], [], []
        for g in range(G):
            n_g = int(sizes[g])
            if n_g == 0:
                continue
            if n_g < need:
                random_fill(match[g], need)
            elif n_g == need:
                small.append(g)
                small_picks.append(np.arange(n_g))
            elif n_g < trunc:
                small.append(g)
                small_picks.append(np.asarray(np.random.choice(n_g, need, replace=False)))
            else:
                big.append(g)
                big_inits.append([init_indices(n_g, need)])
        centers = {}
        if small:
            sc = X[order[rows_of(small, small_picks)]]
            for i, g in enumerate(small):
                centers[g] = sc[i * need:(i + 1) * need]
        if big:
            bsz = sizes[big]
            limits = [adaptive_iter_limit(int(n), need, layer, base_iter_limit=20) for n in bsz]
            bc, _ = fit_segments(X[order[rows_of(big)]].contiguous(), bsz, need, limits, big_inits, half=False)
            for i, g in enumerate(big):
                centers[g] = bc[i * need:(i + 1) * need]
        full = sorted(centers)
        if full:
            match[np.asarray(full)] = greedy_cat(torch.cat([centers[g] for g in full], 0),
                                                 np.full(len(full), need))
        return match

    # ------------------------------------------------------------------------------ sharded training
    def _train_sharded(self, X: np.ndarray, resume: bool) -> Dict:
        """The same training, one process per GPU, every rank holding the same X (the CSV
        is read by every rank; only rows [start, stop) of this rank are copied to its GPU):
        * level 0 (balanced fit_by_min_loss): row-sharded Lloyd (distributed.ShardedLloyd) with the
          row-sharded auction, one all_reduce of the fused [K*D + K] sums per iteration and one of the
          K-bin nearest-centre histogram for the min-loss choice;
        * middle level: segment-parallel -- the parents' rows are regrouped to the rank owning the parent
          (one all_to_all), each rank runs its parents' sub-fits in lockstep (fit_segments with the
          reference's RNG order checked across ranks) and the centres are all-gathered;
        * last level: the two candidate fits row-sharded like level 0; the match-matrix groups
          segment-parallel like the middle level (short groups' greedy rows gathered before the draw
          loop every rank runs identically);
        * reassignment and residuals on each rank's own rows; IDs all-gathered.
        Every rank ends with the single-process model (centres, match matrix, IDs) and the same RNG
        state; rank 0 alone writes checkpoints (resume recomputes the residual chain from them)."""
        from .distributed import Comm, shard_bounds
        cfg = self.config
        if X.shape[1] != cfg.embedding_dim:
            raise ValueError(f"Input dimension {X.shape[1]} does not match config embedding_dim {cfg.embedding_dim}")
        comm = Comm(self.group)
        self._comm = comm
        n = len(X)
        self._n_global = n
        s0, s1 = shard_bounds(n, comm.rank, comm.world)
        t_total = time.time()
        L = len(cfg.layer_clusters)
        current = torch.from_numpy(np.ascontiguousarray(X[s0:s1], dtype=np.float32)).to(self.device)
        self._local_ids = []
        start_layer = 0
        if resume and self.checkpoint_manager:
            start_layer = self.checkpoint_manager.get_last_completed_layer() + 1
        start_layer = int(comm.all_reduce(torch.tensor([start_layer], dtype=torch.int64,
                                                       device=self.device), op=torch.distributed.ReduceOp.MIN).item())
        if start_layer > 0:
            self._load_previous_checkpoints(start_layer)
            self._local_ids = [t.to(self.device).long()[s0:s1] for t in self.result_cluster_ids[:start_layer]]
            current = self._residual_chain(current, self._local_ids, start_layer)
        for layer in range(start_layer, L):
            t0 = time.time()
            n_clusters, need = cfg.layer_clusters[layer], cfg.need_clusters[layer]
            weighted = self._apply_weights(current, layer)
            match = None
            if n_clusters == need:
                centers, ids, residual = self._train_layer_0_sharded(weighted, layer, n)
            elif layer == L - 1:
                centers, ids, residual = self._train_last_layer_sharded(weighted, layer, n)
                match = self.match_matrices[-1]
            else:
                centers, ids, residual = self._train_middle_layer_sharded(weighted, layer)
            self._local_ids.append(ids)
            full = comm.all_gather_rows(ids.long())
            self.cluster_centers_list.append(centers)
            self.result_cluster_ids.append(full)
            if self.checkpoint_manager and comm.rank == 0:
                self.checkpoint_manager.save_layer_checkpoint(layer, full, None, centers, match)
            if layer < L - 1:
                current = residual
            logger.info("[LAYER %d] completed in %.2fs (rank %d of %d)", layer + 1, time.time() - t0, comm.rank,
                        comm.world)
        self.is_trained = True
        if self.checkpoint_manager and comm.rank == 0:
            self.checkpoint_manager.save_metadata({
                "num_layers": L, "embedding_dim": cfg.embedding_dim, "group_dims": cfg.group_dims,
                "hierarchical_weights": cfg.hierarchical_weights, "num_samples": n, "world_size": comm.world})
        logger.info("[TRAINING COMPLETE] Total time: %.2fs", time.time() - t_total)
        return {"cluster_ids": self.result_cluster_ids, "cluster_centers": self.cluster_centers_list}

    def _residual_chain(self, x: torch.Tensor, ids: List[torch.Tensor], n_layers: int) -> torch.Tensor:
        """The training residual after ``n_layers`` completed levels, from their IDs and centres: level 0
        subtracts c0[id0], a middle level its raw block id parent * need + id (:839-904)."""
        cfg = self.config
        cur = x
        for layer in range(min(n_layers, len(cfg.layer_clusters) - 1)):
            w = self._apply_weights(cur, layer)
            raw = ids[0] if layer == 0 else ids[layer - 1] * cfg.need_clusters[layer] + ids[layer]
            cur = self._compute_residuals_with_centers(w, raw, self.cluster_centers_list[layer].float())
        return cur

    def _train_layer_0_sharded(self, X: torch.Tensor, layer: int, n: int):
        """:606-669 over row shards."""
        from .distributed import ShardedLloyd
        cfg = self.config
        n_clusters = cfg.layer_clusters[layer]
        target = 1
        for idx, v in enumerate(cfg.need_clusters):
            if idx != layer:
                target *= v
        iters = adaptive_iter_limit(n, n_clusters, layer, cfg.iter_limit)
        sl = ShardedLloyd(n_clusters, X.contiguous(), n, group=self.group, balanced=True, half=n_clusters >= 512)
        sl.fit_by_min_loss(target, iter_limit=iters)
        centers = sl.cluster_centers.detach().contiguous()
        ids = ops.nearest(X.contiguous(), ops.prepare_centers(centers)).long()
        return centers, ids, self._compute_residuals_with_centers(X, ids, centers)

    def _segment_owners(self, keys_local: torch.Tensor, n_segments: int):
        """Global segment sizes (one all_reduce) and the contiguous segment ranges of the ranks."""
        from .distributed import balanced_ranges
        cnt = torch.bincount(keys_local.long(), minlength=n_segments).to(torch.int64)
        sizes = self._comm.all_reduce(cnt).cpu().numpy().astype(np.int64)
        return sizes, balanced_ranges(sizes, self._comm.world)

    def _train_middle_layer_sharded(self, X: torch.Tensor, layer: int):
        """:671-752, segment-parallel sub-fits."""
        from .distributed import regroup_rows
        cfg = self.config
        comm = self._comm
        cur_need, pre_need = cfg.need_clusters[layer], cfg.need_clusters[layer - 1]
        prev = self._local_ids[layer - 1]
        target = 1
        for idx, v in enumerate(cfg.need_clusters):
            if idx > layer:
                target *= v
        sizes, bounds = self._segment_owners(prev, pre_need)
        xs, _ = regroup_rows(comm, X.contiguous(), prev, bounds)
        limits = [adaptive_iter_limit(int(n_i), cur_need, layer, cfg.iter_limit, is_sub_cluster=True) for n_i in sizes]
        t0 = time.time()
        centers, _ = fit_segments(xs.contiguous(), sizes, cur_need, limits, target_nodes_num=target,
                                  half=cur_need >= 512, comm=comm, owned=(bounds[comm.rank], bounds[comm.rank + 1]))
        logger.info("[LAYER %d] %d segment-parallel sub-fits %.2fs", layer + 1, pre_need, time.time() - t0)
        raw, residual = self._reassign_clusters_middle_layer_with_residuals(X, centers.contiguous(), prev, layer)
        return centers.contiguous(), raw % cur_need, residual

    def _train_last_layer_sharded(self, X: torch.Tensor, layer: int, n: int):
        """:754-837: row-sharded candidate fits, segment-parallel match matrix."""
        from .distributed import ShardedLloyd
        cfg = self.config
        n_clusters, need = cfg.layer_clusters[layer], cfg.need_clusters[layer]
        if len(self._local_ids) < 2:
            raise RuntimeError(
                f"Previous layers cluster IDs not found. "
                f"Expected at least 2 layers but only have {len(self._local_ids)} layers.")
        parts = []
        t0 = time.time()
        for _ in range(2):
            sl = ShardedLloyd(n_clusters, X.contiguous(), n, group=self.group, balanced=True,
                              half=n_clusters >= 512)
            sl.fit(iter_limit=20)
            parts.append(sl.cluster_centers.detach())
        cand = torch.cat(parts, 0).contiguous()
        logger.info("[LAYER %d] row-sharded candidate fits %.2fs", layer + 1, time.time() - t0)
        l1, l2 = self._local_ids[-2], self._local_ids[-1]
        pp_need = cfg.need_clusters[layer - 2]
        match = self._match_matrix_sharded(cand, X, cfg.need_clusters[layer - 1], l1, l2, pp_need, need, 2 * need, layer)
        self.match_matrices.append(match)
        before = l1 * pp_need + l2
        raw, residual = self._reassign_clusters_last_layer_with_residuals(X, cand, before, match, layer)
        ids = self._merge_match_matrix_cluster_ids(match, raw, before)
        return cand, ids, residual

    def _match_matrix_sharded(self, cand, X, prev_need, l1, l2, pp_need, need, trunc, layer) -> np.ndarray:
        """_assign_last_match_matrix (:968-1053) with the (l1, l2) groups owned by ranks (contiguous
        ranges); the draw loop over groups runs identically on every rank."""
        from .distributed import regroup_rows
        comm = self._comm
        G = pp_need * prev_need
        gid = l1.long() * prev_need + l2.long()
        sizes, bounds = self._segment_owners(gid, G)
        o0, o1 = int(bounds[comm.rank]), int(bounds[comm.rank + 1])
        xs, _ = regroup_rows(comm, X.contiguous(), gid, bounds)
        goff = np.concatenate([[0], np.cumsum(sizes[o0:o1])])  # row offsets of my groups in xs
        n_cand = cand.shape[0]
        match = np.zeros((G, n_cand), dtype=np.uint8)

        def rows(g, picks=None):
            a = int(goff[g - o0])
            idx = np.arange(int(sizes[g])) if picks is None else np.asarray(picks)
            return torch.from_numpy(a + idx.astype(np.int64)).to(self.device)

        def greedy_rows(groups, centers_list, counts):
            if not groups:
                return torch.zeros((0, n_cand), dtype=torch.uint8, device=self.device)
            sub_off = torch.tensor(np.concatenate([[0], np.cumsum(counts)]), dtype=torch.int32, device=self.device)
            sc = torch.cat(centers_list, 0).float().contiguous()
            r, _ = ops.greedy_match(ops.pairwise_distance(sc, cand), sub_off, need)
            return r.to(torch.uint8)

        def gather_rows(groups, r):
            g_all = comm.all_gather_rows(torch.tensor(groups, dtype=torch.int64, device=self.device))
            r_all = comm.all_gather_rows(r)
            if len(g_all):
                match[g_all.cpu().numpy()] = r_all.cpu().numpy()

        short = [g for g in range(o0, o1) if 0 < sizes[g] < need]
        gather_rows(short, greedy_rows(short, [xs[rows(g)] for g in short], [int(sizes[g]) for g in short]))
        small, small_picks, big, big_inits = [], [], [], []
        for g in range(G):  # the reference's draw order, on every rank
            n_g = int(sizes[g])
            if n_g == 0:
                continue
            if n_g < need:
                random_fill(match[g], need)
            elif n_g == need:
                small.append(g)
                small_picks.append(np.arange(n_g))
            elif n_g < trunc:
                small.append(g)
                small_picks.append(np.asarray(np.random.choice(n_g, need, replace=False)))
            else:
                big.append(g)
                big_inits.append([init_indices(n_g, need)])
        centers = {}
        for g, pk in zip(small, small_picks):
            if o0 <= g < o1:
                centers[g] = xs[rows(g, pk)]
        if big:
            bsz = sizes[big]
            b0, b1 = int(np.searchsorted(big, o0)), int(np.searchsorted(big, o1))  # my big groups
            xb = xs[torch.cat([rows(big[i]) for i in range(b0, b1)])] if b1 > b0 else xs[:0]
            limits = [adaptive_iter_limit(int(v), need, layer, base_iter_limit=20) for v in bsz]
            bc, _ = fit_segments(xb.contiguous(), bsz, need, limits, big_inits, half=False, comm=comm, owned=(b0, b1))
            for i in range(b0, b1):
                centers[big[i]] = bc[i * need:(i + 1) * need]
        full = sorted(centers)
        gather_rows(full, greedy_rows(full, [centers[g] for g in full], [need] * len(full)))
        return match

    def _load_previous_checkpoints(self, start_layer: int):
        """:1307-1337."""
        for layer in range(start_layer):
            ck = self.checkpoint_manager.load_layer_checkpoint(layer, self.device)
            if not ck:
                raise RuntimeError(f"Incomplete checkpoint data at layer {layer}. "
                                   f"Use --clear-checkpoints flag to start training from scratch.")
            missing = [k for k in ("cluster_ids", "cluster_centers") if k not in ck]
            if missing:
                raise RuntimeError(f"Incomplete checkpoint data at layer {layer}. Missing: {missing}. "
                                   f"Use --clear-checkpoints flag to start training from scratch.")
            self.cluster_centers_list.append(ck["cluster_centers"].float())
            self.result_cluster_ids.append(ck["cluster_ids"])
            if "match_matrix" in ck and ck["match_matrix"].size:
                self.match_matrices.append(ck["match_matrix"])

    # ------------------------------------------------------------------------------------ predict
    def predict(self, X: np.ndarray, reference_quirks: bool = True) -> np.ndarray:
        """:539-581 -> int64 [N, L].  reference_quirks=True reproduces the reference exactly: middle-layer
        residuals use the modulo id (:1143) and the last layer looks up ``match_matrices[layer-1]`` (:1248),
        which does not exist for 3 layers, so its ids are unconstrained raw candidate indices.
        reference_quirks=False gives the training-consistent encode (raw-id residuals, match lookup).
        With a process group the rows are sharded: each rank encodes rows [start, stop) on its GPU
        (``encode_shard``, no collective) and the int32 IDs are all-gathered (SURVEY.md §8e encode)."""
        if not self.is_trained or not self.cluster_centers_list:
            raise RuntimeError("Model not trained. Call train() first or load a trained model.")
        cfg = self.config
        if X.shape[1] != cfg.embedding_dim:
            raise ValueError(f"Input dimension {X.shape[1]} does not match config embedding_dim {cfg.embedding_dim}")
        if self.group is not None:
            from .distributed import Comm, shard_bounds
            comm = Comm(self.group)
            s0, s1 = shard_bounds(len(X), comm.rank, comm.world)
            x = torch.from_numpy(np.ascontiguousarray(X[s0:s1], dtype=np.float32)).to(self.device)
            return self.gather_ids(self.encode_shard(x, reference_quirks)).cpu().numpy().astype(np.int64)
        x = torch.from_numpy(np.ascontiguousarray(X, dtype=np.float32)).to(self.device)
        return self.encode_shard(x, reference_quirks).cpu().numpy().astype(np.int64)

    def _encoder(self, reference_quirks: bool):
        """The fused encoder of the trained codebooks, cached per semantics.  The key holds each centre
        tensor's identity and in-place version counter and each match matrix's identity, so assigning new
        codebooks or changing a centre tensor in place rebuilds it; train / load_model drop the cache, and
        ``invalidate_encoder`` does after an in-place edit of a numpy match matrix."""
        from .encode import LevelSemantics, RQEncoder
        # the cache entry holds the objects themselves (not their id(), which a new object can reuse once the
        # old one is freed) and compares them by identity, plus each tensor's in-place version counter
        objs = (list(self.cluster_centers_list), list(self.match_matrices))
        vers = (bool(reference_quirks), tuple(getattr(c, "_version", 0) for c in self.cluster_centers_list))
        cache = getattr(self, "_enc_cache", None)
        if cache is not None and cache[0] == vers and len(cache[1][0]) == len(objs[0]) and \
                len(cache[1][1]) == len(objs[1]) and all(a is b for a, b in zip(cache[1][0], objs[0])) and \
                all(a is b for a, b in zip(cache[1][1], objs[1])):
            return cache[2]
        cfg = self.config
        L = len(cfg.layer_clusters)
        match = None
        if L >= 3 and not reference_quirks:
            if not self.match_matrices:
                raise RuntimeError("Model has no match matrix for the last layer.")
            match = torch.as_tensor(np.asarray(self.match_matrices[-1], dtype=np.uint8))
        # training-consistent: raw block ids, the match lookup, residuals of the weighted rows (:442)
        sem = LevelSemantics(match_lookup=not reference_quirks, residual_global_id=not reference_quirks,
                             residual_from_weighted=not reference_quirks)
        enc = RQEncoder([c.float() for c in self.cluster_centers_list], cfg.need_clusters, match=match,
                        group_dims=cfg.group_dims, weights=cfg.hierarchical_weights, semantics=sem, device=self.device)
        self._enc_cache = (vers, objs, enc)
        return enc

    def invalidate_encoder(self) -> None:
        """Drop the cached fused encoder (the next predict / encode_shard rebuilds it from the codebooks)."""
        self._enc_cache = None

    def encode_shard(self, x: torch.Tensor, reference_quirks: bool = False) -> torch.Tensor:
        """Encode device-resident rows (this rank's shard): int32 [n, L] on the device.  The hot path of
        ``predict`` and of bench.py (no host copies, no collective)."""
        L = len(self.config.layer_clusters)
        if x.shape[0] == 0:
            return torch.zeros((0, L), dtype=torch.int32, device=self.device)
        return self._encoder(reference_quirks).encode(x)

    def gather_ids(self, ids_local: torch.Tensor) -> torch.Tensor:
        """All ranks' IDs in row order (one variable-size all_gather of int32 rows)."""
        if self.group is None:
            return ids_local
        from .distributed import Comm
        return Comm(self.group).all_gather_rows(ids_local)

    # ------------------------------------------------------------------------------------ persistence
    def save_model(self, model_dir: str):
        """:1340-1360: config.json + cluster_centers.npz (+ match_matrices.npz)."""
        d = Path(model_dir)
        d.mkdir(parents=True, exist_ok=True)
        with open(d / "config.json", "w") as f:
            json.dump(asdict(self.config), f, indent=2)
        np.savez(d / "cluster_centers.npz", **{f"layer_{i}": _np(c) for i, c in enumerate(self.cluster_centers_list)})
        if self.match_matrices:
            np.savez(d / "match_matrices.npz",
                     **{f"match_{i}": np.asarray(m, dtype=np.uint8) for i, m in enumerate(self.match_matrices)})

    def load_model(self, model_dir: str):
        """:1362-1391."""
        self.invalidate_encoder()
        d = Path(model_dir)
        cf = d / "config.json"
        if cf.exists():
            with open(cf) as f:
                for key, value in json.load(f).items():
                    if hasattr(self.config, key):
                        setattr(self.config, key, value)
        cc = d / "cluster_centers.npz"
        if cc.exists():
            with np.load(cc, allow_pickle=False) as z:
                self.cluster_centers_list = [torch.from_numpy(z[f"layer_{i}"]).to(self.device)
                                             for i in range(len(z.files))]
        mm = d / "match_matrices.npz"
        if mm.exists():
            with np.load(mm, allow_pickle=False) as z:
                self.match_matrices = [z[f"match_{i}"] for i in range(len(z.files))]
        self.is_trained = len(self.cluster_centers_list) > 0

    def get_training_status(self) -> Dict:
        """:1393-1409."""
        L = len(self.config.layer_clusters)
        if self.checkpoint_manager:
            last = self.checkpoint_manager.get_last_completed_layer()
            return {"is_trained": self.is_trained, "last_completed_layer": last, "total_layers": L,
                    "can_resume": last >= 0}
        return {"is_trained": self.is_trained, "last_completed_layer": -1, "total_layers": L, "can_resume": False}


class hierarchicalRqClusterParams:
    """hierarchical_rq_kmeans.py:1413-1445 (compatibility parameter class)."""

    def __init__(self, layer_clusters=None, need_clusters=None, embedding_dim=1024, group_dims=None,
                 hierarchical_weights=None):
        layer_clusters = layer_clusters if layer_clusters is not None else [128, 256, 256]
        need_clusters = need_clusters if need_clusters is not None else [128, 128, 128]
        group_dims = group_dims if group_dims is not None else embedding_dim
        hierarchical_weights = hierarchical_weights if hierarchical_weights is not None else 1.0
        self.config = HierarchicalRQKMeansConfig(layer_clusters=layer_clusters, need_clusters=need_clusters,
                                                 embedding_dim=embedding_dim, group_dims=group_dims,
                                                 hierarchical_weights=hierarchical_weights)
        self.layer_clusters = self.config.layer_clusters
        self.need_clusters = self.config.need_clusters
        self.embedding_dim = self.config.embedding_dim
        self.group_dims = self.config.group_dims
        self.hierarchical_weights = self.config.hierarchical_weights
