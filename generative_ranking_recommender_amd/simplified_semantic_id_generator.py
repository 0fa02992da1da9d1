"""``SimplifiedHierarchicalRQ`` on MI355X — the drop-in for
src/semantic_id_generator/simplified_semantic_id_generator.py.

Reference semantics kept: un-normalised residuals (:91, :167), +inf masks (:153-160, :325), zero
placeholder centres for empty parents (:113-118), sampling with replacement for small parents
(:125-127), raw candidate indices as last-layer ids (:305-331), the dynamic match matrix of :247-303
(random candidate draws for empty groups, greedy unique-nearest, random fill), per-song id lists
(a song id repeated in the CSV accumulates ids, :183, 234-236) and the jsonl writer (:368-385).
Arithmetic runs in librqsid.so (see balancekmeans / hierarchical_rq_kmeans); models are saved as
``.npz`` instead of pickle.
"""
from __future__ import annotations

import json
import logging
from dataclasses import asdict
from pathlib import Path
from typing import Dict, List

import numpy as np
import torch

from . import io as rq_io
from . import ops
from .balancekmeans import KMeans, _device, fit_segments, init_indices
from .hierarchical_rq_kmeans import HierarchicalRQKMeansConfig, group_rows, masked_assign, random_fill

logger = logging.getLogger(__name__)


class SimplifiedHierarchicalRQ:
    def __init__(self, config: HierarchicalRQKMeansConfig, device=None):
        self.config = config
        self.device = _device(device)
        self.trained_kmeans_models: List = []
        self.dynamic_match_matrix = None
        self.final_layer_centers = None
        self.middle_layer_centers = None
        # per-parent / per-group sub-fits in lockstep (True) or one after another like the reference
        # (False); both keep the reference's numpy draw order (``fit`` draws only its start)
        self.batched_sub_fits = True

    def _load_data(self, data_path: str, limit: int = None):
        """:38-76 -> (song_ids, tensor fp16/fp32 on the host)."""
        ids, x = rq_io.load_song_vectors(data_path, self.config.embedding_dim, self.config.layer_clusters, limit)
        return ids, torch.from_numpy(x)

    def _get_residuals(self, data: torch.Tensor, kmeans: KMeans) -> torch.Tensor:
        """:78-96: r = x - c[nearest] (no normalisation)."""
        c = kmeans.cluster_centers.float().contiguous()
        ids = ops.nearest(data, ops.prepare_centers(c))
        return ops.residual(data, c, ids, normalize=False)

    def _train_middle_layer(self, data: torch.Tensor, prev_cluster_ids: torch.Tensor, layer_idx: int):
        """:98-174."""
        cfg = self.config
        n_clusters, n_need = cfg.layer_clusters[layer_idx], cfg.need_clusters[layer_idx]
        prev_n_need = cfg.need_clusters[layer_idx - 1]
        use_half = n_clusters > 512
        order, off = group_rows(prev_cluster_ids, prev_n_need)
        if self.batched_sub_fits:
            combined = self._batched_middle_centers(data, order, off, prev_n_need, n_need, use_half)
        else:
            combined = self._sequential_middle_centers(data, order, off, prev_n_need, n_need, use_half)
        self.middle_layer_centers = combined
        cand = ops.contiguous_candidates(prev_n_need, n_need, self.device)
        _, glob = masked_assign(data, combined, prev_cluster_ids, cand, prev_n_need)
        residuals = ops.residual(data, combined, glob, normalize=False)
        return glob.long() % n_need, residuals

    def _batched_middle_centers(self, data, order, off, prev_n_need, n_need, use_half):
        """The per-parent ``fit`` runs of :98-140 in lockstep (balancekmeans.batched_fit).  ``fit`` draws
        only its start from numpy, so drawing every parent's start (or its with-replacement sample when
        it has fewer rows than centres) in parent order keeps the reference's RNG sequence."""
        sizes = np.diff(off).astype(np.int64)
        d = data.shape[1]
        picks, fits, inits = {}, [], []
        for i in range(prev_n_need):
            n_i = int(sizes[i])
            if n_i == 0:
                continue
            if n_i < n_need:
                picks[i] = np.asarray(np.random.choice(n_i, n_need, replace=True))
            else:
                fits.append(i)
                inits.append([init_indices(n_i, n_need)])
        out = torch.zeros(prev_n_need * n_need, d, device=self.device)
        for i, p in picks.items():
            out[i * n_need:(i + 1) * n_need] = data[order[off[i] + torch.from_numpy(p).to(self.device)]]
        if fits:
            fsz = sizes[fits]
            rows = torch.from_numpy(np.concatenate([np.arange(off[i], off[i + 1]) for i in fits])).to(self.device)
            c, _ = fit_segments(data[order[rows]].contiguous(), fsz, n_need, [self.config.iter_limit] * len(fits),
                                inits, half=use_half)
            sel = torch.cat([torch.arange(i * n_need, (i + 1) * n_need) for i in fits]).to(self.device)
            out[sel] = c
        return out.contiguous()

    def _sequential_middle_centers(self, data, order, off, prev_n_need, n_need, use_half):
        """:98-140 one parent after another (the reference's order)."""
        cfg = self.config
        subs = []
        for i in range(prev_n_need):
            n_i = int(off[i + 1] - off[i])
            if n_i == 0:
                subs.append(torch.zeros(n_need, data.shape[1], device=self.device))
                continue
            sub = data[order[off[i]:off[i + 1]]]
            if n_i < n_need:
                subs.append(sub[torch.from_numpy(np.random.choice(n_i, n_need, replace=True)).to(self.device)])
            else:
                km = KMeans(n_clusters=n_need, device=self.device, balanced=True)
                km.fit(X=sub, iter_limit=cfg.iter_limit, half=use_half, tqdm_flag=False)
                subs.append(km.cluster_centers)
        return torch.cat(subs).float().contiguous()

    def train(self, data_path: str, data_limit: int = None):
        """:176-245."""
        song_ids, emb = self._load_data(data_path, limit=data_limit)
        return self.train_rows(song_ids, emb)

    def train_rows(self, song_ids: List[str], emb: torch.Tensor):
        """The body of train (:185-245) on rows already loaded (host or device tensor, fp32 or fp16)."""
        cfg = self.config
        current = emb.float().to(self.device).contiguous()
        all_ids: Dict[str, List[int]] = {sid: [] for sid in song_ids}
        previous = None
        L = len(cfg.layer_clusters)
        for layer_idx in range(L):
            n_clusters = cfg.layer_clusters[layer_idx]
            use_half = n_clusters > 512
            if layer_idx == 0:
                km = KMeans(n_clusters=n_clusters, device=self.device, balanced=True)
                km.fit_by_min_loss(X=current, target_nodes_num=np.prod(cfg.need_clusters[1:]),
                                   iter_limit=cfg.iter_limit, half=use_half)
                self.trained_kmeans_models.append(km)
                ids = km.predict(current)
            elif layer_idx < L - 1:
                ids, current = self._train_middle_layer(current, previous.to(self.device), layer_idx)
                self.trained_kmeans_models.append(None)
            else:
                p1 = KMeans(n_clusters=n_clusters, device=self.device, balanced=True)
                p1.fit(X=current, iter_limit=20, half=use_half)
                p2 = KMeans(n_clusters=n_clusters, device=self.device, balanced=True)
                p2.fit(X=current, iter_limit=20, half=use_half)
                cand = torch.cat([p1.cluster_centers, p2.cluster_centers], 0).float().contiguous()
                self.final_layer_centers = cand
                self.trained_kmeans_models.append(None)
                # the reference reads previous ids back per song (:223-224): a repeated song id
                # yields that song's FIRST occurrence's ids
                l1 = torch.tensor([all_ids[s][layer_idx - 2] for s in song_ids], device=self.device)
                l2 = torch.tensor([all_ids[s][layer_idx - 1] for s in song_ids], device=self.device)
                self.dynamic_match_matrix = self._get_dynamic_match_matrix(current, l1, l2, cand)
                ids = self._predict_with_dynamic_matrix(current, l1, l2, cand, self.dynamic_match_matrix)
            ids_np = ids.cpu().numpy() if isinstance(ids, torch.Tensor) else np.asarray(ids)
            for i, s in enumerate(song_ids):
                all_ids[s].append(int(ids_np[i]))
            previous = torch.as_tensor(ids_np)
            if layer_idx == 0:
                current = self._get_residuals(current, self.trained_kmeans_models[0])
        self.semantic_ids = all_ids
        return None

    def _get_dynamic_match_matrix(self, data, prev_ids_l1, prev_ids_l2, candidate_centers) -> torch.Tensor:
        """:247-303."""
        cfg = self.config
        n_prev1, n_prev2, n_need = cfg.need_clusters[-3], cfg.need_clusters[-2], cfg.need_clusters[-1]
        n_cand = candidate_centers.shape[0]
        G = n_prev1 * n_prev2
        gid = prev_ids_l1.long() * n_prev2 + prev_ids_l2.long()
        order, off = group_rows(gid, G)
        match = np.zeros((G, n_cand), dtype=np.uint8)
        deferred, deferred_c = [], []

        def greedy(centers_list):
            sizes = [len(c) for c in centers_list]
            sub_off = torch.tensor(np.concatenate([[0], np.cumsum(sizes)]), dtype=torch.int32, device=self.device)
            sc = torch.cat(centers_list, 0).float().contiguous()
            rows, _ = ops.greedy_match(ops.pairwise_distance(sc, candidate_centers), sub_off, max(sizes))
            return rows.cpu().numpy()

        if self.batched_sub_fits:
            return self._batched_dynamic_match(data, order, off, G, n_need, candidate_centers, match)
        for g in range(G):
            n_g = int(off[g + 1] - off[g])
            if n_g == 0:
                centers = candidate_centers[torch.from_numpy(np.random.choice(n_cand, n_need, replace=False))
                                            .to(self.device)]
            elif n_g <= n_need:
                centers = data[order[off[g]:off[g + 1]]]
            else:
                km = KMeans(n_clusters=n_need, device=self.device, balanced=True)
                km.fit(X=data[order[off[g]:off[g + 1]]], iter_limit=20, tqdm_flag=False)
                centers = km.cluster_centers
            if len(centers) < n_need:
                match[g] = greedy([centers])[0]
                random_fill(match[g], n_need)
            else:
                deferred.append(g)
                deferred_c.append(centers)
        if deferred:
            match[np.asarray(deferred)] = greedy(deferred_c)
        return torch.from_numpy(match.astype(np.float32))

    def _batched_dynamic_match(self, data, order, off, G, n_need, candidate_centers, match):
        """:247-303 with the groups' ``fit`` runs in lockstep; every numpy draw stays in group order (an
        empty group's candidate sample, a short group's random fill after its greedy step, a large
        group's start)."""
        sizes = np.diff(off).astype(np.int64)
        n_cand = candidate_centers.shape[0]

        def greedy_cat(sc, counts):
            sub_off = torch.tensor(np.concatenate([[0], np.cumsum(counts)]), dtype=torch.int32, device=self.device)
            rows, _ = ops.greedy_match(ops.pairwise_distance(sc.float().contiguous(), candidate_centers), sub_off,
                                       int(max(counts)))
            return rows.cpu().numpy()

        def rows_of(groups):
            return torch.from_numpy(np.concatenate([np.arange(off[g], off[g + 1]) for g in groups])).to(self.device)

        short = [g for g in range(G) if 0 < sizes[g] < n_need]
        if short:
            match[np.asarray(short)] = greedy_cat(data[order[rows_of(short)]], sizes[short])
        centers, fits, inits = {}, [], []
        for g in range(G):
            n_g = int(sizes[g])
            if n_g == 0:
                centers[g] = candidate_centers[torch.from_numpy(np.random.choice(n_cand, n_need, replace=False))
                                               .to(self.device)]
            elif n_g < n_need:
                random_fill(match[g], n_need)
            elif n_g == n_need:
                centers[g] = data[order[off[g]:off[g + 1]]]
            else:
                fits.append(g)
                inits.append([init_indices(n_g, n_need)])
        if fits:
            c, _ = fit_segments(data[order[rows_of(fits)]].contiguous(), sizes[fits], n_need, [20] * len(fits), inits)
            for i, g in enumerate(fits):
                centers[g] = c[i * n_need:(i + 1) * n_need]
        full = sorted(centers)
        if full:
            match[np.asarray(full)] = greedy_cat(torch.cat([centers[g] for g in full], 0), np.full(len(full), n_need))
        return torch.from_numpy(match.astype(np.float32))

    def _predict_with_dynamic_matrix(self, data, prev_ids_l1, prev_ids_l2, candidate_centers, match_matrix):
        """:305-331: raw candidate index of the nearest allowed column."""
        n_prev2 = self.config.need_clusters[-2]
        sub = prev_ids_l1.long().to(self.device) * n_prev2 + prev_ids_l2.long().to(self.device)
        m = torch.as_tensor(match_matrix).to(self.device).to(torch.uint8)
        if sub.numel() and int(sub.max().item()) >= m.shape[0]:
            raise IndexError(f"index {int(sub.max().item())} is out of bounds for dimension 0 with size {m.shape[0]}")
        cand = ops.match_to_candidates(m)
        _, glob = masked_assign(data, candidate_centers, sub, cand, m.shape[0])
        return glob.long()

    def save_model(self, path: str):
        """:333-343 (npz): centres of layer 0, middle and final layers + the match matrix."""
        arrays = {"config": np.frombuffer(json.dumps(asdict(self.config)).encode(), dtype=np.uint8)}
        for i, km in enumerate(self.trained_kmeans_models):
            if km is not None:
                arrays[f"layer_{i}_centers"] = km.cluster_centers.detach().cpu().numpy()
        if self.middle_layer_centers is not None:
            arrays["middle_layer_centers"] = self.middle_layer_centers.detach().cpu().numpy()
        if self.final_layer_centers is not None:
            arrays["final_layer_centers"] = self.final_layer_centers.detach().cpu().numpy()
        if self.dynamic_match_matrix is not None:
            arrays["dynamic_match_matrix"] = np.asarray(self.dynamic_match_matrix, dtype=np.uint8)
        arrays["n_layers"] = np.int64(len(self.trained_kmeans_models))
        np.savez(path, **arrays)

    @classmethod
    def load_model(cls, path: str, device=None):
        with np.load(path, allow_pickle=False) as z:
            cfg = HierarchicalRQKMeansConfig(**json.loads(bytes(z["config"]).decode()))
            model = cls(cfg, device=device)
            for i in range(int(z["n_layers"])):
                key = f"layer_{i}_centers"
                if key in z.files:
                    c = torch.from_numpy(z[key]).to(model.device)
                    model.trained_kmeans_models.append(KMeans(n_clusters=c.shape[0], cluster_centers=c,
                                                              device=model.device))
                else:
                    model.trained_kmeans_models.append(None)
            if "middle_layer_centers" in z.files:
                model.middle_layer_centers = torch.from_numpy(z["middle_layer_centers"]).to(model.device)
            if "final_layer_centers" in z.files:
                model.final_layer_centers = torch.from_numpy(z["final_layer_centers"]).to(model.device)
            if "dynamic_match_matrix" in z.files:
                model.dynamic_match_matrix = torch.from_numpy(z["dynamic_match_matrix"].astype(np.float32))
        return model

    def save_semantic_ids(self, output_file: str):
        """:368-385."""
        if not hasattr(self, "semantic_ids"):
            logger.warning("No semantic IDs generated yet. Run train() or predict() first.")
            return
        n_unique = rq_io.write_semantic_ids(output_file, self.semantic_ids)
        logger.info("Saved %d total IDs, %d unique semantic IDs.", len(self.semantic_ids), n_unique)
