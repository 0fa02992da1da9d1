"""The reference's training driver, src/semantic_id_generator/train_semantic_ids.py:35-365
(``SemanticIDTrainer``), on the MI355X path: CSV -> HierarchicalRQKMeans.train -> save_model ->
training_config.json -> song_semantic_ids.jsonl -> training_statistics.json, with the same file names,
directory layout, contents and byte encoding.

``config`` is any object with the attributes the reference's ``Config`` exposes to this class:
``output_dir``, ``model_dir``, ``data.song_vectors_file``, ``data.semantic_ids_file``, ``h_rqkmeans`` and
``h_rqkmeans_test`` (config.py:42-58, 106-115).  The argparse CLI (:368-434) is not mirrored.

Multi-GPU (``group`` set, one process per GPU): every rank reads the CSV, trains on its contiguous row
block (``HierarchicalRQKMeans(group=...)``), and the semantic IDs are gathered to rank 0,
which alone writes the model, the jsonl and the side files.
"""
from __future__ import annotations

import logging
import os
from pathlib import Path
from typing import Dict, List, Tuple

import numpy as np
import torch

from . import io as rq_io
from .hierarchical_rq_kmeans import HierarchicalRQKMeans

logger = logging.getLogger(__name__)


class SemanticIDTrainer:
    """train_semantic_ids.py:35-365."""

    def __init__(self, config, use_test_config: bool = False, device=None, group=None):
        self.config = config
        self.use_test_config = use_test_config
        self.rqkmeans_config = config.h_rqkmeans_test if use_test_config else config.h_rqkmeans
        self.device = device
        self.group = group
        self.rank = 0
        if group is not None:
            import torch.distributed as dist
            self.rank = dist.get_rank(group)
        self.output_dir = Path(config.output_dir) / "semantic_id"
        self.model_dir = Path(config.model_dir) / "semantic_id"
        self.checkpoint_dir = self.output_dir / "checkpoints"
        if self.rank == 0:
            for d in (self.output_dir, self.model_dir, self.checkpoint_dir):
                d.mkdir(parents=True, exist_ok=True)

    def load_song_vectors(self, max_samples: int = None) -> Tuple[List[str], np.ndarray]:
        """:72-131 (native reader, the reference's skip rules and fp16 rule)."""
        path = self.config.data.song_vectors_file
        if not os.path.isfile(path):
            raise FileNotFoundError(f"Song vector file not found: {path}")
        ids, x = rq_io.load_song_vectors(path, self.rqkmeans_config.embedding_dim, self.rqkmeans_config.layer_clusters,
                                         limit=max_samples)
        logger.info("Successfully loaded %d song vectors", len(ids))
        return ids, x

    def train(self, resume: bool = True) -> Dict:
        """:133-207."""
        max_samples = 100000 if self.use_test_config else None
        song_ids, vectors = self.load_song_vectors(max_samples=max_samples)
        vectors_np = np.asarray(vectors, dtype=np.float32) if vectors.dtype != np.float32 else vectors
        # every rank reads the checkpoints on resume; only rank 0 writes them
        model = HierarchicalRQKMeans(config=self.rqkmeans_config, checkpoint_dir=str(self.checkpoint_dir),
                                     device=self.device, group=self.group)
        logger.info("Training status: %s", model.get_training_status())
        train_result = model.train(vectors_np, resume=resume)
        stats = None
        semantic_ids = None
        if self.rank == 0:
            model.save_model(str(self.model_dir))
            self._save_config(model)
            semantic_ids = self._generate_semantic_ids(song_ids, train_result)
            self._save_semantic_ids(semantic_ids)
            stats = self._generate_statistics(semantic_ids)
            self._save_statistics(stats)
        return {"model": model, "semantic_ids": semantic_ids, "statistics": stats, "song_ids": song_ids}

    def _generate_semantic_ids(self, song_ids: list, train_result: Dict) -> Dict:
        """:209-237 (one host copy per level instead of a per-element .item() loop; a song id repeated in
        the CSV keeps its last row's IDs, as the reference's dict assignment does)."""
        levels = [np.asarray(t.detach().cpu().numpy() if isinstance(t, torch.Tensor) else t, dtype=np.int64)
                  for t in train_result["cluster_ids"]]
        ids = np.stack(levels, 1) if levels else np.zeros((len(song_ids), 0), dtype=np.int64)
        return {sid: [int(v) for v in row] for sid, row in zip(song_ids, ids)}

    def _save_semantic_ids(self, semantic_ids: Dict):
        """:239-264."""
        n_unique = rq_io.write_semantic_ids(self.config.data.semantic_ids_file, semantic_ids)
        logger.info("Saved %d total IDs, %d unique semantic IDs.", len(semantic_ids), n_unique)

    def _save_config(self, model: HierarchicalRQKMeans):
        """:266-288."""
        rq_io.write_json(str(self.output_dir / "training_config.json"),
                         rq_io.training_config(model.config, self.use_test_config))

    def _generate_statistics(self, semantic_ids: Dict) -> Dict:
        """:290-333."""
        return rq_io.semantic_id_statistics(semantic_ids, self.rqkmeans_config.need_clusters)

    def _save_statistics(self, stats: Dict):
        """:335-365."""
        rq_io.write_json(str(self.output_dir / "training_statistics.json"), stats)
