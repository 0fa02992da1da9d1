"""ORACLE — TEST INFRASTRUCTURE ONLY.  Never imported by the product package.

The reference's song-vector CSV reader restated with the same Python machinery it uses
(``csv.reader`` over a universal-newline text file, ``np.array(row[1:], dtype=np.float32)`` per record,
``.half()`` when any layer_clusters entry exceeds 512): simplified_semantic_id_generator.py:38-76 and
train_semantic_ids.py:72-131.  The checker for the native reader ``librqsid_io.so``
(``generative_ranking_recommender_amd/io.py``, ``tests/test_csv_loader.py``).
"""
from __future__ import annotations

import csv
import os
from typing import List, Sequence, Tuple

import numpy as np


def load_song_vectors(path: str, embedding_dim: int, layer_clusters: Sequence[int] = (),
                      limit: int | None = None) -> Tuple[List[str], np.ndarray, int]:
    """(song_ids, vectors, non-numeric rows skipped); simplified…:48-76."""
    if not os.path.isfile(path):
        raise FileNotFoundError(f"The specified data file was not found: {path}")
    song_ids: List[str] = []
    rows: List[np.ndarray] = []
    nonnumeric = 0
    with open(path, "r", encoding="utf-8") as f:
        for i, row in enumerate(csv.reader(f)):
            if limit and i >= limit:
                break
            if len(row) < 2:
                continue
            try:
                embed = np.array(row[1:], dtype=np.float32)
            except ValueError:
                nonnumeric += 1
                continue
            if embed.shape[0] == embedding_dim:
                song_ids.append(row[0])
                rows.append(embed)
    if not song_ids:
        raise ValueError("No valid data with the correct embedding dimension found in the CSV file.")
    x = np.vstack(rows)
    if any(n > 512 for n in layer_clusters):
        x = x.astype(np.float16)
    return song_ids, x, nonnumeric
