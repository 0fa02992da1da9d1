"""Multi-level residual-quantisation encoder on the HIP kernels (the bench hot path).

One ``RQEncoder`` holds the trained codebooks of every level, already prepared
for ``rqsid_assign`` (fp16 copy, norms, candidate lists), and turns an fp32
[N, D] device matrix into int32 [N, L] semantic IDs with no host round trip.

Level semantics:

* level 0: nearest of ``need[0]`` centres (``_predict_layer_0``,
  hierarchical_rq_kmeans.py:1146-1173; simplified :202).
* middle level l: segment = the previous level's ID p; allowed centres are the
  block ``[p*need[l], (p+1)*need[l])``; the ID is the local index in the block
  (``_predict_middle_layer`` :1175-1233 / ``_reassign_clusters_middle_layer_with_
  residuals`` :839-904 / simplified :145-172).
* last level: group = ``ids[l-2]*mult + ids[l-1]`` (mult = ``need[l-2]`` in the
  hierarchical path :824,1256, ``need[-2]`` in the simplified path :311); allowed
  centres = the group's match-matrix row.  ID = rank of the chosen column among
  the allowed ones (``_merge_match_matrix_cluster_ids`` :1055-1086) or the raw
  column (simplified :305-331).

Switches reproduce the reference's predict-time quirks (Appendix A item 2):
``match_lookup`` False = the `match_matrices[layer-1]` miss at :1248 (the last
level is then an unconstrained argmin over every candidate, raw IDs);
``residual_global_id`` False = predict's residual indexing ``centers[id % need]``
(:577,1143) instead of the raw block index the trainer uses (:901).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import List, Optional, Sequence

import torch

from . import ops


@dataclass
class LevelSemantics:
    normalize_residual: bool = True      # hierarchical: r/(||r||+1e-8) per group; simplified: plain
    match_lookup: bool = True            # False: reference predict bug (:1248)
    residual_global_id: bool = True      # False: reference predict bug (:1143 with modded ids)
    remap_last: bool = True              # hierarchical rank remap; simplified keeps raw column
    last_group_mult: str = "need_l_minus_2"  # or "need_minus_2" (simplified)
    residual_from_weighted: bool = False  # train-time residuals use weighted data (:442 vs :577)


HIERARCHICAL_PREDICT_REFERENCE = LevelSemantics(match_lookup=False, residual_global_id=False)
HIERARCHICAL_TRAIN = LevelSemantics(residual_from_weighted=True)
SIMPLIFIED = LevelSemantics(normalize_residual=False, remap_last=False, last_group_mult="need_minus_2")


class RQEncoder:
    def __init__(self, centers: Sequence[torch.Tensor], need_clusters: Sequence[int],
                 match: Optional[torch.Tensor] = None, group_dims: Sequence[int] = (),
                 weights: Optional[Sequence[Sequence[float]]] = None,
                 semantics: LevelSemantics = LevelSemantics(), device=None):
        device = device or torch.device("cuda", torch.cuda.current_device())
        self.device = device
        self.L = len(centers)
        self.need = list(need_clusters)
        self.sem = semantics
        self.dim = centers[0].shape[1]
        self.group_dims = list(group_dims) or [self.dim]
        self.weights = None
        if weights is not None and any(any(w != 1.0 for w in ws) for ws in weights):
            self.weights = [list(ws) for ws in weights]
        self.pcs = [ops.prepare_centers(c.to(device)) for c in centers]
        self.cands: List[Optional[ops.Candidates]] = []
        self.has_penalty = False
        for l in range(self.L):
            if l == 0:
                c = ops.Candidates(torch.zeros(1, dtype=torch.int32, device=device),
                                   torch.full((1,), self.pcs[0].k, dtype=torch.int32, device=device), self.pcs[0].k)
            elif l < self.L - 1:
                c = ops.contiguous_candidates(self.need[l - 1], self.need[l], device)
            else:
                if match is not None and semantics.match_lookup:
                    m = match.to(device)
                    c = ops.match_to_candidates(m)
                    self.has_penalty = bool((c.count == 0).any().item())
                    self.n_groups = m.shape[0]
                else:
                    k = self.pcs[l].k
                    c = ops.Candidates(torch.zeros(1, dtype=torch.int32, device=device),
                                       torch.full((1,), k, dtype=torch.int32, device=device), k)
            # bitwise-duplicate centres can never be the first minimum: drop them from the lists
            self.cands.append(ops.dedup_candidates(c, self.pcs[l].centers))
        self._ws = None
        self._bws = {}  # n_segments -> reusable rqsid_bucket workspace (sticky error word)
        self.last_rescored = []
        self.force_materialized = False

    def _workspace(self, n):
        if self._ws is None or self._ws.n_rows < n:
            if self._ws is not None:  # a bigger workspace replaces it: keep what its word recorded
                ops.check_error_words([self._ws.error_word()], "RQEncoder")
            self._ws = ops.AssignWorkspace(n, self.device)
        return self._ws

    def _bucket(self, keys, n_segments):
        ws = self._bws.get(n_segments)
        if ws is None:
            ws = self._bws[n_segments] = ops.bucket_workspace(n_segments, self.device)
        return ops.bucket(keys, n_segments, workspace=ws)

    def error_words(self):
        """Device views of the sticky error words this encoder's calls write (assign and bucketing)."""
        return ([self._ws.error_word()] if self._ws is not None else []) + \
            [ops.bucket_error_word(w, s) for s, w in self._bws.items()]

    def check_errors(self) -> None:
        """Raise RuntimeError if any counter-driven write of this encoder's calls was dropped (one host sync)."""
        ops.check_error_words(self.error_words(), "RQEncoder.encode")

    def _weighted(self, x, l):
        if self.weights is None:
            return x
        return ops.scale_groups(x, self.group_dims, self.weights[l])

    def _last_mult(self) -> int:
        return self.need[self.L - 3] if self.sem.last_group_mult == "need_l_minus_2" else self.need[-2]

    @property
    def fused(self) -> bool:
        """Residuals computed inside the assignment kernels (no residual matrices in HBM).

        The kernels subtract per-SEGMENT residual centres, so the last level fuses only when its
        group id ``l1*mult + l2`` determines (l1, l2), i.e. mult >= need[1] (true for every shipped
        preset; the reference itself only makes sense there, Appendix A item 8), and only when the
        match lookup is on (the reference-bug predict mode is one unconstrained segment)."""
        if self.L > 3 or len(self.group_dims) != 1 or self.weights is not None or self.force_materialized:
            return False
        if self.L == 3 and not (self.sem.match_lookup and self._last_mult() >= self.need[1]):
            return False
        return True

    def encode(self, x: torch.Tensor, count_rescored: bool = False, check: Optional[bool] = None) -> torch.Tensor:
        """x: f32 [N, D] on the device -> int32 [N, L] semantic IDs (a transposed view of the
        level-major [L, N] buffer the kernels write; no copy).  ``check`` (default: on unless the stream is
        being captured into a graph): read the device error words after the call (one host sync) and raise
        if a counter-driven list write was dropped; a captured step checks with ``check_errors()``."""
        if check is None:
            check = not torch.cuda.is_current_stream_capturing()
        if x.dim() != 2 or x.shape[1] != self.dim:
            raise ValueError(f"Input dimension {x.shape[-1]} does not match config embedding_dim {self.dim}")
        x = x.float().contiguous()
        if self.L == 2:
            raise IndexError("list index out of range")  # reference: all_cluster_ids[-2] with one level
        n = x.shape[0]
        out = torch.empty((self.L, n), dtype=torch.int32, device=x.device)
        if n == 0:
            self.last_rescored = []
            return out.t()
        ws = self._workspace(n)
        self.last_rescored = []
        if self.fused:
            self._encode_fused(x, out, ws, count_rescored)
        else:
            self._encode_materialized(x, out, ws, count_rescored)
        if check:
            self.check_errors()
        return out.t()

    def _last_level_buckets(self, out, l, n, device):
        if self.sem.match_lookup:
            mult = self.need[l - 2] if self.sem.last_group_mult == "need_l_minus_2" else self.need[-2]
            grp = out[l - 2] * mult + out[l - 1]
            # the reference indexes match_matrix_np[before] (hierarchical_rq_kmeans.py:1279-1281) and raises
            # IndexError past the last group; bucketing would silently drop such rows.  Check on the device
            # values only when the largest possible id can reach it (never for the shipped presets:
            # need[l-2] == need[l-1]), so the common encode has no host sync here.
            if (self.need[l - 2] - 1) * mult + self.need[l - 1] - 1 >= self.n_groups:
                gmax = int(grp.max().item())
                if gmax >= self.n_groups:
                    raise IndexError(f"index {gmax} is out of bounds for axis 0 with size {self.n_groups}")
            return self._bucket(grp, self.n_groups)
        return ops.single_segment(n, device)

    def _finish_last(self, out, l, glob):
        if not (self.sem.match_lookup and self.sem.remap_last):
            out[l].copy_(glob)
        elif self.has_penalty:
            bad = torch.nonzero(out[l] < 0)
            if bad.numel():
                # reference: mapping_result[prev_id][cur_id] KeyError (:1084)
                raise KeyError(int(glob[bad[0, 0]].item()))

    def _encode_fused(self, x, out, ws, count_rescored):
        n = x.shape[0]
        dev = x.device
        norm = self.sem.normalize_residual
        # level 0 is one segment over every centre: the local id IS the global id
        ops.assign(x, self.pcs[0], ops.single_segment(n, dev), self.cands[0], out_local=out[0], out_global=out[0],
                   workspace=ws)
        if count_rescored:
            self.last_rescored.append(ws.rescored())
        if self.L == 1:
            return
        n1 = torch.empty(n, dtype=torch.float32, device=dev) if norm else None
        glob1 = torch.empty(n, dtype=torch.int32, device=dev)
        b = self._bucket(out[0], self.need[0]) if self.L == 3 else self._last_level_buckets(out, 1, n, dev)
        fr1 = ops.FusedResidual(1, norm, self.pcs[0].centers, None, den_out=n1)
        ops.assign(x, self.pcs[1], b, self.cands[1], out_local=out[1], out_global=glob1, workspace=ws, fused=fr1)
        if count_rescored:
            self.last_rescored.append(ws.rescored())
        glob2 = torch.empty(n, dtype=torch.int32, device=dev)
        b = self._last_level_buckets(out, 2, n, dev)
        seg_ca, seg_cb = self._last_segment_rows(dev)
        fr2 = ops.FusedResidual(2, norm, self.pcs[0].centers, seg_ca, self.pcs[1].centers, seg_cb, den_in=n1)
        ops.assign(x, self.pcs[2], b, self.cands[2], out_local=out[2], out_global=glob2, workspace=ws, fused=fr2)
        if count_rescored:
            self.last_rescored.append(ws.rescored())
        self._finish_last(out, 2, glob2)

    def _last_segment_rows(self, dev):
        """Per-group residual centre rows of the last level: group g = l1*mult + l2 subtracts
        c0[l1] and c1[l1*need1 + l2] (training / raw id, :901) or c1[l2] (predict's modded id, :1143)."""
        key = (str(dev), self.sem.residual_global_id)
        if getattr(self, "_seg_rows_key", None) != key:
            mult, n1 = self._last_mult(), self.need[1]
            g = torch.arange(self.n_groups, dtype=torch.int64, device=dev)
            l1, l2 = g // mult, (g % mult).clamp(max=n1 - 1)
            seg_ca = l1.clamp(max=self.pcs[0].k - 1).to(torch.int32)
            cb = l1 * n1 + l2 if self.sem.residual_global_id else l2
            seg_cb = cb.clamp(max=self.pcs[1].k - 1).to(torch.int32)
            self._seg_rows, self._seg_rows_key = (seg_ca, seg_cb), key
        return self._seg_rows

    def _encode_materialized(self, x, out, ws, count_rescored):
        n = x.shape[0]
        cur = x
        glob = torch.empty(n, dtype=torch.int32, device=x.device)
        for l in range(self.L):
            w = self._weighted(cur, l)
            if l == 0:
                b = ops.single_segment(n, x.device)
                ops.assign(w, self.pcs[0], b, self.cands[0], out_local=out[0], out_global=glob, workspace=ws)
                out[0].copy_(glob)
            elif l < self.L - 1:
                b = self._bucket(out[l - 1], self.need[l - 1])
                ops.assign(w, self.pcs[l], b, self.cands[l], out_local=out[l], out_global=glob, workspace=ws)
            else:
                b = self._last_level_buckets(out, l, n, x.device)
                ops.assign(w, self.pcs[l], b, self.cands[l], out_local=out[l], out_global=glob, workspace=ws)
                self._finish_last(out, l, glob)
            if count_rescored:
                self.last_rescored.append(ws.rescored())
            if l < self.L - 1:
                src = w if self.sem.residual_from_weighted else cur
                cid = glob if self.sem.residual_global_id else out[l]
                cur = ops.residual(src, self.pcs[l].centers, cid, self.group_dims, self.sem.normalize_residual)
