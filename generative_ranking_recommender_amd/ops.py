"""Tensor-level wrappers over the C ABI (include/rqsid.h).

Every function takes/returns DEVICE tensors on the current HIP device and
enqueues on torch's current stream; nothing here synchronises with the host.
There is deliberately no CPU implementation: a CPU tensor or a missing
``librqsid.so`` raises.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass
from typing import Optional, Sequence

import torch

from . import _lib

_ALIGN = 256


def _ptr(t: Optional[torch.Tensor]):
    return None if t is None else t.data_ptr()


def _stream():
    return torch.cuda.current_stream().cuda_stream


def _require_device(*ts: Optional[torch.Tensor]) -> None:
    for t in ts:
        if t is not None and t.device.type != "cuda":
            raise RuntimeError("rqsid kernels run on the GPU only: got a %s tensor" % t.device.type)
        if t is not None and not t.is_contiguous():
            raise ValueError("rqsid kernels need contiguous tensors")


def lib():
    return _lib.load()


def tile_rows() -> int:
    return int(lib().rqsid_assign_tile_rows())


def centroid_tile_rows() -> int:
    return int(lib().rqsid_centroid_tile_rows())


kMaxList = 8  # candidates a screen can list per row (assign_common.h)
# the 1-term streamed screens gather centre pieces from a hi-only copy of the table (RQSID_HI_TABLE=0: from the
# interleaved table, for A/B); read once at import
HI_TABLE = __import__("os").environ.get("RQSID_HI_TABLE", "1") != "0"


@dataclass
class PreparedCenters:
    """Centres + the derived data rqsid_assign reads (fp16 copy and screening-bound norms)."""
    centers: torch.Tensor      # f32 [K, D]
    c16: torch.Tensor          # int16 [K, D/32, 2, 32]: per 32-dim chunk the hi then lo fp16 terms of c 2^s
    meta: torch.Tensor         # f32 [K+1, 4]: |c|^2, |c|, |2-term residual|, |1-term residual|; row K: 2^-s
    nearest_cand: Optional["Candidates"] = None  # nearest()'s candidate list (duplicates dropped), built once
    c16h: Optional[torch.Tensor] = None  # int16 [K, D]: the hi terms alone (the 1-term streamed screens' source)

    @property
    def k(self) -> int:
        return self.centers.shape[0]

    @property
    def sqnorm(self) -> torch.Tensor:
        return self.meta[:-1, 0]


def prepare_centers(c: torch.Tensor) -> PreparedCenters:
    c = c.float().contiguous()
    _require_device(c)
    k, d = c.shape
    c16 = torch.empty((k, d // 32, 2, 32), dtype=torch.int16, device=c.device)
    meta = torch.empty((k + 1, 4), dtype=torch.float32, device=c.device)
    _lib.check(lib().rqsid_prepare_centers(_ptr(c), k, d, _ptr(c16), _ptr(meta), _stream()),
               "rqsid_prepare_centers")
    c16h = None
    if HI_TABLE and k > 0:
        c16h = torch.empty((k, d), dtype=torch.int16, device=c.device)
        _lib.check(lib().rqsid_prepare_centers_hi(_ptr(c16), k, d, _ptr(c16h), _stream()), "rqsid_prepare_centers_hi")
    return PreparedCenters(c, c16, meta, c16h=c16h)


@dataclass
class Buckets:
    """Rows grouped by segment key (counting sort), as consumed by rqsid_assign."""
    seg_row_off: torch.Tensor   # i32 [S+1]
    seg_tile_off: torch.Tensor  # i32 [S+1]
    row_index: Optional[torch.Tensor]  # i32 [N] or None (identity)
    n_segments: int
    max_tiles: int
    workspace: Optional[torch.Tensor] = None  # rqsid_bucket's workspace (its sticky error word: error_word())

    def error_word(self) -> Optional[torch.Tensor]:
        """Device view of the workspace's sticky error word (include/rqsid.h rqsid_bucket), or None."""
        return None if self.workspace is None else bucket_error_word(self.workspace, self.n_segments)


def bucket_workspace(n_segments: int, device) -> torch.Tensor:
    """A reusable rqsid_bucket workspace with its sticky error word zeroed (the caller's duty)."""
    wsb = int(lib().rqsid_bucket_workspace_bytes(0, n_segments))
    ws = torch.empty(wsb, dtype=torch.uint8, device=device)
    bucket_error_word(ws, n_segments).zero_()
    return ws


def bucket_error_word(ws: torch.Tensor, n_segments: int) -> torch.Tensor:
    return ws[8 * n_segments:8 * n_segments + 4].view(torch.int32)


def single_segment(n: int, device, rows_per_tile: Optional[int] = None) -> Buckets:
    """All n rows in one segment, identity order (layer 0 / dense prediction)."""
    tr = rows_per_tile or tile_rows()
    # built by device fills, not host copies: the encode can be captured in a HIP graph
    off = torch.arange(2, dtype=torch.int32, device=device) * n
    toff = torch.arange(2, dtype=torch.int32, device=device) * ((n + tr - 1) // tr)
    return Buckets(off, toff, None, 1, (n + tr - 1) // tr)


def bucket(keys: torch.Tensor, n_segments: int, rows_per_tile: Optional[int] = None,
           workspace: Optional[torch.Tensor] = None) -> Buckets:
    """Counting sort of rows by key.  ``workspace``: a reusable ``bucket_workspace(n_segments)`` whose sticky
    error word accumulates over calls (default: a fresh one per call)."""
    keys = keys.to(torch.int32).contiguous()
    _require_device(keys)
    n = keys.numel()
    tr = rows_per_tile or tile_rows()
    off = torch.empty(n_segments + 1, dtype=torch.int32, device=keys.device)
    toff = torch.empty(n_segments + 1, dtype=torch.int32, device=keys.device)
    idx = torch.empty(max(n, 1), dtype=torch.int32, device=keys.device)
    wsb = int(lib().rqsid_bucket_workspace_bytes(n, n_segments))
    ws = workspace if workspace is not None and workspace.numel() >= wsb else bucket_workspace(n_segments, keys.device)
    _lib.check(lib().rqsid_bucket(_ptr(keys), n, n_segments, tr, _ptr(off), _ptr(toff), _ptr(idx), _ptr(ws), wsb,
                                  _stream()), "rqsid_bucket")
    return Buckets(off, toff, idx[:n], n_segments, (n + tr - 1) // tr + n_segments, ws)


@dataclass
class Candidates:
    """Per-segment allowed centres: global index of local j = idx[base[s]+j] (idx None: base[s]+j)."""
    base: torch.Tensor          # i32 [S]
    count: torch.Tensor         # i32 [S]
    count_max: int
    idx: Optional[torch.Tensor] = None   # i32
    flags: Optional[torch.Tensor] = None  # u8 [S]
    lid: Optional[torch.Tensor] = None   # i32: local id reported for list position (None: the position)


def contiguous_candidates(n_segments: int, per_segment: int, device) -> Candidates:
    base = torch.arange(n_segments, dtype=torch.int32, device=device) * per_segment
    cnt = torch.full((n_segments,), per_segment, dtype=torch.int32, device=device)
    return Candidates(base, cnt, per_segment)


def match_to_candidates(match: torch.Tensor) -> Candidates:
    """uint8 [groups, n_cand] match matrix -> ascending allowed-column lists (+ penalty flags)."""
    match = match.to(torch.uint8).contiguous()
    _require_device(match)
    g, nc = match.shape
    base = torch.empty(g, dtype=torch.int32, device=match.device)
    cnt = torch.empty(g, dtype=torch.int32, device=match.device)
    flags = torch.empty(g, dtype=torch.uint8, device=match.device)
    idx = torch.empty(g * nc, dtype=torch.int32, device=match.device)
    wsb = int(lib().rqsid_match_workspace_bytes(g))
    ws = torch.empty(wsb, dtype=torch.uint8, device=match.device)
    _lib.check(lib().rqsid_match_to_candidates(_ptr(match), g, nc, _ptr(base), _ptr(cnt), _ptr(idx), _ptr(flags),
                                               _ptr(ws), wsb, _stream()), "rqsid_match_to_candidates")
    # the maximum allowed count decides the kernel variant; match rows are host-known data
    cmax = int(match.sum(1).max().item()) if g else 0
    return Candidates(base, cnt, cmax, idx, flags)


def dedup_candidates(cand: Candidates, centers: torch.Tensor) -> Candidates:
    """Drop every list entry whose centre is bitwise identical to an EARLIER entry of the same list.

    Exact: identical centres have identical distances, and the reference's argmin returns the first
    of equal minima, so a later duplicate can never be the answer.  The kept entries report their
    original local ids through ``lid``.  Without duplicates the input is returned unchanged."""
    dev = centers.device
    canon = torch.unique(centers.float().contiguous().view(torch.int32), dim=0, return_inverse=True)[1]
    n_unique = int(canon.max().item()) + 1 if centers.shape[0] else 0
    if n_unique == centers.shape[0]:
        return cand  # no duplicate rows at all
    S = cand.base.numel()
    cnt = cand.count.long()
    total = int(cnt.sum().item())
    seg = torch.repeat_interleave(torch.arange(S, device=dev), cnt)
    off = torch.zeros(S + 1, dtype=torch.long, device=dev)
    off[1:] = torch.cumsum(cnt, 0)
    pos = torch.arange(total, device=dev) - off[seg]
    if cand.idx is None:
        glob = cand.base.long()[seg] + pos
    else:
        glob = cand.idx.long()[cand.base.long()[seg] + pos]
    lid_in = pos if cand.lid is None else cand.lid.long()[cand.base.long()[seg] + pos]
    key = seg * n_unique + canon[glob]
    first = torch.full((int(key.max().item()) + 1,), total, dtype=torch.long, device=dev)
    first.scatter_reduce_(0, key, pos + off[seg], reduce="amin")
    keep = first[key] == pos + off[seg]
    new_cnt = torch.zeros(S, dtype=torch.long, device=dev).index_add_(0, seg, keep.long())
    new_base = torch.zeros(S, dtype=torch.long, device=dev)
    new_base[1:] = torch.cumsum(new_cnt, 0)[:-1]
    return Candidates(new_base.to(torch.int32), new_cnt.to(torch.int32), int(new_cnt.max().item()) if S else 0,
                      glob[keep].to(torch.int32).contiguous(), cand.flags, lid_in[keep].to(torch.int32).contiguous())


class AssignWorkspace:
    """Re-usable scratch for rqsid_assign (rows needing an fp64 re-score)."""

    def __init__(self, n_rows: int, device):
        self.bytes = int(lib().rqsid_assign_workspace_bytes(n_rows))
        self.buf = torch.empty(self.bytes, dtype=torch.uint8, device=device)
        self.buf[240:256].zero_()  # the sticky error word (include/rqsid.h)
        self.n_rows = n_rows

    def rescored(self) -> int:
        """Rows re-scored in fp64 by the last assign (host sync)."""
        return int(self.buf[:4].view(torch.int32).item())

    def error(self) -> int:
        """Sticky error word of every assign on this workspace (host sync; csrc/assign_common.h kErrSlot):
        bit 0 compaction past n_rows, bit 1 overflow list past n_rows, bit 2 a list entry outside work[],
        bit 3 a tile count past the tile maps / descriptors (clamped). Every such write or count is bounded by
        its slot's capacity; a non-zero word means one was dropped."""
        return int(self.error_word().item())

    def error_word(self) -> torch.Tensor:
        return self.buf[240:244].view(torch.int32)


def check_error_words(words, what: str) -> None:
    """One host sync over device error words (AssignWorkspace / Buckets); raise if any is non-zero: a
    counter-driven write was dropped, so the IDs of that call are not trustworthy."""
    ws = [w for w in words if w is not None]
    if not ws:
        return
    vals = torch.cat(ws).cpu().tolist()
    if any(vals):
        raise RuntimeError(f"{what}: a device error word is set ({vals}): a counter-driven list write fell outside "
                           "its slot and was dropped (csrc/assign_common.h kErrSlot, rqsid_bucket)")


@dataclass
class FusedResidual:
    """On-the-fly residual chain for rqsid_assign (res_levels 1 or 2, one dimension group).
    The subtracted centres are per SEGMENT s (the segment of a level determines its parents):

    levels=1: v = x - ca[seg_ca[s]]            (normalize: / (||v|| + 1e-8), written to den_out)
    levels=2: v = (x - ca[seg_ca[s]])[/den_in] - cb[seg_cb[s]]   (normalize: / (||v|| + 1e-8))
    seg_ca None = identity (segment s subtracts ca[s])."""
    levels: int
    normalize: bool
    ca: torch.Tensor
    seg_ca: Optional[torch.Tensor] = None
    cb: Optional[torch.Tensor] = None
    seg_cb: Optional[torch.Tensor] = None
    den_in: Optional[torch.Tensor] = None
    den_out: Optional[torch.Tensor] = None


def assign(x: torch.Tensor, pc: PreparedCenters, buckets: Buckets, cand: Candidates,
           out_local: Optional[torch.Tensor] = None, out_global: Optional[torch.Tensor] = None,
           workspace: Optional[AssignWorkspace] = None, fused: Optional[FusedResidual] = None,
           screen_terms: int = 0):
    """Exact segmented argmin. Returns (local i32[N], global i32[N]).  ``screen_terms`` (0 auto, 1, 3)
    only changes how much work the exact answer takes."""
    _require_device(x, pc.centers, cand.base, cand.count, cand.idx, cand.flags)
    n, d = x.shape
    if d != pc.centers.shape[1]:
        raise ValueError(f"dimension mismatch: x has {d}, centres {pc.centers.shape[1]}")
    dev = x.device
    if out_local is None:
        out_local = torch.empty(n, dtype=torch.int32, device=dev)
    if out_global is None:
        out_global = torch.empty(n, dtype=torch.int32, device=dev)
    if workspace is None or workspace.n_rows < n:
        workspace = AssignWorkspace(n, dev)
    f = fused
    if f is not None:
        _require_device(f.ca, f.seg_ca, f.cb, f.seg_cb, f.den_in, f.den_out)
    _lib.check(lib().rqsid_assign(
        _ptr(x), n, d, _ptr(buckets.row_index), buckets.n_segments, _ptr(buckets.seg_row_off),
        _ptr(buckets.seg_tile_off), buckets.max_tiles,
        _ptr(pc.centers), _ptr(pc.c16), _ptr(pc.c16h), _ptr(pc.meta), pc.k,
        _ptr(cand.base), _ptr(cand.count), cand.count_max, _ptr(cand.idx), _ptr(cand.lid), _ptr(cand.flags),
        0 if f is None else f.levels, 0 if f is None else int(f.normalize),
        None if f is None else _ptr(f.ca), None if f is None else _ptr(f.seg_ca),
        None if f is None else _ptr(f.cb), None if f is None else _ptr(f.seg_cb),
        None if f is None else _ptr(f.den_in), None if f is None else _ptr(f.den_out),
        _ptr(out_local), _ptr(out_global), int(screen_terms), _ptr(workspace.buf), workspace.bytes, _stream()),
        "rqsid_assign")
    return out_local, out_global


def nearest(x: torch.Tensor, pc: PreparedCenters, workspace: Optional[AssignWorkspace] = None,
            screen_terms: int = 0) -> torch.Tensor:
    """Unconstrained nearest centre (KMeans.predict / pairwise_distance_full + argmin)."""
    n = x.shape[0]
    b = single_segment(n, x.device)
    if pc.nearest_cand is None:
        cand = Candidates(torch.zeros(1, dtype=torch.int32, device=x.device),
                          torch.full((1,), pc.k, dtype=torch.int32, device=x.device), pc.k)
        # bitwise-duplicate centres (e.g. several K-Means centres initialised from equal rows): only the
        # first copy can be the argmin, and with the copies in the list every row nearest to them is an
        # exact > 8-way tie that no screen can split, i.e. an all-candidate fp64 re-score
        pc.nearest_cand = dedup_candidates(cand, pc.centers) if pc.k > kMaxList else cand
    return assign(x, pc, b, pc.nearest_cand, workspace=workspace, screen_terms=screen_terms)[1]


def _groups_tensor(group_dims: Sequence[int], device) -> torch.Tensor:
    return torch.tensor(list(group_dims), dtype=torch.int32, device=device)


def residual(x: torch.Tensor, centers: torch.Tensor, ids: torch.Tensor, group_dims: Sequence[int] = (),
             normalize: bool = True, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    ids = ids.to(torch.int32).contiguous()
    centers = centers.float().contiguous()
    _require_device(x, centers, ids)
    n, d = x.shape
    if out is None:
        out = torch.empty_like(x)
    gd = list(group_dims) or [d]
    g = _groups_tensor(gd, x.device)
    _lib.check(lib().rqsid_residual(_ptr(x), n, d, _ptr(centers), centers.shape[0], _ptr(ids), _ptr(g), len(gd), int(normalize),
                                    _ptr(out), _stream()), "rqsid_residual")
    return out


def scale_groups(x: torch.Tensor, group_dims: Sequence[int], weights: Sequence[float]) -> torch.Tensor:
    _require_device(x)
    n, d = x.shape
    out = torch.empty_like(x)
    g = _groups_tensor(group_dims, x.device)
    w = torch.tensor(list(weights), dtype=torch.float32, device=x.device)
    _lib.check(lib().rqsid_scale_groups(_ptr(x), n, d, _ptr(g), len(group_dims), _ptr(w), _ptr(out), _stream()),
               "rqsid_scale_groups")
    return out


def centroid_update(x: torch.Tensor, assignment: torch.Tensor, k: int, centers: torch.Tensor):
    """New centres = per-cluster means of x (fp64 sums) written into ``centers`` where the
    cluster is non-empty.  Returns (centers, counts i32[k])."""
    _require_device(x, centers)
    n, d = x.shape
    b = bucket(assignment, k, rows_per_tile=centroid_tile_rows())
    sums = torch.zeros((k, d), dtype=torch.float64, device=x.device)
    _lib.check(lib().rqsid_centroid_accumulate(_ptr(x), d, _ptr(b.row_index), k, _ptr(b.seg_row_off),
                                               _ptr(b.seg_tile_off), b.max_tiles, _ptr(sums), _stream()),
               "rqsid_centroid_accumulate")
    _lib.check(lib().rqsid_centroid_finalize(_ptr(sums), _ptr(b.seg_row_off), k, d, _ptr(centers), _stream()),
               "rqsid_centroid_finalize")
    counts = b.seg_row_off[1:] - b.seg_row_off[:-1]
    return centers, counts


def pairwise_distance(x: torch.Tensor, c: torch.Tensor) -> torch.Tensor:
    c = c.float().contiguous()
    _require_device(x, c)
    n, d = x.shape
    out = torch.empty((n, c.shape[0]), dtype=torch.float32, device=x.device)
    _lib.check(lib().rqsid_pairwise_distance(_ptr(x), n, d, _ptr(c), c.shape[0], _ptr(out), _stream()),
               "rqsid_pairwise_distance")
    return out


def pairwise_cosine(x: torch.Tensor, c: torch.Tensor, scores: bool = False) -> torch.Tensor:
    """Cosine distances 1 - x.c / (|x||c|): fp32 [N, K], or with ``scores`` the auction's worker-major fp16
    [K][N] = -distance (include/rqsid.h rqsid_pairwise_cosine)."""
    c = c.float().contiguous()
    _require_device(x, c)
    n, d = x.shape
    if scores:
        out = torch.empty((c.shape[0], n), dtype=torch.float16, device=x.device)
        _lib.check(lib().rqsid_pairwise_cosine(_ptr(x), n, d, _ptr(c), c.shape[0], None, _ptr(out), _stream()),
                   "rqsid_pairwise_cosine")
        return out
    out = torch.empty((n, c.shape[0]), dtype=torch.float32, device=x.device)
    _lib.check(lib().rqsid_pairwise_cosine(_ptr(x), n, d, _ptr(c), c.shape[0], _ptr(out), None, _stream()),
               "rqsid_pairwise_cosine")
    return out


def auction_scores(x: torch.Tensor, c: torch.Tensor, half: bool = False) -> torch.Tensor:
    """Worker-major fp16 scores W[k][n] = -distance (the auction's input), see include/rqsid.h."""
    c = c.float().contiguous()
    _require_device(x, c)
    n, d = x.shape
    out = torch.empty((c.shape[0], n), dtype=torch.float16, device=x.device)
    _lib.check(lib().rqsid_auction_scores(_ptr(x), n, d, _ptr(c), c.shape[0], int(half), _ptr(out), _stream()),
               "rqsid_auction_scores")
    return out


def auction(scores_wj: torch.Tensor, max_rounds: int = 0):
    """Balanced assignment on worker-major fp16 scores [K][N]. Returns (assignment i32[N], rounds)."""
    scores_wj = scores_wj.to(torch.float16).contiguous()
    _require_device(scores_wj)
    k, n = scores_wj.shape
    out = torch.empty(n, dtype=torch.int32, device=scores_wj.device)
    wsb = int(lib().rqsid_auction_workspace_bytes(n, k))
    ws = torch.empty(max(wsb, 1), dtype=torch.uint8, device=scores_wj.device)
    rounds = ctypes.c_int32(0)
    _lib.check(lib().rqsid_auction_lap_half(_ptr(scores_wj), k, n, int(max_rounds), _ptr(out), ctypes.addressof(rounds),
                                            _ptr(ws), wsb, _stream()), "rqsid_auction_lap_half")
    return out, int(rounds.value)


def auction_full(scores_wj: torch.Tensor, max_rounds: int = 0):
    """fp32 balanced assignment on worker-major scores [K][N] (include/rqsid.h rqsid_auction_lap_full).
    Returns (assignment i32[N], rounds)."""
    scores_wj = scores_wj.to(torch.float32).contiguous()
    _require_device(scores_wj)
    k, n = scores_wj.shape
    out = torch.empty(n, dtype=torch.int32, device=scores_wj.device)
    if n == 0:
        return out, 0
    wsb = int(lib().rqsid_auction_full_workspace_bytes(n, k))
    ws = torch.empty(max(wsb, 1), dtype=torch.uint8, device=scores_wj.device)
    rounds = ctypes.c_int32(0)
    _lib.check(lib().rqsid_auction_lap_full(_ptr(scores_wj), k, n, int(max_rounds), _ptr(out), ctypes.addressof(rounds),
                                            _ptr(ws), wsb, _stream()), "rqsid_auction_lap_full")
    return out, int(rounds.value)


def greedy_match(dist: torch.Tensor, sub_off: torch.Tensor, max_take: int):
    """Greedy unique-nearest columns per group (see include/rqsid.h rqsid_greedy_match).
    dist: f32 [total_sub, C]; sub_off: i32 [G+1].  Returns (match u8 [G, C], n_selected i32 [G])."""
    dist = dist.float().contiguous()
    sub_off = sub_off.to(torch.int32).contiguous()
    _require_device(dist, sub_off)
    g = sub_off.numel() - 1
    c = dist.shape[1]
    match = torch.empty((g, c), dtype=torch.uint8, device=dist.device)
    nsel = torch.empty(max(g, 1), dtype=torch.int32, device=dist.device)
    _lib.check(lib().rqsid_greedy_match(_ptr(dist), _ptr(sub_off), g, c, int(max_take), _ptr(match), _ptr(nsel),
                                        _stream()), "rqsid_greedy_match")
    return match, nsel[:g]


def centroid_sums(x: torch.Tensor, assignment: torch.Tensor, k: int):
    """Per-cluster fp64 sums and counts of the rows of x (the first half of the Lloyd update; the
    multi-GPU fit all-reduces these).  Returns (sums f64 [k, D], counts i32 [k])."""
    _require_device(x)
    n, d = x.shape
    b = bucket(assignment, k, rows_per_tile=centroid_tile_rows())
    sums = torch.zeros((k, d), dtype=torch.float64, device=x.device)
    _lib.check(lib().rqsid_centroid_accumulate(_ptr(x), d, _ptr(b.row_index), k, _ptr(b.seg_row_off),
                                               _ptr(b.seg_tile_off), b.max_tiles, _ptr(sums), _stream()),
               "rqsid_centroid_accumulate")
    return sums, b.seg_row_off[1:] - b.seg_row_off[:-1]


class SegmentLayout:
    """Rows grouped by segment (segment s = rows off[s] .. off[s+1] of a segment-ordered matrix), with the
    tile and chunk tables of the segmented auction kernels (include/rqsid.h rqsid_seg_auction_*)."""

    def __init__(self, sizes, device):
        import numpy as np
        sizes = np.asarray(sizes, dtype=np.int64)
        if sizes.ndim != 1 or len(sizes) == 0 or (sizes < 0).any():
            raise ValueError("segment sizes must be a non-empty 1-D array of counts")
        self.sizes = sizes
        self.n_seg = len(sizes)
        off = np.zeros(self.n_seg + 1, dtype=np.int64)
        off[1:] = np.cumsum(sizes)
        if off[-1] > 2**31 - 1:
            raise ValueError("segmented auction: more than 2^31 - 1 rows")
        self.off = off
        self.n = int(off[-1])
        tiles = (sizes + 63) // 64
        ch = int(lib().rqsid_seg_auction_chunk_jobs())
        chunks = (sizes + ch - 1) // ch
        toff = np.concatenate([[0], np.cumsum(tiles)])
        coff = np.concatenate([[0], np.cumsum(chunks)])
        self.n_tiles = int(toff[-1])
        self.total_chunks = int(coff[-1])
        self.n_multi = int((chunks > 1).sum())
        self.seg_off = torch.as_tensor(off, dtype=torch.int32).to(device)
        self.tile_off = torch.as_tensor(toff, dtype=torch.int32).to(device)
        self.chunk_off = torch.as_tensor(coff, dtype=torch.int32).to(device)
        self.seg_of_row = torch.repeat_interleave(torch.arange(self.n_seg, device=device),
                                                  torch.as_tensor(sizes).to(device))


def seg_auction_scores(x: torch.Tensor, centers: torch.Tensor, k: int, layout: SegmentLayout,
                       half: bool = False) -> torch.Tensor:
    """Per-segment worker-major fp16 scores -distance (segment s: rows of layout, centres s*k..s*k+k-1),
    concatenated: a flat fp16 tensor of k * N values."""
    centers = centers.float().contiguous()
    _require_device(x, centers)
    n, d = x.shape
    if n != layout.n or centers.shape[0] != layout.n_seg * k or centers.shape[1] != d:
        raise ValueError("seg_auction_scores: rows / centres do not match the segment layout")
    out = torch.empty(max(k * n, 1), dtype=torch.float16, device=x.device)
    _lib.check(lib().rqsid_seg_auction_scores(_ptr(x), n, d, _ptr(centers), k, layout.n_seg, _ptr(layout.seg_off),
                                              _ptr(layout.tile_off), layout.n_tiles, int(half), _ptr(out), _stream()),
               "rqsid_seg_auction_scores")
    return out


def seg_auction(scores: torch.Tensor, k: int, layout: SegmentLayout, active: Optional[torch.Tensor] = None,
                max_rounds: int = 0, out: Optional[torch.Tensor] = None):
    """One balanced auction per segment, all advanced in lockstep.  Returns (assignment i32 [N] local to
    each segment, rounds i32 [S] on the device).  Segments with active[s] == 0 keep ``out``'s entries."""
    scores = scores.to(torch.float16).contiguous()
    _require_device(scores, active)
    n = layout.n
    if out is None:
        out = torch.full((max(n, 1),), -1, dtype=torch.int32, device=scores.device)
    rounds = torch.zeros(layout.n_seg, dtype=torch.int32, device=scores.device)
    wsb = int(lib().rqsid_seg_auction_workspace_bytes(n, k, layout.n_seg, layout.total_chunks, layout.n_multi))
    ws = torch.empty(max(wsb, 1), dtype=torch.uint8, device=scores.device)
    act = None if active is None else active.to(torch.uint8).contiguous()
    _lib.check(lib().rqsid_seg_auction_lap_half(_ptr(scores), k, layout.n_seg, _ptr(layout.seg_off),
                                                _ptr(layout.chunk_off), layout.total_chunks, layout.n_multi, n,
                                                _ptr(act), int(max_rounds), _ptr(out), _ptr(rounds), _ptr(ws), wsb,
                                                _stream()), "rqsid_seg_auction_lap_half")
    return out[:n], rounds
