/*
 * rqsid.h — C ABI of the MI355X (gfx950) residual-quantisation semantic-ID kernels.
 *
 * The reference (zeehu/generative_ranking_recommender) has no FFI: its hot path
 * is the Python module API of balancekmeans / hierarchical_rq_kmeans /
 * simplified_semantic_id_generator, whose arithmetic is stock PyTorch ops.
 * Each entry point below replaces one of those op sequences; the reference
 * file:line it stands in for is cited per function.  The Python mirror of the
 * reference classes (generative_ranking_recommender_amd/) binds these with
 * ctypes; INTEGRATION.md shows the binding.
 *
 * Conventions
 *  - every pointer is a DEVICE pointer owned by the caller (e.g. torch
 *    tensor.data_ptr()); nothing is allocated inside except what the caller
 *    passes as `workspace` (size from the matching *_workspace_bytes query);
 *  - all work is stream-ordered on the caller's hipStream_t (passed as void*),
 *    no host synchronisation, graph-capturable;
 *  - return 0 on success, a negative RQSID_E* code otherwise; the text of the
 *    last error of the calling thread is in rqsid_last_error();
 *  - matrices are row-major fp32 [rows][dim]; dim must be a multiple of 32.
 */
#ifndef RQSID_H
#define RQSID_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RQSID_OK 0
#define RQSID_E_ARG (-1)      /* bad argument (shape, null pointer, unsupported dim) */
#define RQSID_E_LAUNCH (-2)   /* HIP launch / runtime error */
#define RQSID_E_WORKSPACE (-3)

/* segment flags (rqsid_assign seg_flags[s]) */
#define RQSID_SEG_PENALTY 1u  /* empty allowed set: argmin over ALL centres of fl(d + 10000) */

int rqsid_version(void);
const char* rqsid_last_error(void);
/* 0 for a product build; else the bits of the timing-probe macros it was compiled with (tools/ab_build.sh:
 * 1 RQSID_AB_MODE, 2 RQSID_AB_HALFROW, 4 RQSID_AB_NOROWDMA, 8 RQSID_AB_EPI, 16 RQSID_STAMPS,
 * 32 RQSID_AB_NO_FLUSH) -- such a library returns wrong IDs by design and must never ship. */
int32_t rqsid_build_flags(void);

/* Centre preparation for rqsid_assign.  The table is scaled by a power of two 2^s (largest element
 * just below 2^14) and split into two fp16 terms: hi = fp16(c 2^s) and lo = fp16((c 2^s - hi) 2^12),
 * scaled values outside the fp16 normal range stored as 0 (the MFMA must never see a subnormal).
 * c16 [k][dim/32][2][32] (IEEE half bits: per centre and 32-dim chunk, 32 hi terms then 32 lo terms,
 * one 128-B piece); c_meta [k+1][4]: row j <  k =
 * {|c|^2, |c|, |c - (hi + lo 2^-12) 2^-s|, |c - hi 2^-s|} (fp64-accumulated, feeding the screening
 * error bound), row k = {2^-s, max_j |c - (hi + lo 2^-12) 2^-s| / |c|, max_j |c - hi 2^-s| / |c|,
 * max_j |c|} (rounded up; the single-pass screens collapse their per-candidate bound onto |c|).  Replaces the per-call centre side of torch.cdist's
 * mm-expansion (ATen _euclidean_dist) used by pairwise_distance_full,
 * balancekmeans/__init__.py:576-603. */
int rqsid_prepare_centers(const float* centers, int64_t k, int32_t dim,
                          uint16_t* c16, float* c_meta, void* stream);
/* The hi terms of a prepared table alone, c16_hi [k][dim] fp16 (1 KiB per 512-d centre): the 1-term streamed
 * screens (the ping-pong and row-resident forms) gather their 64-B centre pieces from it when rqsid_assign
 * gets it, touching half the cache lines of the interleaved table (the XL last level's 5120 candidates: 5 MB
 * instead of 10 MB against a 4-MB XCD L2). */
int rqsid_prepare_centers_hi(const uint16_t* c16, int64_t k, int32_t dim, uint16_t* c16_hi, void* stream);

/* Counting sort of rows by segment key (keys in [0, n_segments)).
 * Outputs seg_row_off[S+1], seg_tile_off[S+1] (exclusive scan of
 * ceil(rows_in_segment / tile_rows)), row_index[n] (rows grouped by key).
 * Replaces the per-parent torch.where/mask loops of
 * hierarchical_rq_kmeans.py:711,880-885,1210-1216 and
 * simplified_semantic_id_generator.py:112,154-158,263.
 * Workspace int 2*n_segments (the first int after counts and cursors) is a sticky error word the
 * caller zeroes when it allocates the workspace (a call never clears it): every row_index write takes
 * its position from a device counter, and a position outside its key's segment drops the write and
 * sets bit 1 there (a wrong count can only report an error, never store outside row_index). */
int64_t rqsid_bucket_workspace_bytes(int64_t n, int32_t n_segments);
int rqsid_bucket(const int32_t* keys, int64_t n, int32_t n_segments, int32_t tile_rows,
                 int32_t* seg_row_off, int32_t* seg_tile_off, int32_t* row_index,
                 void* workspace, int64_t workspace_bytes, void* stream);

/* Rows per work tile of rqsid_assign (the tile_rows to pass to rqsid_bucket). */
int32_t rqsid_assign_tile_rows(void);

/* Segmented nearest-centre assignment (exact argmin, lowest index on ties).
 *
 * Segment s owns rows row_index[seg_row_off[s] .. seg_row_off[s+1]) (row_index
 * NULL = identity) and candidates j = 0 .. cand_count[s]-1 whose global centre
 * index is cand_idx[cand_base[s]+j] (cand_idx NULL: cand_base[s]+j).
 * out_local[row] = cand_lid[cand_base[s]+j] (cand_lid NULL: j) of the nearest allowed
 * centre, out_global[row] = its global index.  (A list may omit bitwise duplicates of an
 * earlier entry -- they can never be the first minimum -- and report the original local
 * ids through cand_lid.)  Segments flagged RQSID_SEG_PENALTY reproduce the reference's +10000
 * mask with an empty allowed set (argmin over all n_centers of fl32(d)+10000);
 * their out_local is -1.
 *
 * Replaces pairwise_distance_full + torch.argmin (balancekmeans/__init__.py:
 * 489-534, 576-603), the +10000-masked reassignment/prediction of
 * hierarchical_rq_kmeans.py:839-966,1146-1305 and the +inf-masked ones of
 * simplified_semantic_id_generator.py:145-161,305-331.
 *
 * Fused residuals (res_levels 1/2, one dimension group): the vector assigned for row i of
 * segment s is
 *   0: x_i
 *   1: u = x_i - ca[seg_ca[s]]             [ / (||u|| + 1e-8), written to den_out[i] ]
 *   2: v = (x_i - ca[seg_ca[s]])[/den_in[i]] - cb[seg_cb[s]]   [ / (||v|| + 1e-8) ]
 * (seg_ca NULL = identity), exactly the fp32 operation sequence of
 * _compute_residuals_with_centers (hierarchical_rq_kmeans.py:1088-1128, res_normalize=1) or of
 * the simplified generator's plain residuals (:91,167, res_normalize=0), without materialising
 * the residual matrix.  The residual centres are per SEGMENT: a level's segment (parent cluster,
 * (l1,l2) group) determines the parent IDs whose centres are subtracted.
 *
 * Method: fp16 MFMA screening (v_mfma_f32_32x32x16_f16) with a rigorous per-candidate error
 * bound, then an fp64 re-score of every row whose bound admits more than one candidate.
 * screen_terms: 1 = vh.ch only; 3 = vh.ch + vl.ch + vh.cl (both operands' fp16 rounding
 * residuals, a ~5x tighter bound for 3x the MFMA work; segments of <= 128 candidates only, wider
 * ones use 1); 0 = automatic (3 for residual levels with <= 128 candidates per segment).  The result
 * never depends on it, only the speed.
 *
 * Errors: RQSID_E_ARG / RQSID_E_WORKSPACE before any launch; RQSID_E_LAUNCH for a HIP launch failure
 * or, on the opt-in centre-resident screen (RQSID_SCREEN_VARIANT=6), when a wave's capped role wait
 * gave up (device error word read back after the call; the IDs it left are not returned as valid).
 * c16_hi: NULL or rqsid_prepare_centers_hi's table of the same centres (only where-from changes, never the IDs).
 * Workspace bytes [240, 244) are a sticky error word the caller zeroes when it allocates the workspace
 * (every call zeroes only [0, 240)): each list write whose index comes from a device counter (the
 * re-score compaction, the overflow list) is bounded by its slot's capacity, and a write that would fall
 * outside sets a bit here instead (1 compaction, 2 overflow list, 4 a list entry outside [0, n_rows),
 * 8 a device tile count past the tile maps / descriptors of the streamed, producer/consumer, row- and
 * centre-resident screens: clamped to their capacity). */
int64_t rqsid_assign_workspace_bytes(int64_t n_rows);
int rqsid_assign(const float* x, int64_t n_rows, int32_t dim, const int32_t* row_index,
                 int32_t n_segments, const int32_t* seg_row_off, const int32_t* seg_tile_off,
                 int64_t max_tiles,
                 const float* centers, const uint16_t* c16, const uint16_t* c16_hi, const float* c_meta,
                 int32_t n_centers,
                 const int32_t* cand_base, const int32_t* cand_count, int32_t cand_count_max,
                 const int32_t* cand_idx, const int32_t* cand_lid, const uint8_t* seg_flags,
                 int32_t res_levels, int32_t res_normalize,
                 const float* ca, const int32_t* seg_ca, const float* cb, const int32_t* seg_cb,
                 const float* den_in, float* den_out,
                 int32_t* out_local, int32_t* out_global, int32_t screen_terms,
                 void* workspace, int64_t workspace_bytes, void* stream);

/* Residual r = x - c[center_id[row]]; with normalize != 0 each dimension group
 * g is divided by (||r_g|| + 1e-8).  Replaces _compute_residuals_with_centers
 * (hierarchical_rq_kmeans.py:1088-1128) and the plain residuals of
 * simplified_semantic_id_generator.py:78-96,164-168. */
int rqsid_residual(const float* x, int64_t n, int32_t dim, const float* centers, int32_t n_centers,
                   const int32_t* center_id, const int32_t* group_dims, int32_t n_groups,
                   int32_t normalize, float* out, void* stream);

/* y = x * w_g per dimension group (hierarchical_rq_kmeans.py:583-604). */
int rqsid_scale_groups(const float* x, int64_t n, int32_t dim, const int32_t* group_dims,
                       int32_t n_groups, const float* weights, float* out, void* stream);

/* Lloyd centroid update, first half: per-cluster fp64 sums over the rows of
 * each segment (bucketed by rqsid_bucket with rqsid_centroid_tile_rows()).
 * sums must be zeroed by the caller.  Replaces the per-cluster
 * nonzero/index_select/mean loop of balancekmeans/__init__.py:315-324,434-443. */
int32_t rqsid_centroid_tile_rows(void);
int rqsid_centroid_accumulate(const float* x, int32_t dim, const int32_t* row_index,
                              int32_t n_segments, const int32_t* seg_row_off,
                              const int32_t* seg_tile_off, int64_t max_tiles,
                              double* sums, void* stream);
/* Second half: centers[k] = fp32(sums[k] / count[k]) for count[k] > 0 (others
 * untouched; the caller fills empty clusters exactly as the reference does). */
int rqsid_centroid_finalize(const double* sums, const int32_t* seg_row_off, int32_t k,
                            int32_t dim, float* centers, void* stream);

/* Match matrix (uint8 [groups][n_cand], 1 = allowed) to candidate lists:
 * cand_count[g] = row popcount, cand_base[g] = exclusive scan, cand_idx = allowed
 * columns in ascending order (so the local index IS the remapped id of
 * _merge_match_matrix_cluster_ids, hierarchical_rq_kmeans.py:1055-1086),
 * seg_flags[g] = RQSID_SEG_PENALTY for empty rows. cand_idx needs
 * groups*n_cand entries of room. */
int64_t rqsid_match_workspace_bytes(int32_t groups);
int rqsid_match_to_candidates(const uint8_t* match, int32_t groups, int32_t n_cand,
                              int32_t* cand_base, int32_t* cand_count, int32_t* cand_idx,
                              uint8_t* seg_flags, void* workspace, int64_t workspace_bytes,
                              void* stream);

/* Dense distance matrix out[n][k] = sqrt(max(|x|^2 + |c|^2 - 2 x.c, 0)) in fp32
 * (torch.cdist semantics, pairwise_distance_full balancekmeans/__init__.py:576-603),
 * feeding the balanced auction. */
int rqsid_pairwise_distance(const float* x, int64_t n, int32_t dim, const float* centers,
                            int32_t k, float* out, void* stream);

/* Cosine distances 1 - x.c / (|x| |c|) of pairwise_cosine (balancekmeans/__init__.py:625-655, the
 * distance='cosine' option of KMeans.fit / fit_by_min_loss / predict, :279-280, 511-512): fp32 [n][k] into
 * `out` and / or the auction's worker-major fp16 scores -distance [k][n] into `out_wj` (either may be NULL).
 * fp32 sums in the kernel's order (the reference normalises the operands first, then multiplies: the
 * results agree to a few fp32 ulps of 1). */
int rqsid_pairwise_cosine(const float* x, int64_t n, int32_t dim, const float* centers, int32_t k, float* out,
                          uint16_t* out_wj, void* stream);

/* Auction score matrix: out_wj[k][n] = fp16(-||x_i - c_j||) (fp32 distances, half = 0) or
 * -max(fp16 distance of the fp16-rounded operands, 1e-5) (half != 0), worker-major: the input of
 * auction_lap_half(-pairwise_distance_{full,half}(X, C)), balancekmeans/__init__.py:29-43,
 * 536-603. */
int rqsid_auction_scores(const float* x, int64_t n, int32_t dim, const float* centers, int32_t k,
                         int32_t half, uint16_t* out_wj, void* stream);

/* Balanced assignment: the auction of balancekmeans.auction_lap_half (balancekmeans/__init__.py:
 * 12-140, return_token_to_worker=True) on the fp16 score matrix scores_wj[K][N] (worker-major,
 * IEEE half bits).  out_assign[j] = worker of job j.  Every fp16 operation of the reference is
 * reproduced with one rounding; ties at the top-k boundary keep the lowest job index and equal
 * highest bids go to the lowest worker (the reference leaves both to torch).  N < K reproduces
 * the reference's argmin(-D) fallback.  Blocks the calling thread (one host read per round);
 * *out_rounds = rounds run.  max_rounds <= 0: unbounded (the reference's leftover rule ends every
 * auction by round 1002). */
int64_t rqsid_auction_workspace_bytes(int64_t n_jobs, int32_t n_workers);
int rqsid_auction_lap_half(const uint16_t* scores_wj, int32_t n_workers, int64_t n_jobs,
                           int32_t max_rounds, int32_t* out_assign, int32_t* out_rounds,
                           void* workspace, int64_t workspace_bytes, void* stream);

/* The fp32 auction of balancekmeans.auction_lap_full (balancekmeans/__init__.py:142-210), reached only
 * through KMeans.predict(balanced=True) (:523-525), on fp32 scores scores_wj[K][N] (worker-major).
 * Every fp32 operation of the reference with one rounding; the same tie rules as rqsid_auction_lap_half.
 * Unlike auction_lap_half it has no N < K fallback: with jobs_per_worker = 0 nothing bids until the
 * leftover rule gives every job to worker 0 after round 1000.  Blocks the calling thread (one host read
 * per round); *out_rounds = rounds run.  N >= 1, 2 <= K <= 65535. */
int64_t rqsid_auction_full_workspace_bytes(int64_t n_jobs, int32_t n_workers);
int rqsid_auction_lap_full(const float* scores_wj, int32_t n_workers, int64_t n_jobs, int32_t max_rounds,
                           int32_t* out_assign, int32_t* out_rounds, void* workspace, int64_t workspace_bytes,
                           void* stream);

/* Segmented auction scores for many independent balanced fits at once (the per-parent sub-K-Means of
 * hierarchical_rq_kmeans.py:671-752 and the per-group sub-K-Means of :968-1053, which the reference runs
 * one after another, each through balancekmeans/__init__.py:29-43,536-603).  Segment s owns rows
 * seg_off[s] .. seg_off[s+1] of x (rows grouped by segment) and centres s*k .. s*k+k-1; its scores go to
 * out_wj + k*seg_off[s] as a [k][n_s] worker-major block, each value equal to rqsid_auction_scores on the
 * segment alone.  seg_tile_off[S+1] = exclusive scan of ceil(n_s / 64); n_tiles = seg_tile_off[S]. */
int rqsid_seg_auction_scores(const float* x, int64_t n, int32_t dim, const float* centers, int32_t k,
                             int32_t n_seg, const int32_t* seg_off, const int32_t* seg_tile_off,
                             int64_t n_tiles, int32_t half, uint16_t* out_wj, void* stream);

/* Segmented balanced assignment: one auction_lap_half (balancekmeans/__init__.py:12-140) per segment, all
 * segments advanced in lockstep (one launch sequence per round for all of them; a segment stops at its own
 * round count).  Segment s: jobs seg_off[s] .. seg_off[s+1] (n_s), scores at scores + k*seg_off[s] as
 * [k][n_s] fp16 (the layout of rqsid_seg_auction_scores).  Jobs are cut into chunks of
 * rqsid_seg_auction_chunk_jobs() that never straddle segments: seg_chunk_off[S+1] = exclusive scan of
 * ceil(n_s / chunk), total_chunks = seg_chunk_off[S]; n_multi = number of segments of more than one chunk
 * (checked).  active[s] (NULL = all) == 0 skips a segment (its out_assign entries are untouched).
 * out_assign[j] = worker of job j inside its segment; out_rounds[s] (device) = rounds run (0 for the
 * n_s < k fallback, argmin(-D) = the farthest centre, as the reference).  Each segment's result is
 * bit-identical to rqsid_auction_lap_half on its block alone.  Blocks the calling thread (one host read per
 * 8 rounds).  max_rounds <= 0: unbounded. */
int32_t rqsid_seg_auction_chunk_jobs(void);
int64_t rqsid_seg_auction_workspace_bytes(int64_t n_jobs, int32_t n_workers, int32_t n_seg,
                                          int64_t total_chunks, int32_t n_multi);
int rqsid_seg_auction_lap_half(const uint16_t* scores, int32_t n_workers, int32_t n_seg,
                               const int32_t* seg_off, const int32_t* seg_chunk_off, int64_t total_chunks,
                               int32_t n_multi, int64_t n_jobs, const uint8_t* active, int32_t max_rounds,
                               int32_t* out_assign, int32_t* out_rounds, void* workspace,
                               int64_t workspace_bytes, void* stream);

/* Row-sharded balanced assignment, one pass per call: the auction_lap_half of balancekmeans/__init__.py:
 * 12-140 over jobs spread across ranks (rank r owns a contiguous block of n_local of the n_global jobs,
 * scores [k][n_local] fp16 worker-major).  The caller (distributed.ShardedAuction) runs, per round,
 * hist(0) -> sum the [k][256] u32 histograms over ranks -> select(0) -> hist(1) -> sum -> select(1) ->
 * eqcount -> rank_off[w] = eqtot[w] summed over lower ranks -> bid(rank_off) -> resolve -> sum `have`
 * over ranks -> end_round, and stops when the summed `have` equals n_global; after begin it reduces the
 * {max, min} order keys (max / min over ranks) and calls eps.  Every fp16 operation and the tie rule
 * (lowest GLOBAL job index at the top-k boundary, lowest worker among equal bids) are those of
 * rqsid_auction_lap_half, so the assignment equals the single-process auction of the whole matrix.
 * rqsid_dauction_layout gives the byte offsets, inside the workspace, of the buffers the caller
 * reduces: [0] u32[2] {max key, min key} (min initialised to 0xFFFFFFFF), [1] u32 [k][256] histogram
 * followed by one u32 (summed with it: the ranks whose bid list overflowed), [2] u32 [k] eqtot, [3] u32
 * have, and the state it may poll: [4] u8 flag (bit 0: still bidding; cleared by rqsid_dauction_end_round
 * once the reduced `have` equals n_global, after which every pass is a no-op, so the caller need not read
 * it every round), [5] i32 rounds run.  `offsets` holds 6 entries.
 * Bid lists (RQSID_DAUCTION_LIST=0 turns them off): from round 32 (16 at k >= 1024) a round slot may run
 * from per-rank lists of each worker's values near its threshold instead of sweeping the scores, with the
 * same calls and collectives in the same order (the histograms then count listed values).  When the
 * reduced data show a list did not hold, the slot is void (no job state changes, the round does not
 * count) and the next slot runs that round as a sweep; the result is the sweep's in every case. */
int64_t rqsid_dauction_workspace_bytes(int64_t n_local, int32_t n_workers);
/* List-only round slots: workspace bytes [192, 196) hold the mode of the coming slot (u32: 0 sweep, 1 list,
 * 2 void), identical on every rank.  While it reads 1 the caller may run a slot as list_pass(-1),
 * list_pass(0), sum, select(0), list_pass(1), sum, select(1), list_pass(2), gather, list_pass(3, rank_off),
 * resolve, sum, end_round: the same collectives without launching the sweep kernels; a list-only slot that
 * meets a sweep round is void (nothing changes) and the caller returns to full slots at its next poll. */
/* Diagnostics of the row-sharded list state: out (device u32[8]) = {coming slot's mode, round, longest list,
 * mean list length, worker 0's list base key, worker 0's threshold key, summed overflow word, lists over
 * capacity}. */
int rqsid_dauction_debug(const uint16_t* scores, int32_t n_workers, int64_t n_local, int64_t n_global, uint32_t* out,
                         void* workspace, int64_t workspace_bytes, void* stream);
int rqsid_dauction_list_pass(const uint16_t* scores, int32_t n_workers, int64_t n_local, int64_t n_global,
                             int32_t step, const uint32_t* rank_off, void* workspace, int64_t workspace_bytes,
                             void* stream);
int rqsid_dauction_layout(int64_t n_local, int32_t n_workers, int64_t* offsets);
int rqsid_dauction_begin(const uint16_t* scores, int32_t n_workers, int64_t n_local, int64_t n_global,
                         int32_t* out_assign, void* workspace, int64_t workspace_bytes, void* stream);
int rqsid_dauction_eps(const uint16_t* scores, int32_t n_workers, int64_t n_local, int64_t n_global,
                       void* workspace, int64_t workspace_bytes, void* stream);
int rqsid_dauction_hist(const uint16_t* scores, int32_t n_workers, int64_t n_local, int64_t n_global,
                        int32_t low, void* workspace, int64_t workspace_bytes, void* stream);
int rqsid_dauction_select(const uint16_t* scores, int32_t n_workers, int64_t n_local, int64_t n_global,
                          int32_t low, void* workspace, int64_t workspace_bytes, void* stream);
int rqsid_dauction_eqcount(const uint16_t* scores, int32_t n_workers, int64_t n_local, int64_t n_global,
                           void* workspace, int64_t workspace_bytes, void* stream);
int rqsid_dauction_bid(const uint16_t* scores, int32_t n_workers, int64_t n_local, int64_t n_global,
                       const uint32_t* rank_off, void* workspace, int64_t workspace_bytes, void* stream);
int rqsid_dauction_resolve(const uint16_t* scores, int32_t n_workers, int64_t n_local, int64_t n_global,
                           int32_t* out_assign, void* workspace, int64_t workspace_bytes, void* stream);
int rqsid_dauction_end_round(const uint16_t* scores, int32_t n_workers, int64_t n_local, int64_t n_global,
                             void* workspace, int64_t workspace_bytes, void* stream);

/* Greedy unique-nearest match rows (_assign_last_match_matrix hierarchical_rq_kmeans.py:1022-1038,
 * _get_dynamic_match_matrix simplified_semantic_id_generator.py:282-291): group g owns rows
 * sub_off[g]..sub_off[g+1] of dist [total][n_cand]; its first min(rows, max_take) rows each take, in
 * order, their nearest still-unused column (lowest column on exact ties).  match [groups][n_cand]
 * gets 1 for taken columns, n_selected[g] their count (the reference's random fill is host work). */
int rqsid_greedy_match(const float* dist, const int32_t* sub_off, int32_t groups, int32_t n_cand,
                       int32_t max_take, uint8_t* match, int32_t* n_selected, void* stream);

/* Numerics probe (self-test): d = a.b + c with ONE v_mfma_f32_32x32x16_f16 (f16 == 1) or
 * _bf16 (f16 == 0); a [32][16], b [16][32] (half / bfloat16 bits), c/d fp32 [32][32], row-major.  The tests
 * use it to pin the MFMA accumulation model behind rqsid_assign's screening bound.  f16 == 2: ONE
 * v_mfma_scale_f32_32x32x64_f8f6f4 on OCP fp8 e4m3 bytes with unit scales, a [32][64], b [64][32] (the
 * pointers then address bytes). */
int rqsid_mfma_probe(int32_t f16, const uint16_t* a, const uint16_t* b, const float* c, float* d,
                     void* stream);

#ifdef __cplusplus
}
#endif
#endif /* RQSID_H */
