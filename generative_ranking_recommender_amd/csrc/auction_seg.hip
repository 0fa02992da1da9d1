// auction_seg.hip — many independent balanced assignments (balancekmeans.auction_lap_half,
// balancekmeans/__init__.py:12-140) advanced in lockstep: the per-parent sub-K-Means of the middle layer
// (hierarchical_rq_kmeans.py:671-752) and the per-(l1, l2) group sub-K-Means of the last-layer match
// matrix (:968-1053) run one auction per segment, and the reference runs them one after another.  Here
// every round of every live segment is one sequence of launches over all segments (SURVEY.md §7 item 6,
// hard part 5), and segments finish independently (13 rounds when N_s % K == 0, 1002 otherwise).
//
// Segment s: jobs seg_off[s] .. seg_off[s+1] (N_s of them), workers 0 .. K-1, scores at
// W + K*seg_off[s] as a [K][N_s] worker-major fp16 block.  Inside a segment every step is the
// single-auction step of auction.hip (same fp16 operations, same tie rule: the lowest job indices are
// kept at the top-k boundary, equal highest bids go to the lowest worker), so segment s's result is
// bit-identical to rqsid_auction_lap_half on its block alone.
//
// Jobs are cut into chunks of kCh jobs that never straddle segments (seg_chunk_off = exclusive scan of
// ceil(N_s / kCh)).  A segment of one chunk (the last layer's groups: median ~600 rows) selects its
// per-worker thresholds inside one block from LDS histograms (sa_small_select_kernel); wider segments
// (the middle layer's parents, and the single auction of auction.hip) use per-(segment, worker) global
// histograms.  A round of a wide segment is two sweeps of W when each worker's threshold stays in last
// round's high-byte bin (guessed pass with its per-chunk tie counts, then the bids); a worker whose
// threshold left the bin takes the exact two-pass selection and a tie-count sweep in the same round.
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>

#include "internal.h"

// diagnostic build only (-DRQSID_STAMPS, tools/auction_stamps.py): s_memtime cycles of the list round's phases
// (thread 0 of every block that completes a list round) and of resolve blocks
#ifdef RQSID_STAMPS
__device__ unsigned long long g_al_stamps[16];
#define AST(...) __VA_ARGS__
#define ANOW() __builtin_amdgcn_s_memtime()
#else
#define AST(...)
#endif

namespace rqsid {
namespace {

constexpr int kKG = 16;        // workers per block
constexpr int kCh = 1024;      // jobs per chunk
constexpr int kJPT = kCh / 256;
constexpr int kAbovePad = 32;  // u32 per worker in SegAuction::above
constexpr int kRd = 16;        // first-level arrival counters of the fused round end (SegAuction::rdone)
static_assert(kJPT == 4 && kJPT * kKG == 64, "load_chunk<true> takes 4 jobs per lane; sa_bid_kernel keeps one deferral bit per (job slice, worker) in two u32, "
              "and its 64 x 4 eqm slots are zeroed by the 256 threads");

__device__ __forceinline__ float h2f(uint16_t b) { return (float)__builtin_bit_cast(_Float16, b); }
__device__ __forceinline__ uint16_t f2h(float f) { return __builtin_bit_cast(uint16_t, (_Float16)f); }
__device__ __forceinline__ uint32_t okey(uint16_t b) {
  if (b == 0x8000u) b = 0;
  return (b & 0x8000u) ? (~b & 0xFFFFu) : (b | 0x8000u);
}
__device__ __forceinline__ uint16_t okey_inv(uint32_t k) {
  return (k & 0x8000u) ? (uint16_t)(k & 0x7FFFu) : (uint16_t)(~k & 0xFFFFu);
}

// seg_flag bits
constexpr uint8_t kLive = 1;     // segment still bidding
constexpr uint8_t kSingle = 2;   // one chunk: LDS selection

struct SegAuction {
  const uint16_t* W;
  int32_t K;
  int32_t S;
  int64_t total_chunks;
  const int32_t* seg_off;        // [S+1] jobs
  const int32_t* chunk_off;      // [S+1] chunks
  uint8_t* flag;                 // [S]
  uint16_t* eps;                 // [S]
  uint32_t* mm;                  // [S][2] max key, min key
  uint32_t* have;                // [S] jobs with a bidder this round
  int32_t* rounds;               // [S] rounds run (device)
  int32_t* round_dev;            // [1] the current round (device, so a captured block of rounds replays)
  uint32_t* live_count;          // [4]: live segments, multi-chunk segments, a miss in a lean block, a list
                                 // that failed in this block (a list-only block is then replayed)
  uint16_t* cost;                // [N]
  int32_t* hb;                   // [N]
  uint8_t* nobid;                // [N]
  uint32_t* key;                 // [N]
  int32_t n_multi;               // segments of more than one chunk
  int32_t* hidx;                 // [S] rank among the multi-chunk segments (-1: one chunk)
  int32_t* mseg;                 // [n_multi] the multi-chunk segments in order
  uint32_t* hist;                // [n_multi*K][256]
  uint32_t* sel;                 // [S*K][4]: b1, rank in bin, T, need_eq
  uint32_t* eqcnt;               // [K][total_chunks]
  // row-sharded mode (one segment spread over ranks, rqsid_dauction_*): the global job count decides
  // jobs-per-worker and completion; rank_off[w] = equal-to-T values of worker w on lower ranks
  int64_t n_glob;                // 0: single process
  const uint32_t* rank_off;      // [K] or null
  uint32_t* eqtot;               // [S*K] equal-to-T values per (segment, worker) on this rank
  // guessed high byte (single-process multi-chunk segments; null in the row-sharded mode): one sweep
  // histograms the low bytes of the values in last round's bin b1 and counts the values above it; when
  // the threshold is still in b1 that is the exact selection, otherwise (miss) the worker takes the
  // two-pass selection this round
  uint32_t* above;               // [n_multi*K][kAbovePad] values with high byte > b1 (one line per worker:
                                 // every chunk block adds to it)
  uint8_t* miss;                 // [n_multi*K]
  uint16_t* chist;               // [K][total_chunks][256] each chunk's low-byte histogram of bin b1 from the
                                 // guessed pass: a hit worker's per-chunk tie count is entry T & 255
  uint32_t* any_miss;            // [1] some worker missed this round (the two-pass kernels exit at once if not)
  // the round state at the start of a lean block (rounds without the two-pass kernels, replayed in full
  // when a worker missed): costs, winners, no-bid flags, assignment, selections, segment flags and rounds
  uint16_t* s_cost;
  int32_t* s_hb;
  uint8_t* s_nobid;
  int32_t* s_out;
  uint32_t* s_sel;
  uint8_t* s_flag;
  int32_t* s_rounds;
  // bid lists (multi-chunk segments; sa_list_round_kernel explains them): per (segment, worker) the jobs
  // whose value key was >= lkb when the list was built, with their raw scores
  uint2* lst;                    // per multi-chunk segment r: [K][lcs[r]] entries {job, raw score bits} at loff[r]
  uint32_t* lcnt;                // [n_multi*K][kAbovePad]: entries of the worker's list (0: no list)
  uint32_t* lkb;                 // [n_multi*K]: the list's base key
  uint8_t* lbad;                 // [n_multi*K]: 1 = the worker takes the sweep path this round
  int64_t* loff;                 // [n_multi]
  int32_t* lcs;                  // [n_multi]: capacity per worker, 4 * (N_s / K) + 256
  // multi-block list rounds (one wide segment, long lists; sa_mlist_* kernels): entry chunks per worker
  // (0: the one-block-per-worker sa_list_round_kernel), per worker the two radix histograms, {b1, above, T,
  // need}, the jobs of the values equal to T, their count and the round's list verdict
  int32_t lmb_chunks;
  uint32_t* lh;                  // [n_multi*K][512]
  uint32_t* lsel;                // [n_multi*K][4]
  uint32_t* leq;                 // [n_multi*K][kListEq]
  uint32_t* leqn;                // [n_multi*K]
  uint8_t* lok;                  // [n_multi*K]
  uint32_t* lany;                // [1] some worker's list failed this round (0: the sweep kernels exit at once)
  int32_t lstart;                // first round that builds lists (kListStart; RQSID_LIST_START)
  int32_t ldelta;                // keys below last round's threshold a list keeps (RQSID_LIST_DELTA, 1..128)
  uint32_t* lstat;               // [8] list-round verdict counts (RQSID_LIST_STATS=1; null otherwise): ok, no
                                 // list, overflow, leftover round, threshold below the base, too few values,
                                 // too many ties (multi-block)
  // row-sharded list rounds (rqsid_dauction_*, da_* kernels): dmode[0] = this round slot's mode (kDSweep,
  // kDList, kDVoid), dmode[1] = 1 in a sweep slot (any_miss points here: the sweep kernels exit otherwise);
  // each rank's list of worker w is lst[w * dcap ..], walked by dnb blocks per worker
  uint32_t* dmode;
  int64_t dcap;
  int32_t dnb;
  int32_t dlist_on;              // RQSID_DAUCTION_LIST (default 1): 0 keeps every round a sweep, for A/B
  // one-segment auctions (single process): {blocks arrived << 32 | jobs with a bidder} of the round's resolve;
  // the last block to arrive ends the round (sa_round_end_kernel's work, one launch fewer per round)
  unsigned long long* rdone;
  uint32_t* js;                  // (list rounds) per job {winner & 0xFFFF, cost bits}: one gather per listed job
  int32_t rcount;                // end-of-round: add the live count for the host's poll (a block's last round)
  // one-segment single-process auctions: the segment's job count (0 otherwise).  The segment, its chunks and its
  // list layout are then arithmetic (segment 0, jobs [0, one_n), list capacity 4 * (one_n / K) + 256 at offset
  // 0): the round kernels take them without the dependent table loads that open every block otherwise
  int64_t one_n;
};
constexpr int64_t kListMaxJpw = 16384;  // one-block list rounds only while the average jobs per worker per segment is at most this
constexpr int64_t kListBlockJpw = 8192;  // one wide segment above this many jobs per worker: multi-block list rounds
// lists are built from this round on: an auction whose N is a multiple of K settles in a few dozen rounds,
// where building lists costs more than they save (K=128 x 10M, 24 rounds: 4.93 against 3.26 ms per round);
// the 1002-round auctions (N % K != 0) run lists for the rest.  Starting one-block lists at round 1 was
// measured worse (K=2560 x 6.25M 2.07 -> 2.19 ms per round, K=1280 x 10M 1.99 -> 2.43): thresholds move
// fast in the first rounds and the lists overflow, so those rounds pay the list pass and the sweep)
constexpr int kListStart = 32;
// ... and from round 16 at K >= 1024 (candidate fits: a sweep there reads K x N fp16 scores, up to 32 GB, so
// earlier lists pay even with the overflow failures of the first rounds): K=2560 x 6.25M 1.69 -> 1.34 ms per
// round, K=1280 x 10M 1.71 -> 1.50, K=1280 x 1M 0.190 -> 0.163; at K=128 x 1M round 16 lost (0.105 -> 0.137),
// and a settling K=1280 x 1.28M auction (27 rounds) 4.04 -> 4.83 (profiles/r4_list_start.jsonl)
constexpr int kListStartWide = 16;
constexpr int kListWideK = 1024;
constexpr int kMCH = 2048;               // list entries per block of a multi-block list round
constexpr int kListDelta = 32;   // default keys below last round's threshold kept in the bid list (64 measured the same or slower: DESIGN 3.3)

__device__ __forceinline__ int seg_of(const int32_t* __restrict__ off, int n_seg, int64_t i) {
  int lo = 0, hi = n_seg - 1;  // last s with off[s] <= i
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if ((int64_t)off[mid] <= i) lo = mid; else hi = mid - 1;
  }
  return lo;
}

struct ChunkInfo {
  int s;
  int64_t seg_j0;   // first job of the segment
  int64_t n_s;      // jobs in the segment
  int64_t j0;       // first job of the chunk (global)
  int64_t nj;       // jobs in the chunk
  int64_t cis;      // chunk index inside the segment
};

__device__ __forceinline__ ChunkInfo chunk_info(const SegAuction& a, int64_t c) {
  ChunkInfo ci;
  if (a.one_n) {
    ci.s = 0;
    ci.seg_j0 = 0;
    ci.n_s = a.one_n;
    ci.cis = c;
    ci.j0 = c * kCh;
    ci.nj = min((int64_t)kCh, a.one_n - ci.j0);
    return ci;
  }
  ci.s = seg_of(a.chunk_off, a.S, c);
  ci.seg_j0 = a.seg_off[ci.s];
  ci.n_s = a.seg_off[ci.s + 1] - ci.seg_j0;
  ci.cis = c - a.chunk_off[ci.s];
  ci.j0 = ci.seg_j0 + ci.cis * kCh;
  ci.nj = min((int64_t)kCh, ci.seg_j0 + ci.n_s - ci.j0);
  return ci;
}

__device__ __forceinline__ uint16_t value_bits(int w, uint16_t wv, int32_t hbj, uint16_t cj) {
  if (hbj == w) return wv;  // the previous round's winner keeps its raw score
  return f2h(h2f(wv) - h2f(cj));
}

// the same value as fp16: every step of the reference is one fp16 rounding of an fp32 result of two fp16
// operands, which equals the fp16 operation itself (11-bit operands, 24-bit intermediate: the double
// rounding is innocuous); order and equality of these values are those of okey (-0 == +0, no NaN)
__device__ __forceinline__ _Float16 value_h(int w, uint16_t wv, int32_t hbj, uint16_t cj) {
  const _Float16 r = __builtin_bit_cast(_Float16, wv);
  return hbj == w ? r : (_Float16)(r - __builtin_bit_cast(_Float16, cj));
}

// a job's last winner and cost from the packed word when the list rounds keep one (else the two arrays); the
// packed word's winner is 16 bits (js is allocated only for K <= 65535), 0xFFFF = none
__device__ __forceinline__ int32_t js_hb(const SegAuction& a, int64_t j) {
  if (!a.js) return a.hb[j];
  const uint32_t h = a.js[j] >> 16;
  return h == 0xFFFFu ? -1 : (int32_t)h;
}
__device__ __forceinline__ uint16_t js_cost(const SegAuction& a, int64_t j) {
  return a.js ? (uint16_t)(a.js[j] & 0xFFFFu) : a.cost[j];
}

__device__ __forceinline__ const uint16_t* wrow(const SegAuction& a, const ChunkInfo& ci, int w) {
  return a.W + (int64_t)a.K * ci.seg_j0 + (int64_t)w * ci.n_s - ci.seg_j0;  // index with the global job
}

// One chunk's scores for the block's workers, with the jobs' winners and costs: every load is
// unconditional (the job and worker indices are clamped into the segment), so the compiler issues the
// whole chunk's loads at once and counts them, instead of draining the queue at each conditional load.
// Lanes past the chunk's end (t * 256 + lane >= nj) hold copies and must be masked with `live`.
struct ChunkScores {
  uint16_t v[kJPT][kKG];
  int32_t hb[kJPT];
  uint16_t c[kJPT];
};

// Job of slice t for this thread: slice-major (t * 256 + thread) in general; with VEC every lane takes
// four consecutive jobs (4 * thread + t) and loads them with one 8-byte load per worker row, which needs
// 8-byte aligned rows and chunks of a multiple of 4 jobs (the single auction with N % 4 == 0).
template <bool VEC>
__device__ __forceinline__ int64_t job_of(int t) {
  return VEC ? 4 * (int64_t)threadIdx.x + t : (int64_t)t * 256 + threadIdx.x;
}

template <bool VEC>
__device__ __forceinline__ void load_chunk(const SegAuction& a, const ChunkInfo& ci, int w0, ChunkScores& cs) {
  if (VEC) {
    const int64_t j = ci.j0 + min(4 * (int64_t)threadIdx.x, ci.nj - 4);
    const int4 hb4 = *reinterpret_cast<const int4*>(a.hb + j);
    const uint2 c4 = *reinterpret_cast<const uint2*>(a.cost + j);
    cs.hb[0] = hb4.x;
    cs.hb[1] = hb4.y;
    cs.hb[2] = hb4.z;
    cs.hb[3] = hb4.w;
    cs.c[0] = (uint16_t)c4.x;
    cs.c[1] = (uint16_t)(c4.x >> 16);
    cs.c[2] = (uint16_t)c4.y;
    cs.c[3] = (uint16_t)(c4.y >> 16);
#pragma unroll
    for (int g = 0; g < kKG; ++g) {
      const uint2 q = *reinterpret_cast<const uint2*>(wrow(a, ci, min(w0 + g, a.K - 1)) + j);
      cs.v[0][g] = (uint16_t)q.x;
      cs.v[1][g] = (uint16_t)(q.x >> 16);
      cs.v[2][g] = (uint16_t)q.y;
      cs.v[3][g] = (uint16_t)(q.y >> 16);
    }
    return;
  }
#pragma unroll
  for (int t = 0; t < kJPT; ++t) {
    const int64_t j = ci.j0 + min((int64_t)(t * 256 + threadIdx.x), ci.nj - 1);
    cs.hb[t] = a.hb[j];
    cs.c[t] = a.cost[j];
#pragma unroll
    for (int g = 0; g < kKG; ++g) cs.v[t][g] = wrow(a, ci, min(w0 + g, a.K - 1))[j];
  }
}

// ---- setup ----
__global__ __launch_bounds__(256) void sa_seg_init_kernel(SegAuction a, const uint8_t* __restrict__ active) {
  const int s = blockIdx.x * 256 + threadIdx.x;
  if (s >= a.S) return;
  const int64_t n_s = a.n_glob ? a.n_glob : a.seg_off[s + 1] - a.seg_off[s];
  const int64_t nch = a.chunk_off[s + 1] - a.chunk_off[s];
  uint8_t f = 0;
  // live: requested, non-empty, and N_s >= K (N_s < K takes the argmin fallback, 0 rounds)
  if ((!active || active[s]) && n_s > 0 && n_s >= a.K) f |= kLive;
  if ((f & kLive) && a.live_count) atomicAdd(a.live_count, 1u);
  if (nch == 1 && !a.n_glob) f |= kSingle;
  a.flag[s] = f;
  a.mm[2 * s] = 0;
  a.mm[2 * s + 1] = 0xFFFFFFFFu;
  a.have[s] = 0;
  a.rounds[s] = 0;
  if (s == 0) *a.round_dev = 0;
}

__global__ __launch_bounds__(256) void sa_job_init_kernel(SegAuction a, int64_t n) {
  for (int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x; j < n; j += (int64_t)gridDim.x * 256) {
    a.cost[j] = 0;
    a.hb[j] = -1;
    a.nobid[j] = 0;
    a.key[j] = 0;
    if (a.js) a.js[j] = 0xFFFF0000u;
  }
}

// min / max of each live segment's whole score block (eps), one block per (chunk, worker group)
__global__ __launch_bounds__(256) void sa_minmax_kernel(SegAuction a) {
  const ChunkInfo ci = chunk_info(a, blockIdx.x);
  if (!(a.flag[ci.s] & kLive)) return;
  const int w0 = blockIdx.y * kKG, nw = min(kKG, a.K - w0);
  uint32_t mx = 0, mn = 0xFFFFFFFFu;
  for (int g = 0; g < nw; ++g) {
    const uint16_t* row = wrow(a, ci, w0 + g);
    for (int64_t t = threadIdx.x; t < ci.nj; t += 256) {
      const uint32_t k = okey(row[ci.j0 + t]);
      mx = max(mx, k);
      mn = min(mn, k);
    }
  }
  for (int o = 32; o > 0; o >>= 1) {
    mx = max(mx, (uint32_t)__shfl_xor((int)mx, o));
    mn = min(mn, (uint32_t)__shfl_xor((int)mn, o));
  }
  if ((threadIdx.x & 63) == 0) {
    atomicMax(&a.mm[2 * ci.s], mx);
    atomicMin(&a.mm[2 * ci.s + 1], mn);
  }
}

__global__ __launch_bounds__(256) void sa_eps_kernel(SegAuction a) {
  const int s = blockIdx.x * 256 + threadIdx.x;
  if (s >= a.S || !(a.flag[s] & kLive)) return;
  const float mx = h2f(okey_inv(a.mm[2 * s])), mn = h2f(okey_inv(a.mm[2 * s + 1]));
  const uint16_t spread = f2h(mx - mn);
  uint16_t eps = f2h(h2f(spread) / 50.0f);
  const uint16_t floor_eps = f2h(1e-4f);
  if (!(h2f(eps) >= h2f(floor_eps))) eps = floor_eps;
  a.eps[s] = eps;
}

// N_s < K: the reference's argmin(-D) fallback (the FARTHEST centre), balancekmeans/__init__.py:24-26
__global__ __launch_bounds__(256) void sa_fallback_kernel(SegAuction a, int32_t* __restrict__ out) {
  const ChunkInfo ci = chunk_info(a, blockIdx.x);
  const int64_t n_dec = a.n_glob ? a.n_glob : ci.n_s;
  if (n_dec >= a.K || ci.n_s == 0) return;
  for (int64_t t = threadIdx.x; t < ci.nj; t += 256) {
    const int64_t j = ci.j0 + t;
    float best = INFINITY;
    int bw = 0;
    for (int w = 0; w < a.K; ++w) {
      const float v = h2f(wrow(a, ci, w)[j]);
      if (v < best) { best = v; bw = w; }
    }
    out[j] = bw;
  }
}

// ---- selection of the (jpw+1)-th largest value per (segment, worker) ----
// Walk a 256-bin histogram from the top for the bin holding `rank` (1-based): one wave, 4 bins a lane.
// Returns the bin b and the count strictly above it (b stops at 0 like the serial walk of auction.hip).
__device__ __forceinline__ void wave_select(const uint32_t* __restrict__ h, uint32_t rank, uint32_t& bin,
                                            uint32_t& above) {
  const int lane = threadIdx.x & 63;
  const uint32_t h0 = h[4 * lane], h1 = h[4 * lane + 1], h2 = h[4 * lane + 2], h3 = h[4 * lane + 3];
  const uint32_t own = h0 + h1 + h2 + h3;
  uint32_t suf = own;  // inclusive suffix sum over lanes >= lane
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = (uint32_t)__shfl_down((int)suf, o);
    if (lane + o < 64) suf += y;
  }
  const unsigned long long m = __ballot(suf >= rank);
  const int L = m ? 63 - __clzll(m) : 0;
  uint32_t b = 0, ab = 0;
  if (lane == L) {
    uint32_t acc = suf - own;  // strictly above this lane's bins
    const uint32_t hv[4] = {h0, h1, h2, h3};
    int q = 3;
    for (; q > 0; --q) {
      if (acc + hv[q] >= rank) break;
      acc += hv[q];
    }
    // lane 0 bin 0 is the floor; a higher lane's bin 4L may still fall through to a lower lane only if
    // the ballot was empty, which cannot happen while the segment holds >= rank values
    b = 4 * L + q;
    ab = acc;
  }
  bin = (uint32_t)__shfl((int)b, L);
  above = (uint32_t)__shfl((int)ab, L);
}

// multi-chunk segments: global histograms.  MODE 0: high bytes, 1: low bytes of the values in the
// selected bin b1 (sel[0]).  With the guessed pass on (a.miss), they run only for the workers it missed.
template <int MODE, bool VEC>
__global__ __launch_bounds__(256) void sa_hist_kernel(SegAuction a) {
  if (a.any_miss && !*a.any_miss) return;
  const ChunkInfo ci = chunk_info(a, blockIdx.x);
  const uint8_t f = a.flag[ci.s];
  if (!(f & kLive) || (f & kSingle)) return;
  __shared__ uint32_t h[kKG][256];
  const int w0 = blockIdx.y * kKG, nw = min(kKG, a.K - w0);
  const int lane = threadIdx.x & 63;
  const int64_t sw0 = (int64_t)ci.s * a.K + w0;
  const int64_t hw0 = (int64_t)a.hidx[ci.s] * a.K + w0;
  uint32_t part = (1u << nw) - 1u;  // workers taking this pass
  if (a.miss) {
    part = 0;
    for (int g = 0; g < nw; ++g) part |= (uint32_t)(a.miss[hw0 + g] != 0) << g;
    if (!part) return;
  }
  for (int i = threadIdx.x; i < kKG * 256; i += 256) (&h[0][0])[i] = 0;
  __syncthreads();
  // high-byte pass: a worker's values crowd into one or two high-byte bins, where same-address LDS
  // atomics serialise a wave 64-fold.  The bins at and just below last round's threshold (sel[0]; any
  // value is correct, it only decides which bins take the fast path) are counted with ballots.
  uint32_t b1[kKG], n0[kKG] = {}, n1[kKG] = {};
  for (int g = 0; g < kKG; ++g) b1[g] = g < nw ? a.sel[(sw0 + g) * 4 + 0] & 255u : 0;
  ChunkScores cs;
  load_chunk<VEC>(a, ci, w0, cs);
#pragma unroll
  for (int t = 0; t < kJPT; ++t) {
    const bool live = job_of<VEC>(t) < ci.nj;
#pragma unroll
    for (int g = 0; g < kKG; ++g) {
      if (!((part >> g) & 1u)) continue;
      const uint32_t k = okey(value_bits(w0 + g, cs.v[t][g], cs.hb[t], cs.c[t]));
      if (MODE != 0) {
        if (live && (k >> 8) == b1[g]) atomicAdd(&h[g][k & 255], 1u);
      } else {
        const uint32_t d = b1[g] - (k >> 8);  // 0: the guessed bin, 1: the bin below
        n0[g] += (uint32_t)__popcll(__ballot(live && d == 0));
        n1[g] += (uint32_t)__popcll(__ballot(live && d == 1));
        if (live && d > 1) atomicAdd(&h[g][k >> 8], 1u);
      }
    }
  }
  if (MODE == 0 && lane == 0) {
    for (int g = 0; g < nw; ++g) {
      if (n0[g]) atomicAdd(&h[g][b1[g]], n0[g]);
      if (n1[g]) atomicAdd(&h[g][b1[g] - 1], n1[g]);  // n1 > 0 implies b1 >= 1
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < nw * 256; i += 256) {
    const uint32_t c = (&h[0][0])[i];  // zero for the workers that did not take part
    if (c) atomicAdd(&a.hist[(hw0 + i / 256) * 256 + (i & 255)], c);
  }
}

// Per-lane view of one chunk for the branch-free sweeps: a lane past the chunk's end gets no winner and
// the cost NaN, so every one of its values is NaN (neither above nor equal to any threshold) without a
// per-value liveness test; the histogram pass also offsets its keys below every bin (dead).  A job's
// value for worker w is r - c' with c' = -0 for the previous winner (its raw score r; r - -0 also turns
// -0 into +0) and the job's cost otherwise: one fp16 subtraction, the reference's step (value_h).
struct LaneJobs {
  int32_t hb[kJPT];
  _Float16 c[kJPT];
  int32_t dead[kJPT];  // 0 or -0x20000
};

template <bool VEC>
__device__ __forceinline__ LaneJobs lane_jobs(const ChunkInfo& ci, const ChunkScores& cs) {
  LaneJobs lj;
#pragma unroll
  for (int t = 0; t < kJPT; ++t) {
    const bool live = job_of<VEC>(t) < ci.nj;
    lj.hb[t] = live ? cs.hb[t] : -1;
    lj.c[t] = __builtin_bit_cast(_Float16, live ? cs.c[t] : (uint16_t)0x7E00u);
    lj.dead[t] = live ? 0 : -0x20000;
  }
  return lj;
}

__device__ __forceinline__ _Float16 lane_value(int w, uint16_t v, int32_t hbj, _Float16 c) {
  return __builtin_bit_cast(_Float16, v) - (hbj == w ? (_Float16)-0.0f : c);
}

// The guessed pass: per worker, the histogram of its values' keys in a 256-key window around last round's
// threshold (window_base) and the count of keys above the window, in one sweep with no ballots and no
// branches per value other than the LDS atomic: d = okey(x) - base is the window slot (0..255), >= 256
// above the window (slot 256), negative below.  Both the values in the window and those above it are
// about 1/K of a worker's values, so the predicated atomic is rare.  d comes from x's raw bits in one
// operation, by the sign of the window's keys (uniform per worker): x = v + (0 - c) is never -0 (a
// round-to-nearest sum is -0 only when both addends are), so okey(x) = bits | 0x8000 for x >= +0 and
// 0xFFFF - bits for x < 0, and
//   a window of keys >= 0x8000 (values >= +0): d = sext16(bits) + 0x8000 - base (every x < 0 lands below),
//   a window of negative values:               d = 0xFFFF - base - bits (every x >= +0 lands above).
// A lane past the chunk's end takes the cost +inf (x = -inf: below every window of finite keys); a window
// that reaches -inf's key (base < 0x400) takes explicit dead offsets (DEAD).
constexpr int kGStride = 260;  // LDS words per worker: 256 window slots + the above count, padded to 16 B

// The guessed window: 256 consecutive keys centred on last round's threshold T (sel[2]), kept on one
// side of the sign boundary (0x8000) so that d = okey(x) - base is one operation on x's bits.  A
// threshold that moves less than ~128 keys stays inside it (a window aligned to T's high byte missed
// whenever T crossed a byte boundary).
template <int SH = 0>
__device__ __forceinline__ int32_t window_base(uint32_t T) {
  constexpr int32_t span = 256 << SH;
  const int32_t t = (int32_t)(T & 0xFFFFu) - span / 2;
  return T >= 0x8000u ? min(max(t, 0x8000), 0x10000 - span) : min(max(t, 0), 0x8000 - span);
}

// SH > 0 (one-chunk segments): a coarse window of 256 slots of 2^SH keys; FINE: the second pass, counting
// the keys inside the selected coarse slot csl (2^SH fine slots, stride hs per worker)
template <bool NEG, bool DEAD, int SH, bool FINE>
__device__ __forceinline__ void guess_worker(const uint16_t (&v)[kJPT], const LaneJobs& lj, const _Float16 (&nc)[kJPT],
                                             int w, int32_t addk, int32_t csl, uint32_t* __restrict__ hg) {
#pragma unroll
  for (int t = 0; t < kJPT; ++t) {
    const _Float16 x = __builtin_bit_cast(_Float16, v[t]) + (lj.hb[t] == w ? (_Float16)0.0f : nc[t]);
    const uint32_t b = __builtin_bit_cast(uint16_t, x);
    int32_t d = NEG ? addk - (int32_t)b : (int32_t)(int16_t)b + addk;
    if (DEAD) d += lj.dead[t];
    if (FINE) {
      if ((d >> SH) == csl) atomicAdd(&hg[d & ((1 << SH) - 1)], 1u);
    } else {
      if (d >= 0) atomicAdd(&hg[min(d >> SH, 256)], 1u);
    }
  }
}

template <bool DEAD, int SH = 0, bool FINE = false>
__device__ __forceinline__ void guess_values(const ChunkScores& cs, const LaneJobs& lj, const _Float16 (&nc)[kJPT],
                                             const int32_t (&addk)[kKG], uint32_t negbin, int w0, uint32_t* h,
                                             const int32_t* csl = nullptr, int hs = kGStride) {
#pragma unroll
  for (int g = 0; g < kKG; ++g) {
    const uint16_t v[kJPT] = {cs.v[0][g], cs.v[1][g], cs.v[2][g], cs.v[3][g]};
    const int32_t c = FINE ? csl[g] : 0;
    if ((negbin >> g) & 1u) guess_worker<true, DEAD, SH, FINE>(v, lj, nc, w0 + g, addk[g], c, h + g * hs);
    else guess_worker<false, DEAD, SH, FINE>(v, lj, nc, w0 + g, addk[g], c, h + g * hs);
  }
}

// the list slot of each worker's values: d >= dlist (d as in guess_worker: the offset of the value's
// key from the window base, 256 = above the window), i.e. keys >= T_prev - kListDelta
__device__ __forceinline__ int32_t list_dmin(uint32_t T, int32_t delta) {
  if (T == 0) return 0x7FFFFFFF;  // no threshold yet (round 0: every worker takes the exact passes)
  return max(0, (int32_t)(T & 0xFFFFu) - delta - window_base(T));
}

// list verdict statistics (diagnostics only: RQSID_LIST_STATS=1)
__device__ __forceinline__ void list_stat(const SegAuction& a, int why) {
  if (a.lstat) atomicAdd(&a.lstat[why], 1u);
}
__device__ __forceinline__ int list_fail_why(uint32_t n, uint32_t cap, int counter) {
  return n == 0 ? 1 : n > cap ? 2 : counter > 1000 ? 3 : 4;
}

// Append this block's values of the list range to their workers' lists: the window histogram gives each
// worker's count (slots >= dlist and the above slot), one global atomic per (block, worker) reserves the
// range, an LDS counter places each value inside it (order inside a block's range is arbitrary; the bid
// pass ranks equal values by job index).  Entries past a worker's capacity are dropped (select_guess then
// marks the worker for the sweep).
template <bool VEC>
__device__ __forceinline__ void list_append(const SegAuction& a, const ChunkInfo& ci, const ChunkScores& cs,
                                            const LaneJobs& lj, const _Float16 (&nc)[kJPT], const int32_t (&addk)[kKG],
                                            uint32_t negbin, bool dead, int w0, int nw, int64_t hw0, uint32_t* h) {
  __shared__ uint32_t lbase[kKG], lpos[kKG];
  __shared__ int32_t ldm[kKG];
  __syncthreads();  // the histogram flush above read h
  // per worker: count of slots >= dlist (16 threads per worker, 16 slots each, + the above slot)
  {
    const int g = threadIdx.x >> 4, q = threadIdx.x & 15;
    int32_t dm = 0;
    uint32_t part = 0;
    if (g < nw) {
      dm = list_dmin(a.sel[((int64_t)ci.s * a.K + w0 + g) * 4 + 2], a.ldelta);
      for (int sl = q * 16; sl < q * 16 + 16; ++sl) part += sl >= dm ? h[g * kGStride + sl] : 0u;
      if (q == 0 && dm <= 256) part += h[g * kGStride + 256];  // (no threshold yet: nothing listed)
    }
    for (int o = 8; o > 0; o >>= 1) part += (uint32_t)__shfl_xor((int)part, o);
    if (q == 0 && g < kKG) {
      ldm[g] = dm;
      lpos[g] = 0;
      lbase[g] = g < nw && part ? atomicAdd(&a.lcnt[(hw0 + g) * kAbovePad], part) : 0u;
      if (g < nw && dm <= 256 && a.lbad[hw0 + g] && blockIdx.x == a.chunk_off[ci.s])  // (one block per worker)
        a.lkb[hw0 + g] = (uint32_t)(window_base(a.sel[((int64_t)ci.s * a.K + w0 + g) * 4 + 2]) + dm);
    }
  }
  __syncthreads();
  const int r = a.hidx[ci.s];
  const uint32_t cap = (uint32_t)a.lcs[r];
  uint2* const L0 = a.lst + a.loff[r];
#pragma unroll
  for (int g = 0; g < kKG; ++g) {
    if (g >= nw) break;
    const int w = w0 + g;
    const int32_t addg = addk[g], dm = ldm[g];
    const bool neg = (negbin >> g) & 1u;
#pragma unroll
    for (int t = 0; t < kJPT; ++t) {
      const _Float16 x = __builtin_bit_cast(_Float16, cs.v[t][g]) + (lj.hb[t] == w ? (_Float16)0.0f : nc[t]);
      const uint32_t b = __builtin_bit_cast(uint16_t, x);
      int32_t d = neg ? addg - (int32_t)b : (int32_t)(int16_t)b + addg;
      if (dead) d += lj.dead[t];
      if (d >= dm) {
        const uint32_t pos = lbase[g] + atomicAdd(&lpos[g], 1u);
        if (pos < cap) L0[(int64_t)w * cap + pos] = make_uint2((uint32_t)(ci.j0 + job_of<VEC>(t)), cs.v[t][g]);
      }
    }
  }
}

template <bool VEC>
__global__ __launch_bounds__(256) void sa_guess_hist_kernel(SegAuction a) {
  if (a.lany && !*a.lany) return;  // every list held this round (lany: sa_list_round_kernel)
  const ChunkInfo ci = chunk_info(a, blockIdx.x);
  const uint8_t f = a.flag[ci.s];
  if (!(f & kLive) || (f & kSingle)) return;
  constexpr int kStride = kGStride;
  __shared__ uint32_t h[kKG * kStride];
  const int w0 = blockIdx.y * kKG, nw = min(kKG, a.K - w0);
  const int64_t sw0 = (int64_t)ci.s * a.K + w0;
  const int64_t hw0 = (int64_t)a.hidx[ci.s] * a.K + w0;
  for (int i = threadIdx.x; i < kKG * kStride / 4; i += 256) reinterpret_cast<uint4*>(h)[i] = make_uint4(0, 0, 0, 0);
  // workers past K: a bin of values >= +0 with every d negative
  int32_t addk[kKG];
  uint32_t negbin = 0;
  bool low = false;  // some worker's bin holds -inf
  bool any_bad = !a.lst;
  for (int g = 0; g < kKG; ++g) {
    addk[g] = -0x20000;
    if (g >= nw) continue;
    if (a.lst && !a.lbad[hw0 + g]) continue;  // its list gave this round's threshold and bids: no values here
    any_bad = true;
    const int32_t base = window_base(a.sel[(sw0 + g) * 4 + 2]);
    if (base >= 0x8000) {
      addk[g] = 0x8000 - base;
    } else {
      addk[g] = 0xFFFF - base;
      negbin |= 1u << g;
      low |= base < 0x400;
    }
  }
  if (!any_bad) return;  // block-uniform
  ChunkScores cs;
  load_chunk<VEC>(a, ci, w0, cs);
  const LaneJobs lj = lane_jobs<VEC>(ci, cs);
  _Float16 nc[kJPT];
#pragma unroll
  for (int t = 0; t < kJPT; ++t) nc[t] = lj.dead[t] ? (_Float16)-INFINITY : (_Float16)0.0f - lj.c[t];
  __syncthreads();
  if (low && ci.nj < kCh) guess_values<true>(cs, lj, nc, addk, negbin, w0, h);
  else guess_values<false>(cs, lj, nc, addk, negbin, w0, h);
  __syncthreads();
  if (threadIdx.x < nw && h[threadIdx.x * kStride + 256])
    atomicAdd(&a.above[(hw0 + threadIdx.x) * kAbovePad], h[threadIdx.x * kStride + 256]);
  // counts <= kCh fit 16 bits; one 8-byte store per 4 slots; worker-major, so a worker's per-chunk tie
  // counts (eqscan) lie in one contiguous run
  for (int i = threadIdx.x; i < nw * 64; i += 256) {
    const uint32_t* q = &h[(i >> 6) * kStride + 4 * (i & 63)];
    uint16_t* dst = a.chist + ((int64_t)(w0 + (i >> 6)) * a.total_chunks + blockIdx.x) * 256 + 4 * (i & 63);
    *reinterpret_cast<uint2*>(dst) = make_uint2(q[0] | (q[1] << 16), q[2] | (q[3] << 16));
  }
  for (int i = threadIdx.x; i < nw * 256; i += 256) {
    const uint32_t c = h[(i >> 8) * kStride + (i & 255)];
    if (c) atomicAdd(&a.hist[(hw0 + (i >> 8)) * 256 + (i & 255)], c);
  }
  if (a.lst && *a.round_dev >= a.lstart)  // (block-uniform)
    list_append<VEC>(a, ci, cs, lj, nc, addk, negbin, low && ci.nj < kCh, w0, nw, hw0, h);
}

// one wave per (segment, worker) of the multi-chunk segments
template <bool LOW>
__global__ __launch_bounds__(256) void sa_select_kernel(SegAuction a) {
  if (a.any_miss && !*a.any_miss) return;
  const int64_t hw = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (hw >= (int64_t)a.n_multi * a.K) return;
  const int s = a.mseg[hw / a.K];
  const int w = (int)(hw % a.K);
  if (!(a.flag[s] & kLive)) return;
  if (a.miss && !a.miss[hw]) return;  // the guessed pass found this worker's threshold
  const int64_t n_s = a.n_glob ? a.n_glob : a.seg_off[s + 1] - a.seg_off[s];
  const uint32_t jpw = (uint32_t)(n_s / a.K);
  uint32_t* h = a.hist + hw * 256;
  uint32_t* sel = a.sel + ((int64_t)s * a.K + w) * 4;
  const uint32_t rank = LOW ? sel[1] : jpw + 1;
  uint32_t b, above;
  wave_select(h, rank, b, above);
  const int lane = threadIdx.x & 63;
  if (lane == 0) {
    if (!LOW) {
      sel[0] = b;
      sel[1] = rank - above;
      sel[3] = above;
    } else {
      const uint32_t T = (sel[0] << 8) | b;
      const uint32_t c_gt = sel[3] + above;
      sel[2] = T;
      sel[3] = jpw - c_gt;
    }
  }
  for (int i = lane; i < 256; i += 64) h[i] = 0;  // ready for the next histogram
}

// Exclusive scan of one worker's per-chunk tie counts over its segment's chunks (one wave), into the eqcnt
// offsets and the segment total eqtot.  The counts come from the guessed pass's chunk histograms (ch: the
// worker's run at slot T & 255; a hit worker, from select_guess) or from sa_eqcount_kernel (eqcnt itself).
// Each lane loads kScanPer consecutive chunks' counts at once: one round of load latency per 64 * kScanPer
// chunks.
constexpr int kScanPer = 16;
__device__ __forceinline__ void scan_ties(const SegAuction& a, int s, int w, const uint16_t* __restrict__ ch) {
  const int lane = threadIdx.x & 63;
  uint32_t* e = a.eqcnt + (int64_t)w * a.total_chunks;
  const int64_t c0 = a.chunk_off[s], c1 = a.chunk_off[s + 1];
  uint32_t carry = 0;
  for (int64_t base = c0; base < c1; base += 64 * kScanPer) {
    const int64_t i0 = base + (int64_t)lane * kScanPer;
    uint32_t v[kScanPer];
    uint32_t tot = 0;
#pragma unroll
    for (int q = 0; q < kScanPer; ++q) {
      const int64_t i = min(i0 + q, c1 - 1);
      v[q] = i0 + q < c1 ? (ch ? (uint32_t)ch[i * 256] : e[i]) : 0u;
      tot += v[q];
    }
    uint32_t x = tot;  // inclusive scan of the lanes' totals
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t y = (uint32_t)__shfl_up((int)x, o);
      if (lane >= o) x += y;
    }
    uint32_t run = carry + x - tot;
#pragma unroll
    for (int q = 0; q < kScanPer; ++q) {
      if (i0 + q < c1) e[i0 + q] = run;
      run += v[q];
    }
    carry += (uint32_t)__shfl((int)x, 63);
  }
  if (lane == 0) a.eqtot[(int64_t)s * a.K + w] = carry;
}

// the tie-count scan of the workers the guessed pass missed (one wave per (segment, worker)), or of every
// worker in the row-sharded mode
__global__ __launch_bounds__(256) void sa_eqscan_kernel(SegAuction a) {
  if (a.any_miss && !*a.any_miss) return;
  const int64_t hw = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (hw >= (int64_t)a.n_multi * a.K) return;
  const int s = a.mseg[hw / a.K];
  const int w = (int)(hw % a.K);
  if (!(a.flag[s] & kLive)) return;
  if (a.chist && !a.miss[hw]) return;  // scanned by select_guess
  scan_ties(a, s, w, nullptr);
}

// the guessed pass's selection: exact when the (jpw+1)-th largest value lies in last round's bin b1
// (values above b1 < rank <= values at or above b1); otherwise a miss for the two-pass selection
__global__ __launch_bounds__(256) void sa_select_guess_kernel(SegAuction a) {
  const int64_t hw = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (hw >= (int64_t)a.n_multi * a.K) return;
  const int s = a.mseg[hw / a.K];
  const int w = (int)(hw % a.K);
  if (!(a.flag[s] & kLive)) return;
  const int lane = threadIdx.x & 63;
  if (a.lst && !a.lbad[hw]) {  // threshold and bids from its list this round
    if (lane == 0) a.miss[hw] = 0;
    return;
  }
  const uint32_t jpw = (uint32_t)((a.seg_off[s + 1] - a.seg_off[s]) / a.K);
  const uint32_t rank = jpw + 1;
  uint32_t* h = a.hist + hw * 256;
  uint32_t* sel = a.sel + ((int64_t)s * a.K + w) * 4;
  const uint32_t ab = a.above[hw * kAbovePad];
  uint32_t cnt = h[lane] + h[lane + 64] + h[lane + 128] + h[lane + 192];
  for (int o = 32; o > 0; o >>= 1) cnt += (uint32_t)__shfl_xor((int)cnt, o);
  const bool hit = ab < rank && rank <= ab + cnt;
  uint32_t b = 0, above = 0;
  if (hit) wave_select(h, rank - ab, b, above);
  if (lane == 0) {
    if (hit) {
      const uint32_t T = (uint32_t)window_base(sel[2]) + b;
      sel[0] = T >> 8;
      sel[2] = T;
      sel[3] = jpw - (ab + above);
    }
    a.miss[hw] = hit ? 0 : 1;
    if (!hit) {
      *a.any_miss = 1;
      a.live_count[2] = 1;  // a lean block that met a miss is replayed with the exact passes
    }
    a.above[hw * kAbovePad] = 0;
  }
  for (int i = lane; i < 256; i += 64) h[i] = 0;
  // a hit worker's chunk counts of T are its chunk histograms' slot T & 255 = b
  if (hit) scan_ties(a, s, w, a.chist + (int64_t)w * a.total_chunks * 256 + b);
}

// sorted (descending) top 4 of 4 keys; top 4 of two sorted lists: the bitonic half-cleaner max(a_i,
// b_{3-i}) then the 4-element bitonic merge
__device__ __forceinline__ void cas_desc(uint32_t& x, uint32_t& y) {
  const uint32_t hi = max(x, y), lo = min(x, y);
  x = hi;
  y = lo;
}
__device__ __forceinline__ void top4_sort(uint32_t (&k)[4]) {
  cas_desc(k[0], k[1]);
  cas_desc(k[2], k[3]);
  cas_desc(k[0], k[2]);
  cas_desc(k[1], k[3]);
  cas_desc(k[1], k[2]);
}
__device__ __forceinline__ void top4_merge(uint32_t (&k)[4], const uint32_t (&q)[4]) {
#pragma unroll
  for (int i = 0; i < 4; ++i) k[i] = max(k[i], q[3 - i]);
  cas_desc(k[0], k[2]);
  cas_desc(k[1], k[3]);
  cas_desc(k[0], k[1]);
  cas_desc(k[2], k[3]);
}

// one-chunk segments: the selections inside the block; the chunk offset of the tie ranks is 0.  The block
// holds every value of its workers: the guess is the wide segments' window pass on them (kSmallSh > 0: a
// coarse window of 256 slots of 2^kSmallSh keys, then a second in-register pass over the keys of the
// selected slot; measured slower at 3: 0.74 vs 0.55 ms per round of the PROD groups shape, as more values
// fall inside the window).  A worker whose threshold left the window takes the top-4 merge (jpw < 4, the
// PROD groups: a worker's threshold there moves by ~100 keys per round as its few top jobs change owners)
// or both exact histogram passes.
constexpr int kSmallSh = 0;
__global__ __launch_bounds__(256) void sa_small_select_kernel(SegAuction a) {
  const ChunkInfo ci = chunk_info(a, blockIdx.x);
  const uint8_t f = a.flag[ci.s];
  if (!(f & kLive) || !(f & kSingle)) return;
  __shared__ uint2 lbuf[kKG * 256];  // the histograms, or each lane's sorted top 4 keys per worker (u16 x 4)
  uint32_t* const h = reinterpret_cast<uint32_t*>(lbuf);
  static_assert(kKG * kGStride * 4 <= kKG * 256 * 8, "histograms fit the top-4 buffer");
  constexpr int kFine = 1 << kSmallSh;
  __shared__ uint32_t hf[kKG][kFine];
  __shared__ int32_t csl[kKG];
  __shared__ uint32_t b1s[kKG], rk[kKG], ab1[kKG];
  __shared__ uint32_t missm;
  const int w0 = blockIdx.y * kKG, nw = min(kKG, a.K - w0);
  const int64_t sw0 = (int64_t)ci.s * a.K + w0;
  const uint32_t jpw = (uint32_t)(ci.n_s / a.K);
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  for (int i = threadIdx.x; i < kKG * kGStride / 4; i += 256) reinterpret_cast<uint4*>(h)[i] = make_uint4(0, 0, 0, 0);
  if (threadIdx.x < kKG * kFine) (&hf[0][0])[threadIdx.x] = 0;
  if (threadIdx.x == 0) missm = 0;
  int32_t addk[kKG];
  uint32_t negbin = 0;
  bool low = false;
  for (int g = 0; g < kKG; ++g) {
    addk[g] = -0x20000;
    if (g >= nw) continue;
    const int32_t base = window_base<kSmallSh>(a.sel[(sw0 + g) * 4 + 2]);
    if (base >= 0x8000) {
      addk[g] = 0x8000 - base;
    } else {
      addk[g] = 0xFFFF - base;
      negbin |= 1u << g;
      low |= base < 0x400;
    }
  }
  {
    ChunkScores cs;
    load_chunk<false>(a, ci, w0, cs);
    const LaneJobs lj = lane_jobs<false>(ci, cs);
    _Float16 nc[kJPT];
#pragma unroll
    for (int t = 0; t < kJPT; ++t) nc[t] = lj.dead[t] ? (_Float16)-INFINITY : (_Float16)0.0f - lj.c[t];
    __syncthreads();
    if (low) guess_values<true, kSmallSh>(cs, lj, nc, addk, negbin, w0, h);
    else guess_values<false, kSmallSh>(cs, lj, nc, addk, negbin, w0, h);
    __syncthreads();
    // coarse selection: slot c holds the threshold when the window does
    for (int g = wv; g < kKG; g += 4) {
      const uint32_t* hg = h + g * kGStride;
      const uint32_t ab = hg[256], rank = jpw + 1;
      uint32_t cnt = hg[lane] + hg[lane + 64] + hg[lane + 128] + hg[lane + 192];
      for (int o = 32; o > 0; o >>= 1) cnt += (uint32_t)__shfl_xor((int)cnt, o);
      const bool hit = g < nw && ab < rank && rank <= ab + cnt;
      uint32_t c = 0, above = 0;
      if (hit) wave_select(hg, rank - ab, c, above);
      if (lane == 0) {
        csl[g] = hit ? (int32_t)c : 0x7FFFFFFF;  // a missed worker counts nothing in the fine pass
        rk[g] = rank - ab - above;
        ab1[g] = ab + above;
        if (g < nw && !hit) atomicOr(&missm, 1u << g);
      }
    }
    if constexpr (kSmallSh > 0) {
      __syncthreads();
      int32_t cs_l[kKG];
#pragma unroll
      for (int g = 0; g < kKG; ++g) cs_l[g] = csl[g];
      if (low) guess_values<true, kSmallSh, true>(cs, lj, nc, addk, negbin, w0, &hf[0][0], cs_l, kFine);
      else guess_values<false, kSmallSh, true>(cs, lj, nc, addk, negbin, w0, &hf[0][0], cs_l, kFine);
    }
  }
  __syncthreads();
  {  // fine selection, one thread per hit worker
    const int g = threadIdx.x;
    if (g < nw && !((missm >> g) & 1u)) {
      uint32_t acc = 0;
      int q = kFine - 1;
      if constexpr (kSmallSh > 0) {
        for (; q > 0; --q) {
          if (acc + hf[g][q] >= rk[g]) break;
          acc += hf[g][q];
        }
      }
      uint32_t* sel = a.sel + (sw0 + g) * 4;
      const uint32_t T = (uint32_t)(window_base<kSmallSh>(sel[2]) + (csl[g] << kSmallSh) + q);
      sel[0] = T >> 8;
      sel[2] = T;
      sel[3] = jpw - (ab1[g] + acc);
    }
  }
  __syncthreads();
  const uint32_t miss = missm;
  if (!miss) return;  // block-uniform
  if (jpw < 4) {
    // the last layer's groups (jpw = 2 at PROD): T is the (jpw+1)-th largest key, found by merging each
    // lane's sorted top 4 across the wave and then the block (no histogram: a worker's values crowd into
    // a few high-byte bins, where LDS atomics serialise)
    __shared__ uint4 top[kKG][4];
    {
      ChunkScores cr;  // the chunk again (L2), all loads in flight at once
      int wl = w0;
      asm volatile("" : "+s"(wl));  // new addresses: CSE with the first pass's would keep them live throughout
      load_chunk<false>(a, ci, wl, cr);
      const LaneJobs lj = lane_jobs<false>(ci, cr);
#pragma unroll
      for (int g = 0; g < kKG; ++g) {
        uint32_t k[4];
#pragma unroll
        for (int t = 0; t < kJPT; ++t) {
          // + 0: okey needs one zero; a lane past the end (cost NaN) takes key 0, below every real key
          const _Float16 x = lane_value(w0 + g, cr.v[t][g], lj.hb[t], lj.c[t]) + (_Float16)0.0f;
          k[t] = lj.dead[t] ? 0u : okey(__builtin_bit_cast(uint16_t, x));
        }
        top4_sort(k);
        lbuf[g * 256 + threadIdx.x] = make_uint2(k[0] | (k[1] << 16), k[2] | (k[3] << 16));
      }
    }
    for (uint32_t m = miss; m; m &= m - 1u) {
      const int g = __builtin_ctz(m);
      const uint2 p = lbuf[g * 256 + threadIdx.x];
      uint32_t k[4] = {p.x & 0xFFFFu, p.x >> 16, p.y & 0xFFFFu, p.y >> 16};
      for (int o = 1; o < 64; o <<= 1) {
        uint32_t q[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) q[i] = (uint32_t)__shfl_xor((int)k[i], o);
        top4_merge(k, q);
      }
      if (lane == 0) top[g][wv] = make_uint4(k[0], k[1], k[2], k[3]);
    }
    __syncthreads();
    const int g = threadIdx.x;
    if (g < kKG && ((miss >> g) & 1u)) {
      uint32_t k[4] = {top[g][0].x, top[g][0].y, top[g][0].z, top[g][0].w};
      for (int q = 1; q < 4; ++q) {
        uint32_t o[4] = {top[g][q].x, top[g][q].y, top[g][q].z, top[g][q].w};
        top4_merge(k, o);
      }
      const uint32_t T = k[jpw];
      uint32_t gt = 0;
      for (uint32_t i = 0; i < jpw; ++i) gt += k[i] > T;
      uint32_t* sel = a.sel + (sw0 + g) * 4;
      sel[0] = T >> 8;
      sel[2] = T;
      sel[3] = jpw - gt;
    }
    return;
  }
  for (int pass = 0; pass < 2; ++pass) {
    for (int i = threadIdx.x; i < kKG * kGStride; i += 256) h[i] = 0;
    __syncthreads();
    for (int t = 0; t < kJPT; ++t) {
      const int64_t jj = t * 256 + threadIdx.x;
      if (jj >= ci.nj) break;
      const int64_t j = ci.j0 + jj;
      const int32_t hbj = a.hb[j];
      const uint16_t cj = a.cost[j];
      uint16_t v[kKG];
#pragma unroll
      for (int g = 0; g < kKG; ++g) v[g] = ((miss >> g) & 1u) ? wrow(a, ci, w0 + g)[j] : 0;
#pragma unroll
      for (int g = 0; g < kKG; ++g) {
        if (!((miss >> g) & 1u)) continue;
        const uint32_t k = okey(value_bits(w0 + g, v[g], hbj, cj));
        if (pass == 0) atomicAdd(&h[g * kGStride + (k >> 8)], 1u);
        else if ((k >> 8) == b1s[g]) atomicAdd(&h[g * kGStride + (k & 255)], 1u);
      }
    }
    __syncthreads();
    for (int g = wv; g < nw; g += 4) {
      if (!((miss >> g) & 1u)) continue;
      uint32_t b, above;
      const uint32_t rank = pass == 0 ? jpw + 1 : rk[g];
      wave_select(h + g * kGStride, rank, b, above);
      if (lane == 0) {
        if (pass == 0) {
          b1s[g] = b;
          rk[g] = rank - above;
          ab1[g] = above;
        } else {
          uint32_t* sel = a.sel + (sw0 + g) * 4;
          const uint32_t T = (b1s[g] << 8) | b;
          sel[0] = b1s[g];
          sel[2] = T;
          sel[3] = jpw - (ab1[g] + above);
        }
      }
    }
    __syncthreads();
  }
}

// ---- tie counts (multi-chunk segments) ----
template <bool VEC>
__global__ __launch_bounds__(256) void sa_eqcount_kernel(SegAuction a) {
  if (a.any_miss && !*a.any_miss) return;
  const ChunkInfo ci = chunk_info(a, blockIdx.x);
  const uint8_t f = a.flag[ci.s];
  if (!(f & kLive) || (f & kSingle)) return;
  __shared__ uint32_t c[kKG];
  const int w0 = blockIdx.y * kKG, nw = min(kKG, a.K - w0);
  const int64_t sw0 = (int64_t)ci.s * a.K + w0;
  uint32_t part = (1u << nw) - 1u;  // workers whose counts this pass produces
  if (a.chist) {  // hit workers' counts come from the guessed pass's chunk histograms (select_guess)
    const int64_t hw0 = (int64_t)a.hidx[ci.s] * a.K + w0;
    part = 0;
    for (int g = 0; g < nw; ++g) part |= (uint32_t)(a.miss[hw0 + g] != 0) << g;
    if (!part) return;
  }
  if (threadIdx.x < kKG) c[threadIdx.x] = 0;
  __syncthreads();
  _Float16 vT[kKG];
  for (int g = 0; g < kKG; ++g)
    vT[g] = __builtin_bit_cast(_Float16, g < nw ? okey_inv(a.sel[(sw0 + g) * 4 + 2]) : (uint16_t)0);
  uint32_t cnt[kKG] = {};
  ChunkScores cs;
  load_chunk<VEC>(a, ci, w0, cs);
#pragma unroll
  for (int t = 0; t < kJPT; ++t) {
    const bool live = job_of<VEC>(t) < ci.nj;
#pragma unroll
    for (int g = 0; g < kKG; ++g)
      if (g < nw) cnt[g] += live && value_h(w0 + g, cs.v[t][g], cs.hb[t], cs.c[t]) == vT[g];
  }
  for (int g = 0; g < nw; ++g) {
    uint32_t v = cnt[g];
    for (int o = 32; o > 0; o >>= 1) v += (uint32_t)__shfl_xor((int)v, o);
    if ((threadIdx.x & 63) == 0 && v) atomicAdd(&c[g], v);
  }
  __syncthreads();
  if (threadIdx.x < nw && ((part >> threadIdx.x) & 1u))
    a.eqcnt[(int64_t)(w0 + threadIdx.x) * a.total_chunks + blockIdx.x] = c[threadIdx.x];
}

// ---- resolve one chunk: winners, costs and the count of jobs with a bidder; every load issued before any
// store.  (A bid kernel whose last block per chunk resolved it measured 17x slower: the cross-block
// handoff needs device-scope fences, an L2 writeback per block on the XCD-split L2.) ----
// (live: the segment's flag, loaded by the caller and tested here, after the chunk's loads are issued)
__device__ __forceinline__ void resolve_chunk(const SegAuction& a, const ChunkInfo& ci, int32_t* __restrict__ out,
                                              const uint8_t* live = nullptr) {
  const uint8_t fl = live ? *live : kLive;
  const int counter = a.lst ? *a.round_dev : 0;
  uint32_t k[kJPT];
  uint16_t c[kJPT];
#pragma unroll
  for (int t = 0; t < kJPT; ++t) {
    const int64_t j = ci.j0 + min((int64_t)(t * 256 + threadIdx.x), ci.nj - 1);
    k[t] = a.key[j];
    c[t] = a.cost[j];
  }
  if (!(fl & kLive)) return;
  if (a.lst) {  // list mode: the retention / leftover bids of pairs no list held (the sweep's overrides)
    const uint32_t ek = (uint32_t)a.eps[ci.s] << 16;
    if (counter < 100 || counter > 1000) {
#pragma unroll
      for (int t = 0; t < kJPT; ++t) {
        const int64_t j = ci.j0 + min((int64_t)(t * 256 + threadIdx.x), ci.nj - 1);
        const int32_t hbj = a.hb[j];
        if (counter < 100 && hbj >= 0) k[t] = max(k[t], ek | (0xFFFFu - (uint32_t)hbj));
        if (counter > 1000 && a.nobid[j]) k[t] = max(k[t], ek | 0xFFFFu);
      }
    }
  }
  uint32_t cnt = 0;
#pragma unroll
  for (int t = 0; t < kJPT; ++t) {
    if (t * 256 + (int64_t)threadIdx.x >= ci.nj) break;
    const int64_t j = ci.j0 + t * 256 + threadIdx.x;
    a.key[j] = 0;
    if (k[t]) {
      const int32_t w = (int32_t)(0xFFFFu - (k[t] & 0xFFFFu));
      const uint16_t bid = (uint16_t)(k[t] >> 16);
      out[j] = w;
      a.hb[j] = w;
      a.nobid[j] = 0;
      const uint16_t cn = f2h(h2f(c[t]) + h2f(bid));
      a.cost[j] = cn;
      if (a.js) a.js[j] = ((uint32_t)w << 16) | cn;
      ++cnt;
    } else {
      out[j] = -1;
      a.hb[j] = -1;
      a.nobid[j] = 1;
      if (a.js) a.js[j] = 0xFFFF0000u | c[t];
    }
  }
  // one same-address atomic per block, not per wave: a segment's chunks all count into have[s]
  __shared__ uint32_t wc[4];
  for (int o = 32; o > 0; o >>= 1) cnt += (uint32_t)__shfl_xor((int)cnt, o);
  if ((threadIdx.x & 63) == 0) wc[threadIdx.x >> 6] = cnt;
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint32_t tot = wc[0] + wc[1] + wc[2] + wc[3];
    if (a.rdone) {
      // one 64-bit atomic carries both the arrival and the count, so the last block to arrive sees every
      // other block's count in the value it gets back (no fence between two atomics needed).  Two levels:
      // block b arrives at counter 1 + b % kRd, the last of those at counter 0 (same-address atomics
      // serialise at ~12 ns each: 977 blocks of a 1M-job auction on one word cost 12 us per round)
      const uint32_t G = gridDim.x, sub = blockIdx.x % kRd;
      const uint32_t nsub = (G - sub + kRd - 1) / kRd, ntop = min(G, (uint32_t)kRd);
      unsigned long long* const c1 = a.rdone + 16 * (1 + sub);  // (one 128-B line per counter)
      const unsigned long long o1 = atomicAdd(c1, (1ull << 32) | tot);
      if ((o1 >> 32) != (unsigned long long)(nsub - 1)) return;
      atomicExch(c1, 0ull);
      const uint32_t part = (uint32_t)o1 + tot;
      const unsigned long long old = atomicAdd(a.rdone, (1ull << 32) | part);
      if ((old >> 32) == (unsigned long long)(ntop - 1)) {
        const uint32_t have = (uint32_t)old + part;
        *a.round_dev += 1;
        if (a.any_miss) *a.any_miss = 0;
        if (a.lany) *a.lany = 0;
        a.rounds[0] += 1;
        const bool live = (int64_t)have != (int64_t)(a.seg_off[1] - a.seg_off[0]);
        if (!live) a.flag[0] &= ~kLive;
        atomicExch(a.rdone, 0ull);
        if (a.rcount && live) atomicAdd(a.live_count, 1u);
      }
    } else if (tot) {
      atomicAdd(&a.have[ci.s], tot);
    }
  }
}

// ---- bids: one packed {fp16 bid, ~worker} atomicMax per job and block ----
// A worker bids on its values above T and on the first `need` of its values equal to T in job order.  The
// tie offsets (eqcnt: equal values in the segment's earlier chunks; eqtot: the segment's total) put each
// chunk of a worker in one of three cases: no equal value bids (need <= offset), every equal value bids
// (need >= offset + the chunk's count: the test becomes x >= T, i.e. x > below(T), whose bid (x - T) + eps
// is eps at equality, the deferred bid's key), or the chunk straddles the boundary and its equal values
// need their ranks: one chunk per worker and round of a wide segment, every chunk of a one-chunk segment.
// Only blocks with a straddling worker re-read their chunk (L2) for its equal values and rank them (phase B).
// Phase A is branch-free per value (RET: the retention rounds, where the previous winner bids eps): a bid
// key or a bid-less key (< 2^16) is max-ed into each job slice.  A ranked equal value of an overridden job
// (retention / leftover) is harmless: its phase-B bid is the same eps key.
template <bool RET>
__device__ __forceinline__ void bid_values(const ChunkScores& cs, const LaneJobs& lj, const bool (&nob)[kJPT],
                                           const _Float16 (&vT)[kKG], const _Float16 (&vC)[kKG], int w0,
                                           _Float16 epsh, uint32_t (&best)[kJPT]) {
  const uint32_t eps = __builtin_bit_cast(uint16_t, epsh);
#pragma unroll
  for (int t = 0; t < kJPT; ++t) {
#pragma unroll
    for (int g = 0; g < kKG; ++g) {
      const int w = w0 + g;
      const bool own = lj.hb[t] == w;
      const _Float16 x = __builtin_bit_cast(_Float16, cs.v[t][g]) - (own ? (_Float16)-0.0f : lj.c[t]);
      uint32_t bid = x > vC[g] ? (uint32_t)__builtin_bit_cast(uint16_t, (_Float16)((_Float16)(x - vT[g]) + epsh)) : 0u;
      if (RET) bid = own ? eps : bid;
      if (g == 0) bid = nob[t] ? eps : bid;
      best[t] = max(best[t], (bid << 16) | (0xFFFFu - (uint32_t)w));
    }
  }
}

// the straddling workers' values equal to T: bit (t & 1) * kKG + g of eqs[t >> 1]
__device__ __forceinline__ void equal_values(const ChunkScores& cs, const LaneJobs& lj, const _Float16 (&vT)[kKG],
                                             uint32_t straddle, int w0, uint32_t (&eqs)[2]) {
#pragma unroll
  for (int g = 0; g < kKG; ++g) {
    if (!((straddle >> g) & 1u)) continue;
#pragma unroll
    for (int t = 0; t < kJPT; ++t) {
      const _Float16 x = __builtin_bit_cast(_Float16, cs.v[t][g]) - (lj.hb[t] == w0 + g ? (_Float16)-0.0f : lj.c[t]);
      eqs[t >> 1] |= x == vT[g] ? 1u << ((t & 1) * kKG + g) : 0u;
    }
  }
}

// the largest fp16 value below the one of key k (k of a finite value; +0's predecessor is -min_subnormal)
__device__ __forceinline__ _Float16 value_below(uint32_t k) {
  const uint32_t p = k - 1u == 0x7FFFu ? 0x7FFEu : k - 1u;
  return __builtin_bit_cast(_Float16, okey_inv(p));
}

__device__ __forceinline__ uint32_t lanes_below(unsigned long long m) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// RQ_BID_WAVES: occupancy floor for the bid kernel (0 = the compiler's choice: 103 VGPRs, 4 waves/SIMD, 1.6x
// slower at K=128 x 1M; 5 keeps both forms spill-free, A/B in profiles/r3_auction_ab_waves.txt)
#ifndef RQ_BID_WAVES
#define RQ_BID_WAVES 5
#endif
#if RQ_BID_WAVES
#define RQ_BID_ATTR __attribute__((amdgpu_waves_per_eu(RQ_BID_WAVES)))
#else
#define RQ_BID_ATTR
#endif
template <bool VEC>
__global__ __launch_bounds__(256) RQ_BID_ATTR void sa_bid_kernel(SegAuction a) {
  if (a.lany && a.n_multi == a.S && !*a.lany) return;  // every list held (one-chunk segments have none)
  const int counter = *a.round_dev;
  const ChunkInfo ci = chunk_info(a, blockIdx.x);
  const uint8_t f = a.flag[ci.s];
  if (!(f & kLive)) return;
  if (a.lst && !(f & kSingle)) {  // the list pass bids for workers whose lists hold every bidding value
    const int64_t hwb = (int64_t)a.hidx[ci.s] * a.K + blockIdx.y * kKG;
    const int nwb = min(kKG, a.K - (int)blockIdx.y * kKG);
    bool bad = false;
    for (int g = 0; g < nwb; ++g) bad |= a.lbad[hwb + g] != 0;
    if (!bad) return;  // (in a block with a bad worker the listed workers bid nothing but retention keys)
  }
  __shared__ uint4 eqc[kKG][4];  // per (worker, wave): values equal to T in each job slice
  __shared__ uint32_t gneed[kKG], goff[kKG];
  const int w0 = blockIdx.y * kKG, nw = min(kKG, a.K - w0);
  const int64_t sw0 = (int64_t)ci.s * a.K + w0;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const uint16_t eps = a.eps[ci.s];
  const _Float16 epsh = __builtin_bit_cast(_Float16, eps);
  const bool single = f & kSingle;
  const int64_t c = blockIdx.x, c_last = a.chunk_off[ci.s + 1] - 1;
  _Float16 vT[kKG], vC[kKG];  // T and the comparison bound; NaN for workers past K (nothing bids)
  uint32_t need[kKG], off[kKG];
  uint32_t straddle = 0;
  const bool listed = a.lst && !single;
  for (int g = 0; g < kKG; ++g) {
    vT[g] = vC[g] = __builtin_bit_cast(_Float16, (uint16_t)0x7E00u);
    need[g] = off[g] = 0;
    if (g >= nw) continue;
    if (listed && !a.lbad[(int64_t)a.hidx[ci.s] * a.K + w0 + g]) continue;  // bids from its list (NaN: none here)
    const uint32_t kT = a.sel[(sw0 + g) * 4 + 2];
    need[g] = a.sel[(sw0 + g) * 4 + 3];
    vT[g] = vC[g] = __builtin_bit_cast(_Float16, okey_inv(kT));
    if (single) {  // need < the segment's equal values: all-or-none only at need == 0
      if (need[g]) straddle |= 1u << g;
      continue;
    }
    const uint32_t* e = a.eqcnt + (int64_t)(w0 + g) * a.total_chunks;
    const uint32_t lo = e[c], n = (c < c_last ? e[c + 1] : a.eqtot[sw0 + g]) - lo;
    off[g] = lo + (a.rank_off ? a.rank_off[w0 + g] : 0u);
    if (need[g] >= off[g] + n) vC[g] = value_below(kT);
    else if (need[g] > off[g]) straddle |= 1u << g;
  }
  const bool leftover = counter > 1000 && w0 == 0;   // leftovers go to worker 0
  ChunkScores cs;
  load_chunk<VEC>(a, ci, w0, cs);
  const LaneJobs lj = lane_jobs<VEC>(ci, cs);
  bool nob[kJPT];
#pragma unroll
  for (int t = 0; t < kJPT; ++t) nob[t] = leftover && job_of<VEC>(t) < ci.nj && a.nobid[ci.j0 + job_of<VEC>(t)];
  uint32_t best[kJPT] = {};
  if (counter < 100) bid_values<true>(cs, lj, nob, vT, vC, w0, epsh, best);
  else bid_values<false>(cs, lj, nob, vT, vC, w0, epsh, best);
  if (straddle) {  // block-uniform: phase B's barrier is reached by every wave
    ChunkScores cr;  // the chunk again (L2-resident), so phase A keeps no values alive for this rare path
    int wl = w0;
    asm volatile("" : "+s"(wl));  // new addresses: CSE with phase A's would keep them live throughout
    load_chunk<VEC>(a, ci, wl, cr);
    uint32_t eqs[2] = {};
    equal_values(cr, lj, vT, straddle, w0, eqs);
    // straddling workers with an equal value in this wave (OR over the lanes); loops over worker bits
    // with the worker's need and offset from LDS keep the rare path's registers out of phase A's budget
    uint32_t any = eqs[0] | eqs[1];
    for (int o = 32; o > 0; o >>= 1) any |= (uint32_t)__shfl_xor((int)any, o);
    const uint32_t weq = (uint32_t)__builtin_amdgcn_readfirstlane((int)((any | (any >> kKG)) & straddle));
    if (threadIdx.x == 0) {
      for (int g = 0; g < kKG; ++g) {
        gneed[g] = need[g];
        goff[g] = off[g];
      }
    }
    for (uint32_t m = straddle; m; m &= m - 1u) {
      const int g = __builtin_ctz(m);
      uint32_t n[kJPT] = {};
      if ((weq >> g) & 1u) {
#pragma unroll
        for (int t = 0; t < kJPT; ++t) n[t] = (uint32_t)__popcll(__ballot((eqs[t >> 1] >> ((t & 1) * kKG + g)) & 1u));
      }
      if (lane == 0) eqc[g][wv] = make_uint4(n[0], n[1], n[2], n[3]);
    }
    __syncthreads();
    for (uint32_t m = weq; m; m &= m - 1u) {
      const int g = __builtin_ctz(m);
      const uint32_t wbid = ((uint32_t)eps << 16) | (0xFFFFu - (uint32_t)(w0 + g));
      const uint32_t ng = gneed[g];
      const uint4 q0 = eqc[g][0], q1 = eqc[g][1], q2 = eqc[g][2], q3 = eqc[g][3];
      const uint32_t n0[kJPT] = {q0.x, q0.y, q0.z, q0.w}, n1[kJPT] = {q1.x, q1.y, q1.z, q1.w},
                     n2[kJPT] = {q2.x, q2.y, q2.z, q2.w}, n3[kJPT] = {q3.x, q3.y, q3.z, q3.w};
      bool e[kJPT];
#pragma unroll
      for (int t = 0; t < kJPT; ++t) e[t] = (eqs[t >> 1] >> ((t & 1) * kKG + g)) & 1u;
      if (VEC) {
        // job order: earlier waves (all slices), lower lanes (all slices), this lane's earlier slices
        uint32_t before = goff[g];
#pragma unroll
        for (int t = 0; t < kJPT; ++t)
          before += (wv > 0 ? n0[t] : 0u) + (wv > 1 ? n1[t] : 0u) + (wv > 2 ? n2[t] : 0u) + lanes_below(__ballot(e[t]));
#pragma unroll
        for (int t = 0; t < kJPT; ++t) {
          if (e[t] && before < ng) best[t] = max(best[t], wbid);
          before += e[t];
        }
      } else {
        // job order: slice-major, then waves, then lanes
        uint32_t run = goff[g];
#pragma unroll
        for (int t = 0; t < kJPT; ++t) {
          const uint32_t r = run + (wv > 0 ? n0[t] : 0u) + (wv > 1 ? n1[t] : 0u) + (wv > 2 ? n2[t] : 0u) +
                             lanes_below(__ballot(e[t]));
          if (e[t] && r < ng) best[t] = max(best[t], wbid);
          run += n0[t] + n1[t] + n2[t] + n3[t];
        }
      }
    }
  }
#pragma unroll
  for (int t = 0; t < kJPT; ++t)
    if (best[t] >> 16) atomicMax(&a.key[ci.j0 + job_of<VEC>(t)], best[t]);
}

// ---- list rounds ---------------------------------------------------------------------------------------
// A round of a wide segment sweeps W twice (guessed pass, bids), although a worker's threshold T (its
// (jpw+1)-th largest value) barely moves between rounds (median 0 keys, 99th percentile ~22 keys in an
// oracle simulation of the candidate-fit shape).  So a sweep round also records, per worker, every job whose
// value key is >= lkb = T_prev - kListDelta (with its raw score), and the following rounds run from that
// list alone.  Values only fall between rounds (costs only rise), except that the previous winner's value is
// its raw score; a worker wins a job only by bidding on it, i.e. from a listed value (or in a sweep round,
// after which T >= lkb is checked).  So while a list round's threshold stays >= lkb (>= jpw + 1 listed values
// at or above lkb), the list holds every value >= T and the round's selection, tie ranks and bids are the
// sweep's exactly.  The leftover rounds (> 1000: worker 0 bids on jobs without a bidder, unlisted pairs)
// sweep.  A worker whose list fails (none yet, T_prev < lkb, too few values, too many ties, overflow) takes
// the sweep path this round (lbad = 1), which rebuilds its list.
// One block per (segment, worker): values recomputed from raw score, cost and winner; the two-byte radix
// select of the keys >= lkb; the jobs of the values equal to T sorted in LDS (their first `need` in job order
// bid eps); bids, retention / leftover overrides and the packed atomicMax of the sweep.
constexpr int kListEq = 2048;  // values equal to T a list round ranks in LDS (more: sweep)
constexpr int kLT = 1024;  // threads of a list-round block
// LT threads per block: 1024, or 256 when every list is short (the middle layer's lockstep sub-fits: 128
// segments x 128 workers, lists of ~500 entries, 16384 blocks per round)
// Lists of at most kLE * LT entries stay in registers from the first load (entry tid + q * LT in er[q]): the
// later passes read no list memory, and the first load is issued before the block's validity checks.
constexpr int kLE = 4;
template <int LT>
__global__ __launch_bounds__(LT) void sa_list_round_kernel(SegAuction a) {
  const int64_t hw = blockIdx.x;
  const int r = (int)(hw / a.K), w = (int)(hw % a.K);
  const bool one = a.one_n > 0;  // (then n_multi == 1: r == 0, segment 0)
  const int sg = one ? 0 : a.mseg[r];
  const uint32_t cap = one ? (uint32_t)(4 * (a.one_n / a.K) + 256) : (uint32_t)a.lcs[r];
  uint2* const L = a.lst + (one ? 0 : a.loff[r]) + (int64_t)w * cap;
  const int tid = threadIdx.x;
  const bool regs = cap <= (uint32_t)(kLE * LT);
  // the block's state words and (register lists) the entries, all issued before any test: one round trip
  const int64_t sw = (int64_t)sg * a.K + w;
  const uint8_t sflag = a.flag[sg];
  const int counter = *a.round_dev;
  const uint32_t n = a.lcnt[hw * kAbovePad];
  const uint32_t kb = a.lkb[hw];
  const uint32_t tprev = a.sel[sw * 4 + 2];
  uint2 er[kLE];
  if (regs) {
#pragma unroll
    for (int q = 0; q < kLE; ++q) {
      const uint32_t i = tid + q * LT;
      er[q] = i < cap ? L[i] : make_uint2(0u, 0u);  // (in the worker's list area whatever n is)
    }
  }
  if (!(sflag & kLive)) return;
  __shared__ uint32_t hst[256];
  __shared__ uint32_t sh[4];  // bin, above, T, need | radix-select bin and rank
  const uint32_t jpw = (uint32_t)((one ? a.one_n : (int64_t)(a.seg_off[sg + 1] - a.seg_off[sg])) / a.K);
  // every list entry i < n with its 64-bit word, from registers or from the list
  auto visit = [&](auto&& f) __attribute__((always_inline)) {
    if (regs) {
#pragma unroll
      for (int q = 0; q < kLE; ++q) {
        const uint32_t i = tid + q * LT;
        if (i < n) f(er[q], i);
      }
    } else {
      for (uint32_t i = tid; i < n; i += LT) {
        uint2 e = L[i];
        f(e, i);
      }
    }
  };
  auto fail_list = [&]() {
    if (tid == 0) {
      a.lbad[hw] = 1;
      *a.lany = 1;
      a.live_count[3] = 1;
      a.lcnt[hw * kAbovePad] = 0;  // the sweep's guessed pass rebuilds it
    }
  };
  if (n == 0 || n > cap || counter > 1000 || tprev < kb) {
    if (tid == 0) list_stat(a, list_fail_why(n, cap, counter));
    return fail_list();
  }
  AST(const uint64_t s0 = ANOW(); uint64_t s1 = 0, s2 = 0, s3 = 0;)
  if (tid < 256) hst[tid] = 0;
  __syncthreads();
  // pass 1: this round's value keys (raw score, cost, last winner), kept in the entries' upper 16 bits so
  // the later passes read the list only
  visit([&](uint2& e, uint32_t i) {
    const int32_t hbj = js_hb(a, e.x);
    const uint32_t k = okey(value_bits(w, (uint16_t)e.y, hbj, js_cost(a, e.x)));
    e.y = (e.y & 0xFFFFu) | (k << 16);
    if (!regs) L[i].y = e.y;
    else if (hbj == w) e.x |= 0x80000000u;  // (register copy only: the retention test of the bid pass)
    if (k >= kb) atomicAdd(&hst[k >> 8], 1u);
  });
  __syncthreads();
  if (tid < 64) {
    uint32_t tot = hst[4 * tid] + hst[4 * tid + 1] + hst[4 * tid + 2] + hst[4 * tid + 3];
    for (int o = 32; o > 0; o >>= 1) tot += (uint32_t)__shfl_xor((int)tot, o);
    uint32_t b = 0, above = 0;
    if (tot >= jpw + 1) wave_select(hst, jpw + 1, b, above);
    if (tid == 0) {
      sh[0] = tot >= jpw + 1 ? b : 0xFFFFFFFFu;
      sh[1] = above;
    }
  }
  __syncthreads();
  const uint32_t b1 = sh[0];
  AST(s1 = ANOW();)
  if (b1 == 0xFFFFFFFFu) {  // fewer than jpw + 1 values at or above the list base
    if (tid == 0) list_stat(a, 5);
    return fail_list();
  }
  __syncthreads();
  if (tid < 256) hst[tid] = 0;
  __syncthreads();
  visit([&](uint2& e, uint32_t) {
    const uint32_t k = e.y >> 16;
    if (k >= kb && (k >> 8) == b1) atomicAdd(&hst[k & 255u], 1u);
  });
  __syncthreads();
  if (tid < 64) {
    uint32_t b = 0, above = 0;
    wave_select(hst, jpw + 1 - sh[1], b, above);
    if (tid == 0) {
      const uint32_t T = (b1 << 8) | b;
      sh[2] = T;
      sh[3] = jpw - (sh[1] + above);  // need: equal values that bid
      sh[0] = 0;                      // equal values found (next pass)
    }
  }
  __syncthreads();
  const uint32_t T = sh[2], need = sh[3];
  AST(s2 = ANOW();)
  if (T < kb) return fail_list();  // (cannot happen with >= jpw + 1 values >= kb; kept as a guard)
  // the first `need` of the values equal to T in job order bid: J = the need-th smallest job index among
  // them, by a radix select over the index bytes (no sort, no bound on the number of equal values: fp16
  // half scores put thousands of a worker's jobs on one value)
  uint32_t J = 0;
  if (need) {
    uint32_t rank = need;
    for (int shift = 24; shift >= 0; shift -= 8) {
      __syncthreads();
      if (tid < 256) hst[tid] = 0;
      __syncthreads();
      visit([&](uint2& e, uint32_t) {
        const uint32_t j = e.x & 0x7FFFFFFFu;
        if ((e.y >> 16) == T && (shift == 24 || (j >> (shift + 8)) == J))
          atomicAdd(&hst[(j >> shift) & 255u], 1u);
      });
      __syncthreads();
      if (tid < 64) {  // ascending walk: the bin holding the rank-th smallest
        const uint32_t h0 = hst[4 * tid], h1 = hst[4 * tid + 1], h2 = hst[4 * tid + 2], h3 = hst[4 * tid + 3];
        const uint32_t own = h0 + h1 + h2 + h3;
        uint32_t inc = own;  // inclusive prefix over lanes <= tid
        for (int o = 1; o < 64; o <<= 1) {
          const uint32_t y = (uint32_t)__shfl_up((int)inc, o);
          if (tid >= o) inc += y;
        }
        const unsigned long long m = __ballot(inc >= rank);
        const int Ln = m ? __ffsll((long long)m) - 1 : 63;
        if (tid == Ln) {
          uint32_t acc = inc - own;  // strictly below this lane's bins
          const uint32_t hv[4] = {h0, h1, h2, h3};
          int q = 0;
          for (; q < 3; ++q) {
            if (acc + hv[q] >= rank) break;
            acc += hv[q];
          }
          sh[0] = (uint32_t)(4 * Ln + q);
          sh[1] = rank - acc;
        }
      }
      __syncthreads();
      J = (J << 8) | sh[0];
      rank = sh[1];
    }
  }
  AST(s3 = ANOW();)
  const uint16_t eps = a.eps[sg];
  const _Float16 epsh = __builtin_bit_cast(_Float16, eps);
  const _Float16 vT = __builtin_bit_cast(_Float16, okey_inv(T));
  const bool ret = counter < 100;
  visit([&](uint2& e, uint32_t) {
    const uint32_t j = e.x & 0x7FFFFFFFu, k = e.y >> 16;
    uint32_t bid = 0;
    if (k > T) {
      const _Float16 x = __builtin_bit_cast(_Float16, okey_inv(k));
      bid = __builtin_bit_cast(uint16_t, (_Float16)((_Float16)(x - vT) + epsh));
    } else if (k == T && need && j <= J) {
      bid = eps;
    }
    if (ret && (regs ? (e.x >> 31) != 0u : js_hb(a, j) == w)) bid = eps;  // retention: the previous winner bids eps
    if (bid) atomicMax(&a.key[j], (bid << 16) | (0xFFFFu - (uint32_t)w));
  });
  AST(__syncthreads();)
  if (tid == 0) {
    uint32_t* sel = a.sel + sw * 4;
    sel[0] = T >> 8;
    sel[1] = 0;
    sel[2] = T;
    sel[3] = need;
    a.lbad[hw] = 0;
    list_stat(a, 0);
#ifdef RQSID_STAMPS
    const uint64_t s4 = ANOW();
    atomicAdd(&g_al_stamps[0], (unsigned long long)(s1 - s0));
    atomicAdd(&g_al_stamps[1], (unsigned long long)(s2 - s1));
    atomicAdd(&g_al_stamps[2], (unsigned long long)(s3 - s2));
    atomicAdd(&g_al_stamps[3], (unsigned long long)(s4 - s3));
    atomicAdd(&g_al_stamps[4], 1ull);
    atomicAdd(&g_al_stamps[5], need ? 1ull : 0ull);
    atomicAdd(&g_al_stamps[6], (unsigned long long)n);
#endif
  }
}

// ---- multi-block list rounds: sa_list_round_kernel's steps for long lists (one wide segment), each a grid
// over (worker, chunk of kMCH entries) or one block per worker, so a round of a K=128 x 10M auction is not
// 128 blocks walking ~230k entries each.  Same values, selection, tie ranks and bids; a worker whose list
// fails in any step (lok = 0, lbad = 1) takes the sweep path of the same round before any of its bids.
__device__ __forceinline__ void mlist_fail(const SegAuction& a, int64_t hw) {
  a.lok[hw] = 0;
  a.lbad[hw] = 1;
  *a.lany = 1;
  a.live_count[3] = 1;
  a.lcnt[hw * kAbovePad] = 0;  // the sweep's guessed pass rebuilds it
}

// validity (as sa_list_round_kernel's first test) and zeroed histograms; one block per worker
__global__ __launch_bounds__(256) void sa_mlist_init_kernel(SegAuction a) {
  const int64_t hw = blockIdx.x;
  const int r = (int)(hw / a.K), w = (int)(hw % a.K);
  const int sg = a.mseg[r];
  const int tid = threadIdx.x;
  if (!(a.flag[sg] & kLive)) {
    if (tid == 0) a.lok[hw] = 0;
    return;
  }
  a.lh[hw * 512 + tid] = 0;
  a.lh[hw * 512 + 256 + tid] = 0;
  if (tid == 0) {
    const uint32_t n = a.lcnt[hw * kAbovePad], cap = (uint32_t)a.lcs[r], kb = a.lkb[hw];
    const int counter = *a.round_dev;
    const int64_t sw = (int64_t)sg * a.K + w;
    a.leqn[hw] = 0;
    if (n == 0 || n > cap || counter > 1000 || a.sel[sw * 4 + 2] < kb) {
      list_stat(a, list_fail_why(n, cap, counter));
      mlist_fail(a, hw);
    } else {
      a.lok[hw] = 1;
    }
  }
}

// STEP 0: this round's keys (kept in the entries' upper 16 bits) and the high-byte histogram of the keys
// >= lkb; 1: the low-byte histogram of bin b1; 2: the jobs of the values equal to T (when some of them bid);
// 3: the bids.  Grid: workers x lmb_chunks blocks.
template <int STEP>
__global__ __launch_bounds__(256) void sa_mlist_pass_kernel(SegAuction a) {
  const int64_t hw = blockIdx.x / a.lmb_chunks;
  const uint32_t i0 = (uint32_t)(blockIdx.x % a.lmb_chunks) * kMCH;
  if (!a.lok[hw]) return;
  const uint32_t n = a.lcnt[hw * kAbovePad];
  if (i0 >= n) return;
  const uint32_t i1 = min(n, i0 + (uint32_t)kMCH);
  const int r = (int)(hw / a.K), w = (int)(hw % a.K);
  const int tid = threadIdx.x;
  uint2* const L = a.lst + a.loff[r] + (int64_t)w * a.lcs[r];
  const uint32_t kb = a.lkb[hw];
  if (STEP == 0 || STEP == 1) {
    __shared__ uint32_t hst[256];
    hst[tid] = 0;
    __syncthreads();
    const uint32_t b1 = STEP == 1 ? a.lsel[hw * 4] : 0u;
    for (uint32_t i = i0 + tid; i < i1; i += 256) {
      if (STEP == 0) {
        const uint2 e = L[i];
        const uint32_t k = okey(value_bits(w, (uint16_t)e.y, js_hb(a, e.x), js_cost(a, e.x)));
        L[i].y = (e.y & 0xFFFFu) | (k << 16);
        if (k >= kb) atomicAdd(&hst[k >> 8], 1u);
      } else {
        const uint32_t k = L[i].y >> 16;
        if (k >= kb && (k >> 8) == b1) atomicAdd(&hst[k & 255u], 1u);
      }
    }
    __syncthreads();
    if (hst[tid]) atomicAdd(&a.lh[hw * 512 + STEP * 256 + tid], hst[tid]);
    return;
  }
  const uint32_t T = a.lsel[hw * 4 + 2], need = a.lsel[hw * 4 + 3];
  if (STEP == 2) {
    if (!need) return;
    for (uint32_t i = i0 + tid; i < i1; i += 256) {
      const uint2 e = L[i];
      if ((e.y >> 16) == T) {
        const uint32_t q = atomicAdd(&a.leqn[hw], 1u);
        if (q < (uint32_t)kListEq) a.leq[hw * kListEq + q] = e.x;
      }
    }
    return;
  }
  // STEP 3: bids, exactly as sa_list_round_kernel's last pass (leq sorted by sa_mlist_eq_kernel)
  const int sg = a.mseg[r];
  const uint32_t neq = min(a.leqn[hw], (uint32_t)kListEq);
  const uint32_t* eqj = a.leq + hw * kListEq;
  const uint16_t eps = a.eps[sg];
  const _Float16 epsh = __builtin_bit_cast(_Float16, eps);
  const _Float16 vT = __builtin_bit_cast(_Float16, okey_inv(T));
  const bool ret = *a.round_dev < 100;
  for (uint32_t i = i0 + tid; i < i1; i += 256) {
    const uint2 e = L[i];
    const uint32_t j = e.x, k = e.y >> 16;
    uint32_t bid = 0;
    if (k > T) {
      const _Float16 x = __builtin_bit_cast(_Float16, okey_inv(k));
      bid = __builtin_bit_cast(uint16_t, (_Float16)((_Float16)(x - vT) + epsh));
    } else if (k == T && need) {
      uint32_t lo = 0, hi = neq;  // rank of j among the equal values' jobs
      while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (eqj[mid] < j) lo = mid + 1; else hi = mid;
      }
      if (lo < need) bid = eps;
    }
    if (ret && js_hb(a, j) == w) bid = eps;  // retention: the previous winner bids eps on its job
    if (bid) atomicMax(&a.key[j], (bid << 16) | (0xFFFFu - (uint32_t)w));
  }
}

// the selections: STEP 0 the high byte b1 (>= jpw + 1 values at or above lkb, else the list fails); STEP 1
// the low byte, T and need.  One wave per worker.
template <int STEP>
__global__ __launch_bounds__(64) void sa_mlist_select_kernel(SegAuction a) {
  const int64_t hw = blockIdx.x;
  if (!a.lok[hw]) return;
  const int r = (int)(hw / a.K);
  const int sg = a.mseg[r];
  const int lane = threadIdx.x;
  const uint32_t jpw = (uint32_t)((a.seg_off[sg + 1] - a.seg_off[sg]) / a.K);
  const uint32_t* h = a.lh + hw * 512 + STEP * 256;
  uint32_t* sel = a.lsel + hw * 4;
  if (STEP == 0) {
    uint32_t tot = h[4 * lane] + h[4 * lane + 1] + h[4 * lane + 2] + h[4 * lane + 3];
    for (int o = 32; o > 0; o >>= 1) tot += (uint32_t)__shfl_xor((int)tot, o);
    if (tot < jpw + 1) {  // fewer than jpw + 1 values at or above the list base
      if (lane == 0) {
        list_stat(a, 5);
        mlist_fail(a, hw);
      }
      return;
    }
    uint32_t b = 0, above = 0;
    wave_select(h, jpw + 1, b, above);
    if (lane == 0) {
      sel[0] = b;
      sel[1] = above;
    }
  } else {
    uint32_t b = 0, above = 0;
    wave_select(h, jpw + 1 - sel[1], b, above);
    if (lane == 0) {
      const uint32_t T = (sel[0] << 8) | b;
      sel[2] = T;
      sel[3] = jpw - (sel[1] + above);
      if (T < a.lkb[hw]) mlist_fail(a, hw);  // (cannot happen with >= jpw + 1 values >= lkb; a guard)
    }
  }
}

// the equal values' jobs in ascending order (bitonic sort in LDS), the round's selection published and the
// list verdict; one block per worker
__global__ __launch_bounds__(kLT) void sa_mlist_eq_kernel(SegAuction a) {
  const int64_t hw = blockIdx.x;
  if (!a.lok[hw]) return;
  const int r = (int)(hw / a.K), w = (int)(hw % a.K);
  const int sg = a.mseg[r];
  const int tid = threadIdx.x;
  __shared__ uint32_t eqj[kListEq];
  const uint32_t T = a.lsel[hw * 4 + 2], need = a.lsel[hw * 4 + 3];
  const uint32_t neq = need ? a.leqn[hw] : 0u;
  if (neq > (uint32_t)kListEq) {
    if (tid == 0) {
      list_stat(a, 6);
      mlist_fail(a, hw);
    }
    return;
  }
  uint32_t* const g = a.leq + hw * kListEq;
  if (neq > 1) {
    uint32_t m = 1;
    while (m < neq) m <<= 1;
    for (uint32_t i = tid; i < m; i += kLT) eqj[i] = i < neq ? g[i] : 0xFFFFFFFFu;
    __syncthreads();
    for (uint32_t kk = 2; kk <= m; kk <<= 1)
      for (uint32_t jj = kk >> 1; jj > 0; jj >>= 1) {
        for (uint32_t i = tid; i < m; i += kLT) {
          const uint32_t p = i ^ jj;
          if (p > i) {
            const uint32_t x = eqj[i], y = eqj[p];
            if ((x > y) == ((i & kk) == 0)) {
              eqj[i] = y;
              eqj[p] = x;
            }
          }
        }
        __syncthreads();
      }
    for (uint32_t i = tid; i < neq; i += kLT) g[i] = eqj[i];
  }
  if (tid == 0) {
    uint32_t* sel = a.sel + ((int64_t)sg * a.K + w) * 4;
    sel[0] = T >> 8;
    sel[1] = 0;
    sel[2] = T;
    sel[3] = need;
    a.lbad[hw] = 0;
    list_stat(a, 0);
  }
}

// list regions: segment r's K lists of 4 * (N_s / K) + 256 entries each, in multi-chunk segment order
__global__ void sa_list_layout_kernel(SegAuction a) {
  int64_t off = 0;
  for (int r = 0; r < a.n_multi; ++r) {
    const int s = a.mseg[r];
    const int64_t cap = 4 * ((int64_t)(a.seg_off[s + 1] - a.seg_off[s]) / a.K) + 256;
    a.loff[r] = off;
    a.lcs[r] = (int32_t)cap;
    off += cap * a.K;
  }
}

// ---- resolve: per job of the live segments, one block per chunk ----
__global__ __launch_bounds__(256) void sa_resolve_kernel(SegAuction a, int32_t* __restrict__ out) {
  if (a.dmode && a.dmode[0] == 2) return;  // a void row-sharded slot changes no job state (kDVoid)
  const ChunkInfo ci = chunk_info(a, blockIdx.x);
  AST(const uint64_t r0 = ANOW();)
  resolve_chunk(a, ci, out, a.flag + ci.s);  // (the segment's flag tested after the chunk's loads are issued)
#ifdef RQSID_STAMPS
  if (threadIdx.x == 0) {
    atomicAdd(&g_al_stamps[8], (unsigned long long)(ANOW() - r0));
    atomicAdd(&g_al_stamps[9], 1ull);
  }
#endif
}

// end of a round: a segment whose every job has a bidder is done (it was live from round 0, so its
// round count is the rounds it took); the round number advances for the next round's bids (nothing in
// this kernel reads it)
__global__ __launch_bounds__(256) void sa_round_end_kernel(SegAuction a, int count) {
  const int s = blockIdx.x * 256 + threadIdx.x;
  if (s == 0) {
    *a.round_dev += 1;
    if (a.any_miss) *a.any_miss = 0;  // for the next round's select_guess (a store at the top of the guessed
                                      // pass would turn its uniform loads into vector loads)
    if (a.lany) *a.lany = 0;          // (the next round's list pass sets it for any failed list)
  }

  uint32_t live = 0;
  if (s < a.S && (a.flag[s] & kLive)) {
    const int64_t n_s = a.n_glob ? a.n_glob : a.seg_off[s + 1] - a.seg_off[s];
    a.rounds[s] += 1;
    if ((int64_t)a.have[s] == n_s) a.flag[s] &= ~kLive;
    else live = 1;
    a.have[s] = 0;
  }
  for (int o = 32; o > 0; o >>= 1) live += (uint32_t)__shfl_xor((int)live, o);
  if (count && (threadIdx.x & 63) == 0 && live) atomicAdd(a.live_count, live);
}

// copy the round state into (restore = 0) or back from (1) the lean block's snapshot
__global__ __launch_bounds__(256) void sa_snapshot_kernel(SegAuction a, int32_t* __restrict__ out, int64_t n,
                                                          int restore) {
  const int64_t g0 = (int64_t)blockIdx.x * 256 + threadIdx.x, gs = (int64_t)gridDim.x * 256;
  for (int64_t i = g0; i < n; i += gs) {
    if (!restore) {
      a.s_cost[i] = a.cost[i];
      a.s_hb[i] = a.hb[i];
      a.s_nobid[i] = a.nobid[i];
      a.s_out[i] = out[i];
    } else {
      a.cost[i] = a.s_cost[i];
      a.hb[i] = a.s_hb[i];
      if (a.js) a.js[i] = ((uint32_t)(a.s_hb[i] & 0xFFFF) << 16) | a.s_cost[i];
      a.nobid[i] = a.s_nobid[i];
      out[i] = a.s_out[i];
    }
  }
  const int64_t ns = (int64_t)a.S * a.K * 4;
  for (int64_t i = g0; i < ns; i += gs) {
    if (!restore) a.s_sel[i] = a.sel[i];
    else a.sel[i] = a.s_sel[i];
  }
  for (int64_t i = g0; i < a.S; i += gs) {
    if (!restore) {
      a.s_flag[i] = a.flag[i];
      a.s_rounds[i] = a.rounds[i];
    } else {
      a.flag[i] = a.s_flag[i];
      a.rounds[i] = a.s_rounds[i];
    }
  }
  if (g0 == 0) {
    if (!restore) a.s_sel[ns] = (uint32_t)*a.round_dev;
    else *a.round_dev = (int32_t)a.s_sel[ns];
  }
  // a rollback raises values again (costs of the block's start): lists built inside the block are void
  if (restore && a.lst)
    for (int64_t hw = g0; hw < (int64_t)a.n_multi * a.K; hw += gs) a.lcnt[hw * kAbovePad] = 0;
}

// multi-chunk segment ranks (one block): hidx[s] = rank or -1, mseg[rank] = s; live_count[1] = total,
// live_count[2] = the most jobs in one of them
__global__ __launch_bounds__(1024) void sa_multi_index_kernel(SegAuction a) {
  __shared__ uint32_t ws[16];
  __shared__ uint32_t carry;
  if (threadIdx.x == 0) carry = 0;
  __syncthreads();
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  for (int base = 0; base < a.S; base += 1024) {
    const int s = base + threadIdx.x;
    const uint32_t v = (s < a.S && (a.chunk_off[s + 1] - a.chunk_off[s] > 1 || a.n_glob)) ? 1u : 0u;
    const unsigned long long m = __ballot(v);
    const uint32_t before = __popcll(m & ((1ull << lane) - 1ull));
    if (lane == 0) ws[wv] = __popcll(m);
    __syncthreads();
    uint32_t off = carry;
    for (int q = 0; q < wv; ++q) off += ws[q];
    if (s < a.S) {
      const uint32_t r = off + before;
      a.hidx[s] = v ? (int32_t)r : -1;
      if (v && (int32_t)r < a.n_multi) a.mseg[r] = s;
      if (v) atomicMax(&a.live_count[2], (uint32_t)(a.seg_off[s + 1] - a.seg_off[s]));  // the longest (list size)
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      uint32_t t = 0;
      for (int q = 0; q < 16; ++q) t += ws[q];
      carry += t;
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) a.live_count[1] = carry;
}

struct Carve {
  char* p;
  int64_t used = 0;
  template <class T>
  T* take(int64_t n) {
    T* r = reinterpret_cast<T*>(p + used);
    used += (n * (int64_t)sizeof(T) + 255) / 256 * 256;
    return r;
  }
};

// workspace layout (also the size query when p == nullptr)
void carve(SegAuction& a, Carve& c, int64_t N, int32_t K, int32_t S, int64_t total_chunks, bool guess,
           bool dlist = false) {
  a.flag = c.take<uint8_t>(S);
  a.eps = c.take<uint16_t>(S);
  a.mm = c.take<uint32_t>(2 * (int64_t)S);
  a.have = c.take<uint32_t>(S);
  a.live_count = c.take<uint32_t>(4);
  a.round_dev = c.take<int32_t>(1);
  a.hidx = c.take<int32_t>(S);
  a.mseg = c.take<int32_t>(a.n_multi > 0 ? a.n_multi : 1);
  a.cost = c.take<uint16_t>(N);
  a.hb = c.take<int32_t>(N);
  a.nobid = c.take<uint8_t>(N);
  a.key = c.take<uint32_t>(N);
  a.hist = c.take<uint32_t>((int64_t)a.n_multi * K * 256 + (dlist ? 64 : 0));  // (+ the list failure count)
  a.sel = c.take<uint32_t>((int64_t)S * K * 4);
  a.eqcnt = c.take<uint32_t>((int64_t)K * total_chunks);
  a.eqtot = c.take<uint32_t>((int64_t)S * K);
  a.above = guess ? c.take<uint32_t>((int64_t)a.n_multi * K * kAbovePad) : nullptr;
  a.miss = guess ? c.take<uint8_t>((int64_t)a.n_multi * K) : nullptr;
  a.chist = guess && a.n_multi > 0 ? c.take<uint16_t>(total_chunks * K * 256) : nullptr;
  a.any_miss = guess ? c.take<uint32_t>(1) : nullptr;
  const bool snap = guess && a.n_multi > 0;
  a.s_cost = snap ? c.take<uint16_t>(N) : nullptr;
  a.s_hb = snap ? c.take<int32_t>(N) : nullptr;
  a.s_nobid = snap ? c.take<uint8_t>(N) : nullptr;
  a.s_out = snap ? c.take<int32_t>(N) : nullptr;
  a.s_sel = snap ? c.take<uint32_t>((int64_t)S * K * 4 + 1) : nullptr;  // + the round number
  a.s_flag = snap ? c.take<uint8_t>(S) : nullptr;
  a.s_rounds = snap ? c.take<int32_t>(S) : nullptr;
  // the bid lists of the multi-chunk segments (RQSID_AUCTION_LIST=0: the sweep, for A/B): segment s holds
  // K * (4 * (N_s / K) + 256) <= 4 N_s + 256 K entries
  // Only while a worker's list is short enough for its one block: at ~80k jobs per worker (K=128 over 10M
  // rows) the one-block-per-worker list round lost to the sweep (10M PROD training, level 1: 23 -> 33 s)
  const char* el = getenv("RQSID_AUCTION_LIST");
  const int64_t nm = a.n_multi > 0 ? a.n_multi : 1;
  const int lmode = el ? atoi(el) : 1;  // 0: sweep only; 1: lists (default); 2: one-block lists at any size
  // one wide segment with long lists: the multi-block list rounds (any jobs per worker); otherwise one block
  // per worker while the lists are short
  const char* emb = getenv("RQSID_LIST_MB_JPW");  // (A/B) the jobs per worker above which lists go multi-block
  const int64_t mb_jpw = emb ? std::max<int64_t>(1, atoll(emb)) : kListBlockJpw;
  const bool mb = guess && a.n_multi == 1 && lmode == 1 && N / K > mb_jpw;
  const bool list = guess && a.n_multi > 0 && lmode != 0 && (lmode == 2 || mb || N / (nm * K) <= kListMaxJpw);
  a.lmb_chunks = mb ? (int32_t)((4 * (N / K) + 256 + kMCH - 1) / kMCH) : 0;
  a.lh = mb ? c.take<uint32_t>(nm * K * 512) : nullptr;
  a.lsel = mb ? c.take<uint32_t>(nm * K * 4) : nullptr;
  a.leq = mb ? c.take<uint32_t>(nm * K * kListEq) : nullptr;
  a.leqn = mb ? c.take<uint32_t>(nm * K) : nullptr;
  a.lok = mb ? c.take<uint8_t>(nm * K) : nullptr;
  a.lst = list ? c.take<uint2>(4 * N + 256 * (int64_t)K * nm) : nullptr;
  a.lcnt = list ? c.take<uint32_t>(nm * K * kAbovePad) : nullptr;
  a.lkb = list ? c.take<uint32_t>(nm * K) : nullptr;
  a.lbad = list ? c.take<uint8_t>(nm * K) : nullptr;
  a.loff = list ? c.take<int64_t>(nm) : nullptr;
  a.lcs = list ? c.take<int32_t>(nm) : nullptr;
  a.lany = list ? c.take<uint32_t>(1) : nullptr;
  const char* ej = getenv("RQSID_LIST_JS");  // 0: the list rounds gather winner and cost separately (A/B)
  a.js = list && K <= 65535 && !(ej && atoi(ej) == 0) ? c.take<uint32_t>(N) : nullptr;
  const char* ls = getenv("RQSID_LIST_START");
  a.lstart = ls ? std::max(1, atoi(ls)) : K >= kListWideK ? kListStartWide : kListStart;
  const char* ed = getenv("RQSID_LIST_DELTA");
  a.ldelta = ed ? std::min(128, std::max(1, atoi(ed))) : kListDelta;
  a.rdone = guess && S == 1 && a.n_multi == 1 ? c.take<unsigned long long>(16 * (1 + kRd)) : nullptr;
  const char* es = getenv("RQSID_LIST_STATS");
  a.lstat = list && es && atoi(es) ? c.take<uint32_t>(8) : nullptr;
  if (dlist) {  // the row-sharded auction's lists: one rank's share, 8 * (N / K) + 256 entries per worker
    a.dcap = 8 * (N / K) + 256;
    a.dnb = (int32_t)std::max<int64_t>(1, (4 * (N / K) + 256 + kMCH - 1) / kMCH);
    a.lst = c.take<uint2>(a.dcap * K);
    a.lcnt = c.take<uint32_t>((int64_t)K * kAbovePad);
    a.lkb = c.take<uint32_t>(K);
    a.lbad = c.take<uint8_t>(K);
    a.lany = c.take<uint32_t>(1);
    a.lsel = c.take<uint32_t>((int64_t)K * 4);
    const char* ed2 = getenv("RQSID_DAUCTION_LIST");
    a.dlist_on = ed2 ? atoi(ed2) != 0 : 1;
  }
}

}  // namespace
}  // namespace rqsid

using namespace rqsid;

extern "C" {

int32_t rqsid_seg_auction_chunk_jobs(void) { return kCh; }

int64_t rqsid_seg_auction_workspace_bytes(int64_t n_jobs, int32_t n_workers, int32_t n_seg, int64_t total_chunks,
                                          int32_t n_multi) {
  if (n_jobs < 0 || n_workers <= 0 || n_seg <= 0 || total_chunks < 0 || n_multi < 0 || n_multi > n_seg) return -1;
  SegAuction a{};
  a.n_multi = n_multi;
  Carve c{nullptr};
  carve(a, c, n_jobs, n_workers, n_seg, total_chunks, true);
  return c.used;
}

int rqsid_seg_auction_lap_half(const uint16_t* scores, int32_t n_workers, int32_t n_seg, const int32_t* seg_off,
                               const int32_t* seg_chunk_off, int64_t total_chunks, int32_t n_multi, int64_t n_jobs,
                               const uint8_t* active, int32_t max_rounds, int32_t* out_assign, int32_t* out_rounds,
                               void* workspace, int64_t workspace_bytes, void* stream) {
  return rqsid::seg_auction_run(scores, n_workers, n_seg, seg_off, seg_chunk_off, total_chunks, n_multi, n_jobs,
                                active, max_rounds, out_assign, out_rounds, workspace, workspace_bytes, stream, false);
}

}  // extern "C"

namespace rqsid {
// vec: one segment whose rows and chunks allow 8-byte loads (rqsid_auction_lap_half with N % 4 == 0)
int seg_auction_run(const uint16_t* scores, int32_t n_workers, int32_t n_seg, const int32_t* seg_off,
                    const int32_t* seg_chunk_off, int64_t total_chunks, int32_t n_multi, int64_t n_jobs,
                    const uint8_t* active, int32_t max_rounds, int32_t* out_assign, int32_t* out_rounds,
                    void* workspace, int64_t workspace_bytes, void* stream, bool vec, bool single_layout) {
  single_layout = single_layout && n_seg == 1;
  vec = vec && n_seg == 1 && n_jobs % 4 == 0 && ((uintptr_t)scores & 7) == 0;
  if (!scores || !seg_off || !seg_chunk_off || !out_assign || !out_rounds || n_workers <= 0 || n_seg <= 0 ||
      total_chunks < 0 || total_chunks > INT32_MAX || n_jobs < 0 || n_jobs > INT32_MAX || n_multi < 0 ||
      n_multi > n_seg)
    return fail(RQSID_E_ARG, "seg_auction: bad arguments (K=%d S=%d chunks=%lld multi=%d)", n_workers, n_seg,
                (long long)total_chunks, n_multi);
  if (n_workers == 1) return fail(RQSID_E_ARG, "seg_auction: a single worker cannot bid on N + 1 jobs");
  if (!workspace ||
      workspace_bytes < rqsid_seg_auction_workspace_bytes(n_jobs, n_workers, n_seg, total_chunks, n_multi))
    return fail(RQSID_E_WORKSPACE, "seg_auction: workspace too small");
  hipStream_t st = (hipStream_t)stream;
  SegAuction a{};
  a.W = scores;
  a.K = n_workers;
  a.S = n_seg;
  a.total_chunks = total_chunks;
  a.seg_off = seg_off;
  a.chunk_off = seg_chunk_off;
  a.rounds = out_rounds;
  a.n_multi = n_multi;
  a.one_n = single_layout && n_multi == 1 ? n_jobs : 0;
  Carve c{(char*)workspace};
  carve(a, c, n_jobs, n_workers, n_seg, total_chunks, true);
  const unsigned gs = (unsigned)cdiv(n_seg, 256);
  // pinned readback ([0] live segments, [1] multi-chunk segments): one buffer per host thread, kept
  // for the thread's lifetime (the lockstep fits call this once per iteration)
  static thread_local uint32_t* host = nullptr;
  if (!host && hipHostMalloc((void**)&host, 4 * sizeof(uint32_t)) != hipSuccess) {
    host = nullptr;
    return fail(RQSID_E_LAUNCH, "seg_auction: pinned readback buffer");
  }
  int rc = RQSID_OK;
  if (fill_async(a.live_count, 0, 16, st) != hipSuccess || (a.rdone && fill_async(a.rdone, 0, 128 * (1 + kRd), st) != hipSuccess))
    return fail(RQSID_E_LAUNCH, "seg_auction: memset");
  hipLaunchKernelGGL(sa_seg_init_kernel, dim3(gs), dim3(256), 0, st, a, active);
  hipLaunchKernelGGL(sa_multi_index_kernel, dim3(1), dim3(1024), 0, st, a);
  if ((rc = check_launch("seg_auction_init")) ||
      hipMemcpyAsync(host, a.live_count, 12, hipMemcpyDeviceToHost, st) != hipSuccess ||
      hipStreamSynchronize(st) != hipSuccess)
    return rc ? rc : fail(RQSID_E_LAUNCH, "seg_auction: init readback");
  if ((int32_t)host[1] != n_multi)
    return fail(RQSID_E_ARG, "seg_auction: %u segments span more than one chunk, n_multi = %d", host[1], n_multi);
  if (total_chunks == 0) return RQSID_OK;
  if (host[0] == 0) {
    // no segment bids (all inactive, empty or N_s < K): only the argmin fallback runs, no rounds
    hipLaunchKernelGGL(sa_fallback_kernel, dim3((unsigned)total_chunks), dim3(256), 0, st, a, out_assign);
    return check_launch("seg_auction_fallback");
  }
  const bool any_single = n_multi < n_seg;
  const size_t mk = (size_t)n_multi * n_workers;
  if (n_multi > 0 && (fill_async(a.hist, 0, mk * 256 * 4, st) != hipSuccess ||
                      fill_async(a.above, 0, mk * kAbovePad * 4, st) != hipSuccess ||
                      fill_async(a.miss, 1, mk, st) != hipSuccess ||
                      fill_async(a.any_miss, 0, 4, st) != hipSuccess))
    return fail(RQSID_E_LAUNCH, "seg_auction: memset");
  // thresholds start at key 0 (a window of NaN keys: every worker takes the exact passes in round 0)
  if (fill_async(a.sel, 0, (size_t)n_seg * n_workers * 16, st) != hipSuccess)
    return fail(RQSID_E_LAUNCH, "seg_auction: memset");
  hipLaunchKernelGGL(sa_job_init_kernel, dim3(grid_cap(cdiv(n_jobs, 256), 8192)), dim3(256), 0, st, a, n_jobs);
  const dim3 gcw((unsigned)total_chunks, (unsigned)cdiv(n_workers, kKG));
  const dim3 gc((unsigned)total_chunks);
  const unsigned gmw = (unsigned)cdiv((int64_t)n_multi * n_workers, 4);
  hipLaunchKernelGGL(sa_fallback_kernel, gc, dim3(256), 0, st, a, out_assign);
  hipLaunchKernelGGL(sa_minmax_kernel, gcw, dim3(256), 0, st, a);
  hipLaunchKernelGGL(sa_eps_kernel, dim3(gs), dim3(256), 0, st, a);
  if ((rc = check_launch("seg_auction_init"))) return rc;
  // Rounds run in blocks of kPoll: the live count is read back after each block (rounds of finished
  // segments are no-ops, so stopping late only costs empty launches) and only a block's last round counts,
  // into a counter zeroed after each read.  The round number lives on the device, so one captured block
  // (a HIP graph of kPoll rounds) replays for every block: the auction is launch-bound at small N.
  constexpr int kPoll = 8;
  // list-only blocks are longer: their rounds are a few launches each, and the host's readback and launch
  // between two blocks (tens of us) cost as much as several rounds; a failed list replays the block's first
  // kPoll rounds in full from its snapshot, then the loop goes on from there
  const char* elb = getenv("RQSID_LIST_BLOCK");  // list-only rounds per captured block (A/B; default 32)
  const int kPollList = elb ? std::min(256, std::max(kPoll, atoi(elb))) : 32;
  // lean rounds leave out the two-pass kernels of missed workers (five launches of a few us each, empty
  // in most rounds); a lean block runs from a snapshot of the round state and is replayed with the full
  // rounds when any worker missed in it, so the result is the full rounds' in every case
  if (a.lst) {
    if (fill_async(a.lcnt, 0, (size_t)n_multi * n_workers * kAbovePad * 4, st) != hipSuccess ||
        fill_async(a.lbad, 1, (size_t)n_multi * n_workers, st) != hipSuccess)
      return fail(RQSID_E_LAUNCH, "seg_auction: memset");
    hipLaunchKernelGGL(sa_list_layout_kernel, dim3(1), dim3(1), 0, st, a);
    if (fill_async(a.lany, 0, 4, st) != hipSuccess) return fail(RQSID_E_LAUNCH, "seg_auction: memset");
    if (a.lstat && fill_async(a.lstat, 0, 32, st) != hipSuccess) return fail(RQSID_E_LAUNCH, "seg_auction: memset");
  }
  int n_lean = 0, n_replay = 0, n_full = 0, n_list = 0;  // (RQSID_LIST_STATS) round blocks by kind
  // list-only rounds (one wide-segment auctions whose lists all held in the last block): the list pass,
  // resolve and round end, without the guessed pass, selection and bid sweep, whose blocks all exit when
  // every list holds but whose dispatch over total_chunks x K/16 blocks costs ~0.2 ms per kernel at K=2560
  // over 6.25M jobs.  Such a block runs from a snapshot like a lean block and is replayed in full when any
  // list failed in it (live_count[3]).
  const bool list_only_ok = a.lst && !any_single;
  // short lists take 256-thread list-round blocks: capacity <= 4096 entries in every segment when there are
  // many segments (S x K blocks per round), <= 1024 for one segment (a 100k x 128 auction, capacity 3380, ran
  // 0.0194 -> 0.0207 ms per round with 256 threads; K=1280 x 100k, capacity 568, 0.0295 -> 0.0253)
  const char* els = getenv("RQSID_LIST_SMALL");  // 0: always 1024 threads; n > 1: one capacity limit (A/B)
  const int64_t lcap_max = 4 * ((int64_t)host[2] / n_workers) + 256;
  const int64_t lsmall_cap = els && atoi(els) > 1 ? atoi(els) : (n_multi > 1 ? 4096 : 1024);
  const bool lsmall = lcap_max <= lsmall_cap && !(els && atoi(els) == 0);
  auto launch_round = [&](hipStream_t q, bool count, bool lean, bool list_only = false) {
    if (a.lst && a.lmb_chunks) {
      const dim3 gw((unsigned)(n_multi * a.K)), gp((unsigned)((int64_t)n_multi * a.K * a.lmb_chunks));
      hipLaunchKernelGGL(sa_mlist_init_kernel, gw, dim3(256), 0, q, a);
      hipLaunchKernelGGL(sa_mlist_pass_kernel<0>, gp, dim3(256), 0, q, a);
      hipLaunchKernelGGL(sa_mlist_select_kernel<0>, gw, dim3(64), 0, q, a);
      hipLaunchKernelGGL(sa_mlist_pass_kernel<1>, gp, dim3(256), 0, q, a);
      hipLaunchKernelGGL(sa_mlist_select_kernel<1>, gw, dim3(64), 0, q, a);
      hipLaunchKernelGGL(sa_mlist_pass_kernel<2>, gp, dim3(256), 0, q, a);
      hipLaunchKernelGGL(sa_mlist_eq_kernel, gw, dim3(kLT), 0, q, a);
      hipLaunchKernelGGL(sa_mlist_pass_kernel<3>, gp, dim3(256), 0, q, a);
    } else if (a.lst) {
      if (lsmall) hipLaunchKernelGGL(sa_list_round_kernel<256>, dim3((unsigned)(n_multi * a.K)), dim3(256), 0, q, a);
      else hipLaunchKernelGGL(sa_list_round_kernel<kLT>, dim3((unsigned)(n_multi * a.K)), dim3(kLT), 0, q, a);
    }
    SegAuction ar = a;
    ar.rcount = count ? 1 : 0;
    if (list_only) {
      hipLaunchKernelGGL(sa_resolve_kernel, gc, dim3(256), 0, q, ar, out_assign);
      if (!a.rdone) hipLaunchKernelGGL(sa_round_end_kernel, dim3(gs), dim3(256), 0, q, a, (int)count);
      return;
    }
    if (n_multi > 0) {
      if (vec) hipLaunchKernelGGL((sa_guess_hist_kernel<true>), gcw, dim3(256), 0, q, a);
      else hipLaunchKernelGGL((sa_guess_hist_kernel<false>), gcw, dim3(256), 0, q, a);
      hipLaunchKernelGGL(sa_select_guess_kernel, dim3(gmw), dim3(256), 0, q, a);
      if (!lean) {
        // the two-pass selection for the workers the guessed pass missed (every block exits at once
        // when none of its workers missed)
        if (vec) hipLaunchKernelGGL((sa_hist_kernel<0, true>), gcw, dim3(256), 0, q, a);
        else hipLaunchKernelGGL((sa_hist_kernel<0, false>), gcw, dim3(256), 0, q, a);
        hipLaunchKernelGGL((sa_select_kernel<false>), dim3(gmw), dim3(256), 0, q, a);
        if (vec) hipLaunchKernelGGL((sa_hist_kernel<1, true>), gcw, dim3(256), 0, q, a);
        else hipLaunchKernelGGL((sa_hist_kernel<1, false>), gcw, dim3(256), 0, q, a);
        hipLaunchKernelGGL((sa_select_kernel<true>), dim3(gmw), dim3(256), 0, q, a);
        if (vec) hipLaunchKernelGGL((sa_eqcount_kernel<true>), gcw, dim3(256), 0, q, a);
        else hipLaunchKernelGGL((sa_eqcount_kernel<false>), gcw, dim3(256), 0, q, a);
        hipLaunchKernelGGL(sa_eqscan_kernel, dim3(gmw), dim3(256), 0, q, a);
      }
    }
    if (any_single) hipLaunchKernelGGL(sa_small_select_kernel, gcw, dim3(256), 0, q, a);
    if (vec) hipLaunchKernelGGL((sa_bid_kernel<true>), gcw, dim3(256), 0, q, a);
    else hipLaunchKernelGGL((sa_bid_kernel<false>), gcw, dim3(256), 0, q, a);
    hipLaunchKernelGGL(sa_resolve_kernel, gc, dim3(256), 0, q, ar, out_assign);
    if (!a.rdone) hipLaunchKernelGGL(sa_round_end_kernel, dim3(gs), dim3(256), 0, q, a, (int)count);
  };
  // capture blocks on a private stream (the caller's may be the null stream, which cannot capture)
  auto capture = [&](bool lean, bool list_only = false) {
    hipGraphExec_t ex = nullptr;
    hipStream_t cs = nullptr;
    hipGraph_t graph = nullptr;
    const int nr = list_only ? kPollList : kPoll;
    if (hipStreamCreateWithFlags(&cs, hipStreamNonBlocking) == hipSuccess) {
      if (hipStreamBeginCapture(cs, hipStreamCaptureModeRelaxed) == hipSuccess) {
        for (int i = 0; i < nr; ++i) launch_round(cs, i == nr - 1, lean, list_only);
        if (hipStreamEndCapture(cs, &graph) == hipSuccess && graph) {
          if (hipGraphInstantiate(&ex, graph, nullptr, nullptr, 0) != hipSuccess) ex = nullptr;
          (void)hipGraphDestroy(graph);
        }
      }
      (void)hipStreamDestroy(cs);
    }
    (void)hipGetLastError();  // a failed capture falls back to direct launches
    return ex;
  };
  hipGraphExec_t exec = capture(false);
  hipGraphExec_t exec_lean = n_multi > 0 && exec ? capture(true) : nullptr;
  const char* elo = getenv("RQSID_LIST_ONLY");  // 0: no list-only blocks (A/B)
  hipGraphExec_t exec_list = list_only_ok && exec_lean && !(elo && atoi(elo) == 0) ? capture(true, true) : nullptr;
  bool try_list = false;
  const unsigned gsnap = (unsigned)grid_cap(cdiv(std::max<int64_t>(n_jobs, (int64_t)n_seg * n_workers * 4), 256), 4096);
  if (fill_async(a.live_count, 0, 4, st) != hipSuccess) rc = fail(RQSID_E_LAUNCH, "seg_auction: memset");
  bool try_lean = false;  // round 0 misses everywhere (thresholds start at key 0)
  for (int done = 0; rc == RQSID_OK && (max_rounds <= 0 || done < max_rounds);) {
    int n = max_rounds > 0 ? std::min(kPoll, max_rounds - done) : kPoll;
    bool lonly = try_list && exec_list && (max_rounds <= 0 || max_rounds - done >= kPollList);
    // a list-only block must end by round 1000 (the leftover rounds > 1000 bid on unlisted pairs: every list
    // fails there, and a failed block costs its rounds plus a full replay): the rounds up to 1000 that no
    // whole block fits run list-only by direct launches (the list tail), from the same snapshot
    bool ltail = false;
    if (lonly && done + kPollList > 1001) {
      lonly = false;
      ltail = done < 1001 && (max_rounds <= 0 || max_rounds - done >= 1001 - done);
      if (ltail) n = 1001 - done;
    }
    if (lonly) n = kPollList;
    const bool lean = !lonly && !ltail && try_lean && exec_lean && n == kPoll;
    (lonly || ltail ? n_list : lean ? n_lean : n_full) += 1;
    if (fill_async(a.live_count + 2, 0, 8, st) != hipSuccess) {
      rc = fail(RQSID_E_LAUNCH, "seg_auction: memset");
      break;
    }
    if (ltail) {
      hipLaunchKernelGGL(sa_snapshot_kernel, dim3(gsnap), dim3(256), 0, st, a, out_assign, n_jobs, 0);
      for (int i = 0; i < n; ++i) launch_round(st, i == n - 1, true, true);
    } else if (lonly || lean) {
      hipLaunchKernelGGL(sa_snapshot_kernel, dim3(gsnap), dim3(256), 0, st, a, out_assign, n_jobs, 0);
      if (hipGraphLaunch(lonly ? exec_list : exec_lean, st) != hipSuccess) {
        rc = fail(RQSID_E_LAUNCH, "seg_auction: graph launch");
        break;
      }
    } else if (exec && n == kPoll) {
      if (hipGraphLaunch(exec, st) != hipSuccess) {
        rc = fail(RQSID_E_LAUNCH, "seg_auction: graph launch");
        break;
      }
    } else {
      for (int i = 0; i < n; ++i) launch_round(st, i == n - 1, false);
    }
    if ((rc = check_launch("seg_auction_round"))) break;
    if (hipMemcpyAsync(host, a.live_count, 16, hipMemcpyDeviceToHost, st) != hipSuccess ||
        fill_async(a.live_count, 0, 4, st) != hipSuccess || hipStreamSynchronize(st) != hipSuccess) {
      rc = fail(RQSID_E_LAUNCH, "seg_auction: readback");
      break;
    }
    if ((lean && host[2]) || ((lonly || ltail) && host[3])) {
      // a worker missed inside the lean block, or a list failed inside the list-only block: back to its
      // start, replay it with the exact passes
      hipLaunchKernelGGL(sa_snapshot_kernel, dim3(gsnap), dim3(256), 0, st, a, out_assign, n_jobs, 1);
      if (hipGraphLaunch(exec, st) != hipSuccess) {
        rc = fail(RQSID_E_LAUNCH, "seg_auction: graph launch");
        break;
      }
      if ((rc = check_launch("seg_auction_replay"))) break;
      if (hipMemcpyAsync(host, a.live_count, 4, hipMemcpyDeviceToHost, st) != hipSuccess ||
          fill_async(a.live_count, 0, 4, st) != hipSuccess || hipStreamSynchronize(st) != hipSuccess) {
        rc = fail(RQSID_E_LAUNCH, "seg_auction: readback");
        break;
      }
      try_lean = false;
      try_list = false;
      ++n_replay;
      n = kPoll;  // the replayed block's rounds (a list-only block's later rounds are not run)
    } else {
      try_lean = n_multi > 0;
      // every list held through this block, and the block's sweep rounds reached the list start (lists exist)
      try_list = host[3] == 0 && done + n > a.lstart;
    }
    done += n;
    if (host[0] == 0) break;
    if (max_rounds > 0 && done >= max_rounds)
      rc = fail(RQSID_E_LAUNCH, "seg_auction: %u segments still bidding after %d rounds", host[0], max_rounds);
  }
  if (exec_list) (void)hipGraphExecDestroy(exec_list);
  if (exec_lean) (void)hipGraphExecDestroy(exec_lean);
  if (exec) (void)hipGraphExecDestroy(exec);
  if (rc == RQSID_OK && a.lstat) {
    uint32_t v[8] = {};
    if (hipMemcpyAsync(v, a.lstat, 32, hipMemcpyDeviceToHost, st) == hipSuccess && hipStreamSynchronize(st) == hipSuccess)
      fprintf(stderr,
              "rqsid list stats K=%d N=%lld: ok %u none %u overflow %u leftover %u drift %u few %u ties %u | "
              "blocks list-only %d lean %d full %d replayed %d\n",
              n_workers, (long long)n_jobs, v[0], v[1], v[2], v[3], v[4], v[5], v[6], n_list, n_lean, n_full, n_replay);
  }
  return rc;
}

}  // namespace rqsid

// ---------------------------------------------------------------------------------------------------------
// Row-sharded single auction, one pass per call (distributed.ShardedAuction drives the rounds and the
// collectives between the passes).  The workspace holds a 512-B header (segment / chunk tables, round
// count) and the segmented state with S = 1, every chunk on the global-histogram path.
// ---------------------------------------------------------------------------------------------------------
namespace {
constexpr int64_t kDHeader = 512;

// ---- row-sharded list rounds --------------------------------------------------------------------------------
// The single-process list rounds (sa_list_round_kernel) with the rank's own jobs: a sweep round that starts the
// list phase appends each worker's values of this rank's jobs with key >= lkb = T - kListDelta (T: the round's
// threshold, the same on every rank) to the worker's list; the next rounds take their selection, tie ranks and
// bids from the lists alone.  The collectives are the sweep round's, in the same order, so the host protocol
// (ShardedAuction.run) does not know which kind of round runs: the list histograms (keys >= lkb) are summed
// over the ranks like the sweep's, the per-rank counts of values equal to T are all-gathered like the sweep's,
// and `have` is summed.  Validity is global and decided on every rank from reduced data only: no rank's list
// overflowed (a count summed with the high-byte histogram), >= jpw + 1 listed values >= lkb over all ranks,
// T_prev >= lkb and round <= 1000.  When it fails the slot turns void (kDVoid: nothing of the job state
// changes, the round counter does not advance) and the next slot runs the same round as a sweep, which
// rebuilds the lists.  Why the lists are exact while they hold: sa_list_round_kernel's argument, per rank
// (values only fall between rounds except the previous winner's, a worker only wins jobs it bid on, i.e.
// listed ones).  The ties at T: the first `need` equal values in global job order bid, the ranks' blocks
// follow each other, so rank r's equal values rank after the lower ranks' (rank_off, from the gather).
constexpr uint32_t kDSweep = 0, kDList = 1, kDVoid = 2;

__device__ __forceinline__ bool dl_build_round(const SegAuction& a) {  // the next round runs from lists
  const int next = *a.round_dev + 1;
  return a.dlist_on && next >= a.lstart && next <= 1000;
}

// before a list build: empty lists with base key lkb = T - delta
__global__ __launch_bounds__(256) void da_list_prep_kernel(SegAuction a) {
  if (a.dmode[0] != kDSweep || !dl_build_round(a) || !(a.flag[0] & kLive)) return;
  for (int w = blockIdx.x * 256 + threadIdx.x; w < a.K; w += gridDim.x * 256) {
    a.lcnt[(int64_t)w * kAbovePad] = 0;
    const uint32_t T = a.sel[(int64_t)w * 4 + 2];
    a.lkb[w] = T > (uint32_t)a.ldelta ? T - (uint32_t)a.ldelta : 0u;
  }
}

// the build: every value of this rank's chunk with key >= lkb, as {local job, raw score}; one global atomic
// per (block, worker) reserves its range (entries past the capacity are dropped: the next list round fails)
template <bool VEC>
__global__ __launch_bounds__(256) void da_list_build_kernel(SegAuction a) {
  if (a.dmode[0] != kDSweep || !dl_build_round(a)) return;
  const ChunkInfo ci = chunk_info(a, blockIdx.x);
  if (!(a.flag[ci.s] & kLive)) return;
  __shared__ uint32_t cnt[kKG], base[kKG];
  const int w0 = blockIdx.y * kKG, nw = min(kKG, a.K - w0);
  const int lane = threadIdx.x & 63;
  if (threadIdx.x < kKG) cnt[threadIdx.x] = 0;
  __syncthreads();
  uint32_t kb[kKG];
#pragma unroll
  for (int g = 0; g < kKG; ++g) kb[g] = g < nw ? a.lkb[w0 + g] : 0xFFFFFFFFu;
  ChunkScores cs;
  load_chunk<VEC>(a, ci, w0, cs);
  uint32_t mine[kKG] = {};
#pragma unroll
  for (int t = 0; t < kJPT; ++t) {
    const bool live = job_of<VEC>(t) < ci.nj;
#pragma unroll
    for (int g = 0; g < kKG; ++g) {
      const bool in = live && okey(value_bits(w0 + g, cs.v[t][g], cs.hb[t], cs.c[t])) >= kb[g];
      mine[g] |= (uint32_t)in << t;
      const uint32_t c = (uint32_t)__popcll(__ballot(in));
      if (lane == 0 && c) atomicAdd(&cnt[g], c);
    }
  }
  __syncthreads();
  if (threadIdx.x < nw) {
    const uint32_t c = cnt[threadIdx.x];
    base[threadIdx.x] = c ? atomicAdd(&a.lcnt[(int64_t)(w0 + threadIdx.x) * kAbovePad], c) : 0u;
    cnt[threadIdx.x] = 0;
  }
  __syncthreads();
  const uint32_t cap = (uint32_t)a.dcap;
#pragma unroll
  for (int g = 0; g < kKG; ++g) {
    if (!mine[g]) continue;
#pragma unroll
    for (int t = 0; t < kJPT; ++t) {
      if (!((mine[g] >> t) & 1u)) continue;
      const uint32_t pos = base[g] + atomicAdd(&cnt[g], 1u);
      if (pos < cap)
        a.lst[(int64_t)(w0 + g) * a.dcap + pos] = make_uint2((uint32_t)(ci.j0 + job_of<VEC>(t)), cs.v[t][g]);
    }
  }
}

// the list passes, a grid of K x dnb blocks (block c of worker w walks the worker's entry chunks c, c + dnb, ..):
// STEP 0: this round's keys (kept in the entries' upper 16 bits; an overflowed list counts into the failure
// word) and the high-byte histogram of the keys >= lkb; 1: the low-byte histogram of bin b1; 2: this rank's
// count of values equal to T; 3: the bids
template <int STEP>
__global__ __launch_bounds__(256) void da_list_pass_kernel(SegAuction a) {
  if (a.dmode[0] != kDList || !(a.flag[0] & kLive)) return;
  const int w = (int)(blockIdx.x / a.dnb), c0 = (int)(blockIdx.x % a.dnb);
  const int tid = threadIdx.x;
  const uint32_t cap = (uint32_t)a.dcap, n_raw = a.lcnt[(int64_t)w * kAbovePad], n = min(n_raw, cap);
  uint2* const L = a.lst + (int64_t)w * a.dcap;
  const uint32_t kb = a.lkb[w];
  const uint32_t stride = (uint32_t)a.dnb * kMCH;
  if (STEP == 0 && c0 == 0 && tid == 0 && n_raw > cap) atomicAdd(a.hist + (int64_t)a.K * 256, 1u);
  if (STEP <= 1) {
    __shared__ uint32_t hst[256];
    hst[tid] = 0;
    __syncthreads();
    const uint32_t b1 = STEP == 1 ? a.sel[(int64_t)w * 4] : 0u;
    for (uint32_t i0 = (uint32_t)c0 * kMCH; i0 < n; i0 += stride) {
      const uint32_t i1 = min(n, i0 + (uint32_t)kMCH);
      for (uint32_t i = i0 + tid; i < i1; i += 256) {
        if (STEP == 0) {
          const uint2 e = L[i];
          const uint32_t k = okey(value_bits(w, (uint16_t)e.y, a.hb[e.x], a.cost[e.x]));
          L[i].y = (e.y & 0xFFFFu) | (k << 16);
          if (k >= kb) atomicAdd(&hst[k >> 8], 1u);
        } else {
          const uint32_t k = L[i].y >> 16;
          if (k >= kb && (k >> 8) == b1) atomicAdd(&hst[k & 255u], 1u);
        }
      }
    }
    __syncthreads();
    if (hst[tid]) atomicAdd(&a.hist[(int64_t)w * 256 + tid], hst[tid]);
    return;
  }
  const uint32_t T = a.sel[(int64_t)w * 4 + 2];
  if (STEP == 2) {
    uint32_t c = 0;
    for (uint32_t i0 = (uint32_t)c0 * kMCH; i0 < n; i0 += stride) {
      const uint32_t i1 = min(n, i0 + (uint32_t)kMCH);
      for (uint32_t i = i0 + tid; i < i1; i += 256) c += (L[i].y >> 16) == T ? 1u : 0u;
    }
    for (int o = 32; o > 0; o >>= 1) c += (uint32_t)__shfl_xor((int)c, o);
    if ((tid & 63) == 0 && c) atomicAdd(&a.eqtot[w], c);
    return;
  }
  // STEP 3: values above T bid (x - T) + eps; of the values equal to T the first `need` in global job order
  // (lsel: 0 none of this rank's, 1 all of them, 2 those with job <= J); the retention override; one packed
  // {bid, ~worker} atomicMax per job as the sweep's bid kernel
  const uint32_t md = a.lsel[(int64_t)w * 4 + 1], J = a.lsel[(int64_t)w * 4];
  const uint16_t eps = a.eps[0];
  const _Float16 epsh = __builtin_bit_cast(_Float16, eps);
  const _Float16 vT = __builtin_bit_cast(_Float16, okey_inv(T));
  const bool ret = *a.round_dev < 100;
  for (uint32_t i0 = (uint32_t)c0 * kMCH; i0 < n; i0 += stride) {
    const uint32_t i1 = min(n, i0 + (uint32_t)kMCH);
    for (uint32_t i = i0 + tid; i < i1; i += 256) {
      const uint2 e = L[i];
      const uint32_t j = e.x, k = e.y >> 16;
      uint32_t bid = 0;
      if (k > T) {
        const _Float16 x = __builtin_bit_cast(_Float16, okey_inv(k));
        bid = __builtin_bit_cast(uint16_t, (_Float16)((_Float16)(x - vT) + epsh));
      } else if (k == T && (md == 1 || (md == 2 && j <= J))) {
        bid = eps;
      }
      if (ret && a.hb[j] == w) bid = eps;  // retention: the previous winner bids eps on its job
      if (bid) atomicMax(&a.key[j], (bid << 16) | (0xFFFFu - (uint32_t)w));
    }
  }
}

// the selections from the summed list histograms (one wave per worker), and the round's global list verdict
template <bool LOW>
__global__ __launch_bounds__(256) void da_list_select_kernel(SegAuction a) {
  // (the high-byte selection also runs in a slot another wave has just made void: every wave clears its
  // worker's histogram for the sweep that follows)
  if (a.dmode[0] != kDList && (LOW || a.dmode[0] != kDVoid)) return;
  if (!(a.flag[0] & kLive)) return;
  const int w = (int)(blockIdx.x * 4 + (threadIdx.x >> 6));
  if (w >= a.K) return;
  const int lane = threadIdx.x & 63;
  const uint32_t jpw = (uint32_t)(a.n_glob / a.K);
  uint32_t* h = a.hist + (int64_t)w * 256;
  uint32_t* sel = a.sel + (int64_t)w * 4;
  if (!LOW) {
    uint32_t tot = h[4 * lane] + h[4 * lane + 1] + h[4 * lane + 2] + h[4 * lane + 3];
    for (int o = 32; o > 0; o >>= 1) tot += (uint32_t)__shfl_xor((int)tot, o);
    const bool bad = a.dmode[0] != kDList || a.hist[(int64_t)a.K * 256] != 0 || tot < jpw + 1 || sel[2] < a.lkb[w] ||
                     *a.round_dev > 1000;
    if (bad) {  // the slot turns void on every rank (each decides from the same reduced data)
      if (lane == 0) {
        a.dmode[0] = kDVoid;
        *a.lany = 0;
      }
    } else {
      uint32_t b, above;
      wave_select(h, jpw + 1, b, above);
      if (lane == 0) {
        sel[0] = b;
        sel[1] = jpw + 1 - above;
        sel[3] = above;
      }
    }
  } else {
    uint32_t b, above;
    wave_select(h, sel[1], b, above);
    if (lane == 0) {
      const uint32_t T = (sel[0] << 8) | b;
      sel[3] = jpw - (sel[3] + above);
      sel[2] = T;
      a.eqtot[w] = 0;
    }
  }
  for (int i = lane; i < 256; i += 64) h[i] = 0;  // ready for the next histogram
}

// which of this rank's values equal to T bid: need - rank_off of them (in job order); when that is neither
// none nor all, J = the (need - rank_off)-th smallest job among them by a radix select over the job bytes.
// One block per worker (most exit at once: the threshold's ties straddle the rank boundary rarely)
__global__ __launch_bounds__(256) void da_list_rank_kernel(SegAuction a) {
  if (a.dmode[0] != kDList || !(a.flag[0] & kLive)) return;
  const int w = blockIdx.x;
  const int tid = threadIdx.x;
  const uint32_t need = a.sel[(int64_t)w * 4 + 3], off = a.rank_off ? a.rank_off[w] : 0u, loc = a.eqtot[w];
  const uint32_t nl = need > off ? min(need - off, loc) : 0u;
  if (tid == 0) a.lsel[(int64_t)w * 4 + 1] = nl == 0 ? 0u : nl == loc ? 1u : 2u;
  if (nl == 0 || nl == loc) return;
  __shared__ uint32_t hst[256];
  __shared__ uint32_t sh[2];
  const uint32_t T = a.sel[(int64_t)w * 4 + 2];
  const uint32_t n = min(a.lcnt[(int64_t)w * kAbovePad], (uint32_t)a.dcap);
  const uint2* const L = a.lst + (int64_t)w * a.dcap;
  uint32_t J = 0, rank = nl;
  for (int shift = 24; shift >= 0; shift -= 8) {
    __syncthreads();
    hst[tid] = 0;
    __syncthreads();
    for (uint32_t i = tid; i < n; i += 256) {
      const uint2 e = L[i];
      if ((e.y >> 16) == T && (shift == 24 || (e.x >> (shift + 8)) == J)) atomicAdd(&hst[(e.x >> shift) & 255u], 1u);
    }
    __syncthreads();
    if (tid < 64) {  // ascending walk: the bin holding the rank-th smallest
      const uint32_t h0 = hst[4 * tid], h1 = hst[4 * tid + 1], h2 = hst[4 * tid + 2], h3 = hst[4 * tid + 3];
      const uint32_t own = h0 + h1 + h2 + h3;
      uint32_t inc = own;
      for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = (uint32_t)__shfl_up((int)inc, o);
        if (tid >= o) inc += y;
      }
      const unsigned long long m = __ballot(inc >= rank);
      const int Ln = m ? __ffsll((long long)m) - 1 : 63;
      if (tid == Ln) {
        uint32_t acc = inc - own;
        const uint32_t hv[4] = {h0, h1, h2, h3};
        int q = 0;
        for (; q < 3; ++q) {
          if (acc + hv[q] >= rank) break;
          acc += hv[q];
        }
        sh[0] = (uint32_t)(4 * Ln + q);
        sh[1] = rank - acc;
      }
    }
    __syncthreads();
    J = (J << 8) | sh[0];
    rank = sh[1];
  }
  if (tid == 0) a.lsel[(int64_t)w * 4] = J;
}

// end of a row-sharded round slot (one block): a void slot leaves the round as it was; otherwise the round
// counts, the auction is done when the summed `have` covers every job, and the next slot lists iff lists exist
// (built in this sweep slot or held in this list slot) and the next round is in the list range
__global__ __launch_bounds__(256) void da_round_end_kernel(SegAuction a) {
  const uint32_t mode = a.dmode[0];
  const uint32_t next = mode == kDVoid ? kDSweep : (dl_build_round(a) ? kDList : kDSweep);
  __syncthreads();  // every thread read the round before thread 0 advances it
  if (threadIdx.x == 0) {
    if (mode != kDVoid) {
      *a.round_dev += 1;
      if (a.flag[0] & kLive) {
        a.rounds[0] += 1;
        if ((int64_t)a.have[0] == a.n_glob) a.flag[0] &= ~kLive;
      }
    }
    a.have[0] = 0;
    a.dmode[0] = next;
    a.dmode[1] = next == kDSweep ? 1u : 0u;
    *a.lany = next == kDSweep ? 1u : 0u;
    a.hist[(int64_t)a.K * 256] = 0;
  }
  for (int w = threadIdx.x; w < a.K; w += 256) a.lbad[w] = next == kDSweep ? 1 : 0;
}

// start of a list-only slot (the caller launched no sweep kernel for it): when the slot is a sweep, it turns void
// (nothing changes; the round runs as a sweep in the first full slot after the caller's next poll)
__global__ void da_slot_list_only_kernel(SegAuction a) {
  if (a.dmode[0] == kDSweep) {
    a.dmode[0] = kDVoid;
    a.dmode[1] = 0;
    *a.lany = 0;
  }
}

__global__ void da_list_init_kernel(SegAuction a) {  // the first slot sweeps; no lists yet
  a.dmode[0] = kDSweep;
  a.dmode[1] = 1;
  *a.lany = 1;
  a.hist[(int64_t)a.K * 256] = 0;
}

__global__ void dauction_tables_kernel(int32_t* seg_off, int32_t* chunk_off, int32_t n, int32_t nch) {
  seg_off[0] = 0;
  seg_off[1] = n;
  chunk_off[0] = 0;
  chunk_off[1] = nch;
}

int dstate(SegAuction& a, const uint16_t* scores, int32_t k, int64_t n_local, int64_t n_global, void* ws,
           int64_t wsb) {
  if (!scores && n_local > 0) return fail(RQSID_E_ARG, "dauction: null scores");
  if (k <= 1 || n_local < 0 || n_local > INT32_MAX || n_global < n_local || !ws)
    return fail(RQSID_E_ARG, "dauction: bad arguments (K=%d n_local=%lld n_global=%lld)", k, (long long)n_local,
                (long long)n_global);
  const int64_t nch = cdiv(n_local, kCh);
  a = SegAuction{};
  a.W = scores;
  a.K = k;
  a.S = 1;
  a.total_chunks = nch;
  a.n_multi = 1;
  a.n_glob = n_global > 0 ? n_global : 1;
  char* p = (char*)ws;
  a.seg_off = (const int32_t*)p;
  a.chunk_off = (const int32_t*)(p + 64);
  a.rounds = (int32_t*)(p + 128);
  a.dmode = (uint32_t*)(p + 192);  // [0] slot mode (the caller may poll it), [1] sweep-slot flag
  Carve c{p + kDHeader};
  carve(a, c, n_local, k, 1, nch, false, true);
  a.any_miss = a.dmode + 1;        // after carve (which clears it): the sweep kernels exit unless it is set
  if (wsb < kDHeader + c.used) return fail(RQSID_E_WORKSPACE, "dauction: workspace too small");
  return RQSID_OK;
}

// a rank's share takes the 8-byte-load sweeps when its rows and chunks allow them (load_chunk<true>)
bool dvec(const uint16_t* scores, int64_t n_local) {
  return n_local % 4 == 0 && ((uintptr_t)scores & 7) == 0;
}

int64_t dws(int64_t n_local, int32_t k) {
  SegAuction a{};
  a.n_multi = 1;
  Carve c{nullptr};
  carve(a, c, n_local, k, 1, cdiv(n_local, kCh), false, true);
  return kDHeader + c.used;
}
}  // namespace

extern "C" {

int64_t rqsid_dauction_workspace_bytes(int64_t n_local, int32_t n_workers) {
  if (n_local < 0 || n_workers <= 0) return -1;
  return dws(n_local, n_workers);
}

int rqsid_dauction_layout(int64_t n_local, int32_t n_workers, int64_t* offsets) {
  if (!offsets || n_local < 0 || n_workers <= 0) return fail(RQSID_E_ARG, "dauction_layout: bad arguments");
  SegAuction a{};
  a.n_multi = 1;
  Carve c{(char*)nullptr + kDHeader};
  carve(a, c, n_local, n_workers, 1, cdiv(n_local, kCh), false, true);
  offsets[0] = (int64_t)((char*)a.mm - (char*)nullptr);     // u32 [2]: max key, min key
  offsets[1] = (int64_t)((char*)a.hist - (char*)nullptr);   // u32 [K][256]
  offsets[2] = (int64_t)((char*)a.eqtot - (char*)nullptr);  // u32 [K]
  offsets[3] = (int64_t)((char*)a.have - (char*)nullptr);   // u32 [1]
  offsets[4] = (int64_t)((char*)a.flag - (char*)nullptr);   // u8 [1]: bit 0 = still bidding
  offsets[5] = 128;                                         // i32 [1]: rounds run (header, see dstate)
  return RQSID_OK;
}

int rqsid_dauction_begin(const uint16_t* scores, int32_t n_workers, int64_t n_local, int64_t n_global,
                         int32_t* out_assign, void* workspace, int64_t workspace_bytes, void* stream) {
  SegAuction a;
  int rc = dstate(a, scores, n_workers, n_local, n_global, workspace, workspace_bytes);
  if (rc) return rc;
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(dauction_tables_kernel, dim3(1), dim3(1), 0, st, (int32_t*)a.seg_off, (int32_t*)a.chunk_off,
                     (int32_t)n_local, (int32_t)a.total_chunks);
  hipLaunchKernelGGL(sa_seg_init_kernel, dim3(1), dim3(256), 0, st, a, (const uint8_t*)nullptr);
  hipLaunchKernelGGL(sa_multi_index_kernel, dim3(1), dim3(1024), 0, st, a);
  if (fill_async(a.hist, 0, ((size_t)n_workers * 256 + 64) * 4, st) != hipSuccess ||
      fill_async(a.lcnt, 0, (size_t)n_workers * kAbovePad * 4, st) != hipSuccess ||
      fill_async(a.lbad, 1, (size_t)n_workers, st) != hipSuccess || fill_async(a.lsel, 0, (size_t)n_workers * 16, st) != hipSuccess)
    return fail(RQSID_E_LAUNCH, "dauction: memset");
  hipLaunchKernelGGL(da_list_init_kernel, dim3(1), dim3(1), 0, st, a);
  if (n_local > 0) {
    hipLaunchKernelGGL(sa_job_init_kernel, dim3(grid_cap(cdiv(n_local, 256), 8192)), dim3(256), 0, st, a, n_local);
    hipLaunchKernelGGL(sa_fallback_kernel, dim3((unsigned)a.total_chunks), dim3(256), 0, st, a, out_assign);
    hipLaunchKernelGGL(sa_minmax_kernel, dim3((unsigned)a.total_chunks, (unsigned)cdiv(n_workers, kKG)), dim3(256), 0,
                       st, a);
  }
  return check_launch("dauction_begin");
}

// eps from the (caller-reduced) global min / max keys
int rqsid_dauction_eps(const uint16_t* scores, int32_t n_workers, int64_t n_local, int64_t n_global, void* workspace,
                       int64_t workspace_bytes, void* stream) {
  SegAuction a;
  int rc = dstate(a, scores, n_workers, n_local, n_global, workspace, workspace_bytes);
  if (rc) return rc;
  hipLaunchKernelGGL(sa_eps_kernel, dim3(1), dim3(256), 0, (hipStream_t)stream, a);
  return check_launch("dauction_eps");
}

// local histogram of the high (low = 0) or low (low = 1) byte of every worker's value keys
int rqsid_dauction_hist(const uint16_t* scores, int32_t n_workers, int64_t n_local, int64_t n_global, int32_t low,
                        void* workspace, int64_t workspace_bytes, void* stream) {
  SegAuction a;
  int rc = dstate(a, scores, n_workers, n_local, n_global, workspace, workspace_bytes);
  if (rc) return rc;
  if (n_local == 0) return RQSID_OK;
  const dim3 g((unsigned)a.total_chunks, (unsigned)cdiv(n_workers, kKG));
  hipStream_t st = (hipStream_t)stream;
  const bool vec = dvec(scores, n_local);
  // (each kernel exits at once unless the slot is its kind: sweep, or list)
  if (low && vec) hipLaunchKernelGGL((sa_hist_kernel<1, true>), g, dim3(256), 0, st, a);
  else if (low) hipLaunchKernelGGL((sa_hist_kernel<1, false>), g, dim3(256), 0, st, a);
  else if (vec) hipLaunchKernelGGL((sa_hist_kernel<0, true>), g, dim3(256), 0, st, a);
  else hipLaunchKernelGGL((sa_hist_kernel<0, false>), g, dim3(256), 0, st, a);
  const dim3 gl((unsigned)((int64_t)n_workers * a.dnb));
  if (low) hipLaunchKernelGGL((da_list_pass_kernel<1>), gl, dim3(256), 0, st, a);
  else hipLaunchKernelGGL((da_list_pass_kernel<0>), gl, dim3(256), 0, st, a);
  return check_launch("dauction_hist");
}

// selection from the (caller-reduced) histograms; clears them for the next pass
int rqsid_dauction_select(const uint16_t* scores, int32_t n_workers, int64_t n_local, int64_t n_global, int32_t low,
                          void* workspace, int64_t workspace_bytes, void* stream) {
  SegAuction a;
  int rc = dstate(a, scores, n_workers, n_local, n_global, workspace, workspace_bytes);
  if (rc) return rc;
  const unsigned g = (unsigned)cdiv(n_workers, 4);
  hipStream_t st = (hipStream_t)stream;
  if (low) {
    hipLaunchKernelGGL((sa_select_kernel<true>), dim3(g), dim3(256), 0, st, a);
    hipLaunchKernelGGL((da_list_select_kernel<true>), dim3(g), dim3(256), 0, st, a);
  } else {
    hipLaunchKernelGGL((sa_select_kernel<false>), dim3(g), dim3(256), 0, st, a);
    hipLaunchKernelGGL((da_list_select_kernel<false>), dim3(g), dim3(256), 0, st, a);
  }
  return check_launch("dauction_select");
}

// values equal to each worker's threshold: per-chunk offsets on this rank and the rank's totals (eqtot)
int rqsid_dauction_eqcount(const uint16_t* scores, int32_t n_workers, int64_t n_local, int64_t n_global,
                           void* workspace, int64_t workspace_bytes, void* stream) {
  SegAuction a;
  int rc = dstate(a, scores, n_workers, n_local, n_global, workspace, workspace_bytes);
  if (rc) return rc;
  hipStream_t st = (hipStream_t)stream;
  if (n_local == 0) {
    if (fill_async(a.eqtot, 0, (size_t)n_workers * 4, st) != hipSuccess)
      return fail(RQSID_E_LAUNCH, "dauction: memset");
    return RQSID_OK;
  }
  const dim3 g((unsigned)a.total_chunks, (unsigned)cdiv(n_workers, kKG));
  const bool vec = dvec(scores, n_local);
  if (vec) hipLaunchKernelGGL((sa_eqcount_kernel<true>), g, dim3(256), 0, st, a);
  else hipLaunchKernelGGL((sa_eqcount_kernel<false>), g, dim3(256), 0, st, a);
  hipLaunchKernelGGL(sa_eqscan_kernel, dim3((unsigned)cdiv(n_workers, 4)), dim3(256), 0, st, a);
  // a sweep slot before the list phase builds the lists from this round's values (T is final here)
  hipLaunchKernelGGL(da_list_prep_kernel, dim3((unsigned)cdiv(n_workers, 256)), dim3(256), 0, st, a);
  if (vec) hipLaunchKernelGGL((da_list_build_kernel<true>), g, dim3(256), 0, st, a);
  else hipLaunchKernelGGL((da_list_build_kernel<false>), g, dim3(256), 0, st, a);
  // a list slot counts its equal values from the lists
  hipLaunchKernelGGL((da_list_pass_kernel<2>), dim3((unsigned)((int64_t)n_workers * a.dnb)), dim3(256), 0, st, a);
  return check_launch("dauction_eqcount");
}

// bids of round `round` (rank_off[w]: equal-to-T values of worker w on lower ranks, device u32 [K])
int rqsid_dauction_bid(const uint16_t* scores, int32_t n_workers, int64_t n_local, int64_t n_global,
                       const uint32_t* rank_off, void* workspace, int64_t workspace_bytes, void* stream) {
  SegAuction a;
  int rc = dstate(a, scores, n_workers, n_local, n_global, workspace, workspace_bytes);
  if (rc) return rc;
  if (n_local == 0) return RQSID_OK;
  a.rank_off = rank_off;
  const dim3 g((unsigned)a.total_chunks, (unsigned)cdiv(n_workers, kKG));
  hipStream_t st = (hipStream_t)stream;
  if (dvec(scores, n_local)) hipLaunchKernelGGL((sa_bid_kernel<true>), g, dim3(256), 0, st, a);
  else hipLaunchKernelGGL((sa_bid_kernel<false>), g, dim3(256), 0, st, a);
  hipLaunchKernelGGL(da_list_rank_kernel, dim3((unsigned)n_workers), dim3(256), 0, st, a);
  hipLaunchKernelGGL((da_list_pass_kernel<3>), dim3((unsigned)((int64_t)n_workers * a.dnb)), dim3(256), 0, st, a);
  return check_launch("dauction_bid");
}

// winners and costs of this rank's jobs; the rank's count of jobs with a bidder goes to `have`
int rqsid_dauction_resolve(const uint16_t* scores, int32_t n_workers, int64_t n_local, int64_t n_global,
                           int32_t* out_assign, void* workspace, int64_t workspace_bytes, void* stream) {
  SegAuction a;
  int rc = dstate(a, scores, n_workers, n_local, n_global, workspace, workspace_bytes);
  if (rc) return rc;
  if (n_local == 0) return RQSID_OK;
  hipLaunchKernelGGL(sa_resolve_kernel, dim3((unsigned)a.total_chunks), dim3(256), 0, (hipStream_t)stream, a,
                     out_assign);
  return check_launch("dauction_resolve");
}

// end of a round, after the caller summed `have` over the ranks: done when it equals n_global
int rqsid_dauction_end_round(const uint16_t* scores, int32_t n_workers, int64_t n_local, int64_t n_global,
                             void* workspace, int64_t workspace_bytes, void* stream) {
  SegAuction a;
  int rc = dstate(a, scores, n_workers, n_local, n_global, workspace, workspace_bytes);
  if (rc) return rc;
  hipLaunchKernelGGL(da_round_end_kernel, dim3(1), dim3(256), 0, (hipStream_t)stream, a);
  return check_launch("dauction_end_round");
}

// diagnostics (tools/auction_bench.py --sharded with RQSID_DAUCTION_STATS=1): out u32[8] = {slot mode, round,
// max list entries, mean list entries, worker 0's lkb, worker 0's T, overflow word, lists over capacity}
__global__ void da_debug_kernel(SegAuction a, uint32_t* out) {
  uint64_t sum = 0;
  uint32_t mx = 0, over = 0;
  for (int w = 0; w < a.K; ++w) {
    const uint32_t n = a.lcnt[(int64_t)w * kAbovePad];
    sum += n;
    mx = n > mx ? n : mx;
    over += n > (uint32_t)a.dcap ? 1u : 0u;
  }
  out[0] = a.dmode[0];
  out[1] = (uint32_t)*a.round_dev;
  out[2] = mx;
  out[3] = (uint32_t)(sum / (uint64_t)a.K);
  out[4] = a.lkb[0];
  out[5] = a.sel[2];
  out[6] = a.hist[(int64_t)a.K * 256];
  out[7] = over;
}

int rqsid_dauction_debug(const uint16_t* scores, int32_t n_workers, int64_t n_local, int64_t n_global, uint32_t* out,
                         void* workspace, int64_t workspace_bytes, void* stream) {
  SegAuction a;
  int rc = dstate(a, scores, n_workers, n_local, n_global, workspace, workspace_bytes);
  if (rc) return rc;
  hipLaunchKernelGGL(da_debug_kernel, dim3(1), dim3(1), 0, (hipStream_t)stream, a, out);
  return check_launch("dauction_debug");
}

// the list kernels of one pass alone, for list-only slots (the sweep kernels of hist / eqcount / bid are not
// launched: at K = 2560 over 6.25M jobs each such launch costs ~0.2 ms of dispatch even when every block exits):
// step -1 starts the slot (a sweep slot turns void), 0 / 1 the histograms, 2 the equal-value counts, 3 the
// tie ranks and bids (rank_off as for rqsid_dauction_bid)
int rqsid_dauction_list_pass(const uint16_t* scores, int32_t n_workers, int64_t n_local, int64_t n_global, int32_t step,
                             const uint32_t* rank_off, void* workspace, int64_t workspace_bytes, void* stream) {
  SegAuction a;
  int rc = dstate(a, scores, n_workers, n_local, n_global, workspace, workspace_bytes);
  if (rc) return rc;
  if (step < -1 || step > 3) return fail(RQSID_E_ARG, "dauction_list_pass: step %d", step);
  hipStream_t st = (hipStream_t)stream;
  if (step == -1) {
    hipLaunchKernelGGL(da_slot_list_only_kernel, dim3(1), dim3(1), 0, st, a);
    return check_launch("dauction_list_pass");
  }
  if (n_local == 0) {
    if (step == 2 && fill_async(a.eqtot, 0, (size_t)n_workers * 4, st) != hipSuccess)
      return fail(RQSID_E_LAUNCH, "dauction: memset");
    return RQSID_OK;
  }
  const dim3 gl((unsigned)((int64_t)n_workers * a.dnb));
  a.rank_off = rank_off;
  if (step == 0) hipLaunchKernelGGL((da_list_pass_kernel<0>), gl, dim3(256), 0, st, a);
  else if (step == 1) hipLaunchKernelGGL((da_list_pass_kernel<1>), gl, dim3(256), 0, st, a);
  else if (step == 2) hipLaunchKernelGGL((da_list_pass_kernel<2>), gl, dim3(256), 0, st, a);
  else {
    hipLaunchKernelGGL(da_list_rank_kernel, dim3((unsigned)n_workers), dim3(256), 0, st, a);
    hipLaunchKernelGGL((da_list_pass_kernel<3>), gl, dim3(256), 0, st, a);
  }
  return check_launch("dauction_list_pass");
}

}  // extern "C"

#ifdef RQSID_STAMPS
extern "C" int rqsid_debug_al_stamps(unsigned long long* out16) {
  if (hipMemcpyFromSymbol(out16, HIP_SYMBOL(g_al_stamps), 16 * sizeof(unsigned long long)) != hipSuccess) return -1;
  unsigned long long z[16] = {};
  return hipMemcpyToSymbol(HIP_SYMBOL(g_al_stamps), z, sizeof(z)) == hipSuccess ? 0 : -1;
}
#endif
