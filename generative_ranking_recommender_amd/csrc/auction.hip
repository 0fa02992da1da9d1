// auction.hip — the balanced assignment of balancekmeans.auction_lap_half (balancekmeans/__init__.py:12-140,
// SURVEY.md §8a row A5) as a sequence of dense passes over the fp16 score matrix on gfx950.
//
// Reference round (workers w = clusters, jobs j = rows, W = fp16(-distance) stored worker-major):
//   value[w][j] = W[w][j] if (w, j) won the previous round, else fp16(W[w][j] - cost[j])
//   each worker bids on its top jobs_per_worker = N / K jobs of value (torch.topk(jpw + 1)):
//       bid = fp16(fp16(value - (jpw+1)-th largest value) + eps)
//   retention (round < 100): the previous winner of j bids exactly eps on j   (bids.view(-1)[index] = eps)
//   leftovers (round > 1000): worker 0 bids eps on every job that had no bidder last round
//   each job goes to its highest bidder; stop when every job has one; else cost[j] = fp16(cost[j] + bid)
//
// The only implementation-defined step of the reference is which of several EQUAL values torch.topk /
// torch.max keep at the selection boundary.  Here the rule is fixed and documented: among values equal
// to the (jpw+1)-th largest, the lowest job indices are kept; among equal highest bids, the lowest worker
// wins.  oracle/rq_oracle.py auction_lap_half(tie_rule="stable") restates exactly this rule and
// tests/test_gpu_auction.py checks the kernels against it bit for bit.
//
// Per round (all passes are coalesced sweeps over W; job-side state is read once per block of KG workers):
//   P1 histogram of the high byte of a 16-bit order key of value, per worker
//   P2 histogram of the low byte inside the selected high-byte bin -> exact threshold key T[w]
//   P3 per-(worker, job chunk) count of values equal to T[w] (tie ranks)
//   P4 bids + overwrites, reduced to one packed {fp16 bid, ~worker} atomicMax per job and block
//   P5 per job: winner, cost update, bookkeeping; count of jobs with a bidder
#include <cmath>

#include "internal.h"

namespace rqsid {
namespace {

constexpr int kKG = 16;                 // workers per block
constexpr int kChunkJobs = 4096;        // jobs per block (256 threads x 16 jobs)
constexpr int kJobsPerThread = kChunkJobs / 256;

__device__ __forceinline__ float h2f(uint16_t b) { return (float)__builtin_bit_cast(_Float16, b); }
__device__ __forceinline__ uint16_t f2h(float f) { return __builtin_bit_cast(uint16_t, (_Float16)f); }

// order key: larger value <-> larger key; -0 and +0 share a key (they compare equal)
__device__ __forceinline__ uint32_t okey(uint16_t b) {
  if (b == 0x8000u) b = 0;
  return (b & 0x8000u) ? (~b & 0xFFFFu) : (b | 0x8000u);
}
__device__ __forceinline__ uint16_t okey_inv(uint32_t k) {
  return (k & 0x8000u) ? (uint16_t)(k & 0x7FFFu) : (uint16_t)(~k & 0xFFFFu);
}

struct AuctionState {
  const uint16_t* W;  // [K][N] fp16 bits
  int32_t K;
  int64_t N;
  int32_t jpw;
  int64_t nchunks;
  uint16_t* cost;     // [N]
  int32_t* hb;        // [N] winner of the previous round (-1 none)
  uint8_t* nobid;     // [N] 1 = no bidder in the previous round
  uint32_t* key;      // [N] packed max bid of this round
  uint32_t* hist;     // [K][256]
  uint32_t* sel;      // [K][4]: b1 (high byte), rank inside the bin, T, need_eq
  uint32_t* eqcnt;    // [K][nchunks] -> exclusive offsets after the scan
  uint32_t* scal;     // [0]=eps bits, [1]=jobs with bidder, [2]=max key, [3]=min key
};

__device__ __forceinline__ uint16_t value_bits(const AuctionState& s, int w, int64_t j, uint16_t wv, int32_t hbj,
                                               uint16_t cj) {
  if (hbj == w) return wv;  // the previous round's winner keeps its raw score
  return f2h(h2f(wv) - h2f(cj));
}

// ---- eps: fp16((max - min) / 50), at least fp16(1e-4); min/max over the whole matrix ----
__global__ __launch_bounds__(256) void auction_minmax_kernel(const uint16_t* __restrict__ W, int64_t total,
                                                             uint32_t* __restrict__ scal) {
  uint32_t mx = 0, mn = 0xFFFFFFFFu;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
    const uint32_t k = okey(W[i]);
    mx = max(mx, k);
    mn = min(mn, k);
  }
  for (int o = 32; o > 0; o >>= 1) {
    mx = max(mx, (uint32_t)__shfl_xor((int)mx, o));
    mn = min(mn, (uint32_t)__shfl_xor((int)mn, o));
  }
  if ((threadIdx.x & 63) == 0) {
    atomicMax(&scal[2], mx);
    atomicMin(&scal[3], mn);
  }
}

__global__ void auction_eps_kernel(uint32_t* __restrict__ scal) {
  const float mx = h2f(okey_inv(scal[2])), mn = h2f(okey_inv(scal[3]));
  const uint16_t spread = f2h(mx - mn);          // fp16 op
  uint16_t eps = f2h(h2f(spread) / 50.0f);        // fp16 op
  const uint16_t floor_eps = f2h(1e-4f);
  if (!(h2f(eps) >= h2f(floor_eps))) eps = floor_eps;  // max(eps, 1e-4): the reference keeps eps unless it is smaller
  scal[0] = eps;
}

// ---- P1 / P2: per-worker histograms ----
template <bool LOW>
__global__ __launch_bounds__(256) void auction_hist_kernel(AuctionState s) {
  __shared__ uint32_t h[kKG][256];
  const int w0 = blockIdx.y * kKG;
  const int64_t j0 = (int64_t)blockIdx.x * kChunkJobs;
  for (int i = threadIdx.x; i < kKG * 256; i += 256) (&h[0][0])[i] = 0;
  __syncthreads();
  const int nw = min(kKG, s.K - w0);
  uint32_t b1[kKG];
  if (LOW)
    for (int g = 0; g < kKG; ++g) b1[g] = g < nw ? s.sel[(w0 + g) * 4 + 0] : 0;
  for (int t = 0; t < kJobsPerThread; ++t) {
    const int64_t j = j0 + t * 256 + threadIdx.x;
    if (j >= s.N) break;
    const int32_t hbj = s.hb[j];
    const uint16_t cj = s.cost[j];
    for (int g = 0; g < nw; ++g) {
      const int w = w0 + g;
      const uint32_t k = okey(value_bits(s, w, j, s.W[(int64_t)w * s.N + j], hbj, cj));
      if (!LOW) atomicAdd(&h[g][k >> 8], 1u);
      else if ((k >> 8) == b1[g]) atomicAdd(&h[g][k & 255], 1u);
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < nw * 256; i += 256) {
    const uint32_t c = (&h[0][0])[i];
    if (c) atomicAdd(&s.hist[(int64_t)(w0 + i / 256) * 256 + (i & 255)], c);
  }
}

// one thread per worker: walk the histogram from the top to the bin holding rank jpw+1
template <bool LOW>
__global__ void auction_select_kernel(AuctionState s) {
  const int w = blockIdx.x * blockDim.x + threadIdx.x;
  if (w >= s.K) return;
  uint32_t* h = s.hist + (int64_t)w * 256;
  uint32_t* sel = s.sel + w * 4;
  uint32_t rank = LOW ? sel[1] : (uint32_t)(s.jpw + 1);  // 1-based rank from the top inside the range
  uint32_t above = 0;
  int b = 255;
  for (; b > 0; --b) {
    if (above + h[b] >= rank) break;
    above += h[b];
  }
  if (!LOW) {
    sel[0] = (uint32_t)b;
    sel[1] = rank - above;
    sel[3] = above;  // count strictly above the bin (partial c_gt)
  } else {
    const uint32_t T = (sel[0] << 8) | (uint32_t)b;
    const uint32_t c_gt = sel[3] + above;   // values with key > T
    sel[2] = T;
    sel[3] = (uint32_t)s.jpw - c_gt;        // tied values at T kept in the top jpw
  }
  for (int i = 0; i < 256; ++i) h[i] = 0;   // ready for the next histogram
}

// ---- P3: count of values equal to T per (worker, chunk) ----
__global__ __launch_bounds__(256) void auction_eqcount_kernel(AuctionState s) {
  __shared__ uint32_t c[kKG];
  const int w0 = blockIdx.y * kKG;
  const int64_t j0 = (int64_t)blockIdx.x * kChunkJobs;
  if (threadIdx.x < kKG) c[threadIdx.x] = 0;
  __syncthreads();
  const int nw = min(kKG, s.K - w0);
  uint32_t T[kKG];
  for (int g = 0; g < kKG; ++g) T[g] = g < nw ? s.sel[(w0 + g) * 4 + 2] : 0xFFFFFFFFu;
  uint32_t cnt[kKG] = {};
  for (int t = 0; t < kJobsPerThread; ++t) {
    const int64_t j = j0 + t * 256 + threadIdx.x;
    if (j >= s.N) break;
    const int32_t hbj = s.hb[j];
    const uint16_t cj = s.cost[j];
    for (int g = 0; g < nw; ++g) {
      const int w = w0 + g;
      cnt[g] += okey(value_bits(s, w, j, s.W[(int64_t)w * s.N + j], hbj, cj)) == T[g];
    }
  }
  for (int g = 0; g < nw; ++g) {
    uint32_t v = cnt[g];
    for (int o = 32; o > 0; o >>= 1) v += (uint32_t)__shfl_xor((int)v, o);
    if ((threadIdx.x & 63) == 0 && v) atomicAdd(&c[g], v);
  }
  __syncthreads();
  if (threadIdx.x < nw) s.eqcnt[(int64_t)(w0 + threadIdx.x) * s.nchunks + blockIdx.x] = c[threadIdx.x];
}

// exclusive scan of eqcnt over chunks, one block per worker
__global__ __launch_bounds__(256) void auction_eqscan_kernel(AuctionState s) {
  __shared__ uint32_t carry;
  const int w = blockIdx.x;
  uint32_t* e = s.eqcnt + (int64_t)w * s.nchunks;
  if (threadIdx.x == 0) carry = 0;
  __syncthreads();
  for (int64_t base = 0; base < s.nchunks; base += 256) {
    const int64_t i = base + threadIdx.x;
    const uint32_t v = i < s.nchunks ? e[i] : 0;
    // block inclusive scan (wave scan + LDS)
    uint32_t x = v;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t y = (uint32_t)__shfl_up((int)x, o);
      if (lane >= o) x += y;
    }
    __shared__ uint32_t ws[4];
    if (lane == 63) ws[wv] = x;
    __syncthreads();
    uint32_t off = carry;
    for (int q = 0; q < wv; ++q) off += ws[q];
    if (i < s.nchunks) e[i] = off + x - v;
    __syncthreads();
    if (threadIdx.x == 255) carry = off + x;
    __syncthreads();
  }
}

// ---- P4: bids ----
__global__ __launch_bounds__(256) void auction_bid_kernel(AuctionState s, int counter) {
  __shared__ uint32_t wsum[kKG][4];
  const int w0 = blockIdx.y * kKG;
  const int64_t j0 = (int64_t)blockIdx.x * kChunkJobs;
  const int nw = min(kKG, s.K - w0);
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const uint16_t eps = (uint16_t)s.scal[0];
  const float epsf = h2f(eps);
  uint32_t T[kKG], need[kKG], off[kKG];
  float vT[kKG];
  for (int g = 0; g < kKG; ++g) {
    T[g] = g < nw ? s.sel[(w0 + g) * 4 + 2] : 0xFFFFFFFFu;
    need[g] = g < nw ? s.sel[(w0 + g) * 4 + 3] : 0;
    off[g] = g < nw ? s.eqcnt[(int64_t)(w0 + g) * s.nchunks + blockIdx.x] : 0;
    vT[g] = g < nw ? h2f(okey_inv(T[g])) : 0.f;
  }
  for (int t = 0; t < kJobsPerThread; ++t) {
    const int64_t j = j0 + t * 256 + threadIdx.x;
    const bool live = j < s.N;
    const int32_t hbj = live ? s.hb[j] : -1;
    const uint16_t cj = live ? s.cost[j] : 0;
    const bool nob = live && s.nobid[j];
    uint32_t best = 0;
    for (int g = 0; g < nw; ++g) {
      const int w = w0 + g;
      const uint16_t vb = live ? value_bits(s, w, j, s.W[(int64_t)w * s.N + j], hbj, cj) : 0;
      const uint32_t k = okey(vb);
      const bool eq = live && k == T[g];
      // rank of this job among the equal values of worker w, in job order (chunk offset + block prefix)
      const unsigned long long m = __ballot(eq);
      const uint32_t before_in_wave = __popcll(m & ((1ull << lane) - 1ull));
      if (lane == 0) wsum[g][wv] = __popcll(m);
      __syncthreads();
      uint32_t before = off[g] + before_in_wave;
      for (int q = 0; q < wv; ++q) before += wsum[g][q];
      const uint32_t tot = wsum[g][0] + wsum[g][1] + wsum[g][2] + wsum[g][3];
      __syncthreads();
      off[g] += tot;
      uint16_t bid = 0;
      if (live && k > T[g]) {
        bid = f2h(h2f(f2h(h2f(vb) - vT[g])) + epsf);
      } else if (eq && before < need[g]) {
        bid = f2h(0.0f + epsf);
      }
      if (counter < 100 && hbj == w) bid = eps;   // retention bid of the previous winner
      if (counter > 1000 && w == 0 && nob) bid = eps;  // leftovers go to worker 0
      if (bid) {
        const uint32_t pk = ((uint32_t)bid << 16) | (0xFFFFu - (uint32_t)w);
        best = max(best, pk);
      }
    }
    if (best) atomicMax(&s.key[j], best);
  }
}

// ---- P5: resolve ----
__global__ __launch_bounds__(256) void auction_resolve_kernel(AuctionState s, int32_t* __restrict__ out) {
  uint32_t cnt = 0;
  for (int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x; j < s.N; j += (int64_t)gridDim.x * 256) {
    const uint32_t k = s.key[j];
    s.key[j] = 0;
    if (k) {
      const int32_t w = (int32_t)(0xFFFFu - (k & 0xFFFFu));
      const uint16_t bid = (uint16_t)(k >> 16);
      out[j] = w;
      s.hb[j] = w;
      s.nobid[j] = 0;
      s.cost[j] = f2h(h2f(s.cost[j]) + h2f(bid));
      ++cnt;
    } else {
      out[j] = -1;
      s.hb[j] = -1;
      s.nobid[j] = 1;
    }
  }
  for (int o = 32; o > 0; o >>= 1) cnt += (uint32_t)__shfl_xor((int)cnt, o);
  if ((threadIdx.x & 63) == 0 && cnt) atomicAdd(&s.scal[1], cnt);
}

__global__ void auction_init_kernel(AuctionState s) {
  for (int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x; j < s.N; j += (int64_t)gridDim.x * 256) {
    s.cost[j] = 0;
    s.hb[j] = -1;
    s.nobid[j] = 0;
    s.key[j] = 0;
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    s.scal[1] = 0;
    s.scal[2] = 0;
    s.scal[3] = 0xFFFFFFFFu;
  }
}

// argmin over workers of W for N < K (the reference's fallback returns torch.argmin(-D) = the FARTHEST
// centre, balancekmeans/__init__.py:24-26; with W = -D that is the argmin of W)
__global__ void auction_fallback_kernel(const uint16_t* __restrict__ W, int K, int64_t N, int32_t* __restrict__ out) {
  for (int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x; j < N; j += (int64_t)gridDim.x * 256) {
    float best = INFINITY;
    int bw = 0;
    for (int w = 0; w < K; ++w) {
      const float v = h2f(W[(int64_t)w * N + j]);
      if (v < best) { best = v; bw = w; }
    }
    out[j] = bw;
  }
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

int64_t auction_ws(int64_t N, int32_t K) {
  const int64_t nch = (N + kChunkJobs - 1) / kChunkJobs;
  Carve c{nullptr};
  c.take<uint16_t>(N);
  c.take<int32_t>(N);
  c.take<uint8_t>(N);
  c.take<uint32_t>(N);
  c.take<uint32_t>((int64_t)K * 256);
  c.take<uint32_t>((int64_t)K * 4);
  c.take<uint32_t>((int64_t)K * nch);
  c.take<uint32_t>(8);
  return c.used;
}

}  // namespace
}  // namespace rqsid

using namespace rqsid;

extern "C" {

int64_t rqsid_auction_workspace_bytes(int64_t n_jobs, int32_t n_workers) {
  if (n_jobs < 0 || n_workers <= 0) return -1;
  return auction_ws(n_jobs, n_workers);
}

int rqsid_auction_lap_half(const uint16_t* scores_wj, int32_t n_workers, int64_t n_jobs, int32_t max_rounds,
                           int32_t* out_assign, int32_t* out_rounds, void* workspace, int64_t workspace_bytes,
                           void* stream) {
  if (!scores_wj || !out_assign || n_workers <= 0 || n_jobs < 0 || n_jobs > INT32_MAX)
    return fail(RQSID_E_ARG, "auction: bad arguments (K=%d N=%lld)", n_workers, (long long)n_jobs);
  if (!workspace || workspace_bytes < auction_ws(n_jobs, n_workers))
    return fail(RQSID_E_WORKSPACE, "auction: workspace too small");
  hipStream_t st = (hipStream_t)stream;
  if (out_rounds) *out_rounds = 0;
  if (n_jobs == 0) return RQSID_OK;
  if (n_jobs < n_workers) {
    hipLaunchKernelGGL(auction_fallback_kernel, dim3(grid_cap(cdiv(n_jobs, 256), 4096)), dim3(256), 0, st,
                       scores_wj, n_workers, n_jobs, out_assign);
    return check_launch("auction_fallback");
  }
  if (n_workers == 1) {  // torch.topk(N + 1) would raise in the reference
    return fail(RQSID_E_ARG, "auction: a single worker cannot bid on N + 1 jobs");
  }
  AuctionState s{};
  s.W = scores_wj;
  s.K = n_workers;
  s.N = n_jobs;
  s.jpw = (int32_t)(n_jobs / n_workers);
  s.nchunks = (n_jobs + kChunkJobs - 1) / kChunkJobs;
  Carve c{(char*)workspace};
  s.cost = c.take<uint16_t>(n_jobs);
  s.hb = c.take<int32_t>(n_jobs);
  s.nobid = c.take<uint8_t>(n_jobs);
  s.key = c.take<uint32_t>(n_jobs);
  s.hist = c.take<uint32_t>((int64_t)n_workers * 256);
  s.sel = c.take<uint32_t>((int64_t)n_workers * 4);
  s.eqcnt = c.take<uint32_t>((int64_t)n_workers * s.nchunks);
  s.scal = c.take<uint32_t>(8);
  int rc;
  const unsigned gj = grid_cap(cdiv(n_jobs, 256), 8192);
  if (hipMemsetAsync(s.hist, 0, (size_t)n_workers * 256 * 4, st) != hipSuccess)
    return fail(RQSID_E_LAUNCH, "auction: memset");
  hipLaunchKernelGGL(auction_init_kernel, dim3(gj), dim3(256), 0, st, s);
  hipLaunchKernelGGL(auction_minmax_kernel, dim3(grid_cap(cdiv(n_jobs * n_workers, 256 * 16), 8192)), dim3(256), 0,
                     st, scores_wj, n_jobs * n_workers, s.scal);
  hipLaunchKernelGGL(auction_eps_kernel, dim3(1), dim3(1), 0, st, s.scal);
  if ((rc = check_launch("auction_init"))) return rc;
  const dim3 g2((unsigned)s.nchunks, (unsigned)cdiv(n_workers, kKG));
  const unsigned gsel = (unsigned)cdiv(n_workers, 64);
  for (int round = 0; max_rounds <= 0 || round < max_rounds; ++round) {
    hipLaunchKernelGGL((auction_hist_kernel<false>), g2, dim3(256), 0, st, s);
    hipLaunchKernelGGL((auction_select_kernel<false>), dim3(gsel), dim3(64), 0, st, s);
    hipLaunchKernelGGL((auction_hist_kernel<true>), g2, dim3(256), 0, st, s);
    hipLaunchKernelGGL((auction_select_kernel<true>), dim3(gsel), dim3(64), 0, st, s);
    hipLaunchKernelGGL(auction_eqcount_kernel, g2, dim3(256), 0, st, s);
    hipLaunchKernelGGL(auction_eqscan_kernel, dim3((unsigned)n_workers), dim3(256), 0, st, s);
    hipLaunchKernelGGL(auction_bid_kernel, g2, dim3(256), 0, st, s, round);
    if (hipMemsetAsync(s.scal + 1, 0, 4, st) != hipSuccess) return fail(RQSID_E_LAUNCH, "auction: memset");
    hipLaunchKernelGGL(auction_resolve_kernel, dim3(gj), dim3(256), 0, st, s, out_assign);
    if ((rc = check_launch("auction_round"))) return rc;
    uint32_t have = 0;
    if (hipMemcpyAsync(&have, s.scal + 1, 4, hipMemcpyDeviceToHost, st) != hipSuccess ||
        hipStreamSynchronize(st) != hipSuccess)
      return fail(RQSID_E_LAUNCH, "auction: readback");
    if (out_rounds) *out_rounds = round + 1;
    if ((int64_t)have == n_jobs) return RQSID_OK;
  }
  return fail(RQSID_E_LAUNCH, "auction: no complete assignment after %d rounds", max_rounds);
}

}  // extern "C"
