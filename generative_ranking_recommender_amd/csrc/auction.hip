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
// tests/test_gpu_training.py and tests/test_gpu_batched.py check the kernels against it bit for bit.
//
// The passes (auction_seg.hip; all are coalesced sweeps over W, job-side state read once per block of
// 16 workers), per round:
//   P1 histogram of the high byte of a 16-bit order key of value, per worker
//   P2 histogram of the low byte inside the selected high-byte bin -> exact threshold key T[w]
//   P3 per-(worker, job chunk) count of values equal to T[w] (tie ranks)
//   P4 bids + overwrites, reduced to one packed {fp16 bid, ~worker} atomicMax per job and block
//   P5 per job: winner, cost update, bookkeeping; count of jobs with a bidder
#include <cmath>
#include <cstring>

#include "internal.h"

using namespace rqsid;

namespace {
constexpr int64_t kSmallAlign = 256;

__global__ void single_layout_kernel(int32_t* seg_off, int32_t* chunk_off, int32_t n, int32_t nch) {
  seg_off[0] = 0;
  seg_off[1] = n;
  chunk_off[0] = 0;
  chunk_off[1] = nch;
}

int64_t single_ws(int64_t n_jobs, int32_t n_workers) {
  const int64_t ch = rqsid_seg_auction_chunk_jobs();
  const int64_t nch = (n_jobs + ch - 1) / ch;
  return 3 * kSmallAlign + rqsid_seg_auction_workspace_bytes(n_jobs, n_workers, 1, nch, nch > 1 ? 1 : 0);
}
// ---- auction_lap_full: the fp32 auction (balancekmeans/__init__.py:142-210) ----------------------------
// Reached only through KMeans.predict(balanced=True) (:523-525): kept simple.  One 1024-thread block per
// worker finds its (jpw+1)-th largest value by a 4-digit radix select over the 32-bit order keys of
// value = W - cost (W for the jobs it won last round), then bids in job order: (v - T) + eps above T, eps
// for the first `need` jobs equal to T (lowest job index, the oracle's stable rule), eps retention bids
// before round 100, eps leftover bids of worker 0 after round 1000.  A per-job pass resolves the highest
// bid (equal bids: lowest worker) and adds it to the job's cost, all in fp32 as the reference.
struct FullAuction {
  const float* W;
  int32_t K;
  int64_t N;
  int64_t jpw;
  float* cost;
  int32_t* hb;
  uint8_t* nobid;
  unsigned long long* key;
  uint32_t* have;
  uint32_t* mm;  // [2] max, min order keys of W
};

__device__ __forceinline__ uint32_t fkey(float f) {
  uint32_t b = __float_as_uint(f);
  if (b == 0x80000000u) b = 0;  // -0 orders as +0
  return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
}
__device__ __forceinline__ float fkey_inv(uint32_t k) {
  return __uint_as_float((k & 0x80000000u) ? (k & 0x7FFFFFFFu) : ~k);
}
__device__ __forceinline__ float full_value(const FullAuction& a, int w, int64_t j) {
  const float s = a.W[(int64_t)w * a.N + j];
  return a.hb[j] == w ? s : s - a.cost[j];
}

__global__ __launch_bounds__(256) void full_init_kernel(FullAuction a) {
  for (int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x; j < a.N; j += (int64_t)gridDim.x * 256) {
    a.cost[j] = 0.f;
    a.hb[j] = -1;
    a.nobid[j] = 0;
    a.key[j] = 0ull;
  }
}

__global__ __launch_bounds__(256) void full_minmax_kernel(FullAuction a) {
  uint32_t mx = 0, mn = 0xFFFFFFFFu;
  const int64_t total = (int64_t)a.K * a.N;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
    const uint32_t k = fkey(a.W[i]);
    mx = max(mx, k);
    mn = min(mn, k);
  }
  for (int o = 32; o > 0; o >>= 1) {
    mx = max(mx, (uint32_t)__shfl_xor((int)mx, o));
    mn = min(mn, (uint32_t)__shfl_xor((int)mn, o));
  }
  if ((threadIdx.x & 63) == 0) {
    atomicMax(&a.mm[0], mx);
    atomicMin(&a.mm[1], mn);
  }
}

__global__ __launch_bounds__(1024) void full_bid_kernel(FullAuction a, int counter, float eps) {
  const int w = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  __shared__ uint32_t hist[256];
  __shared__ uint32_t s_digit, s_rank;
  __shared__ uint32_t wcnt[16];
  uint32_t prefix = 0, rank = (uint32_t)(a.jpw + 1), c_gt = 0;
  for (int pass = 0; pass < 4; ++pass) {
    const int shift = 24 - 8 * pass;
    for (int i = tid; i < 256; i += 1024) hist[i] = 0;
    __syncthreads();
    for (int64_t j = tid; j < a.N; j += 1024) {
      const uint32_t k = fkey(full_value(a, w, j));
      if (pass == 0 || (k >> (shift + 8)) == (prefix >> (shift + 8))) atomicAdd(&hist[(k >> shift) & 255u], 1u);
    }
    __syncthreads();
    if (tid == 0) {
      uint32_t acc = 0;
      int b = 255;
      for (; b > 0; --b) {
        if (acc + hist[b] >= rank) break;
        acc += hist[b];
      }
      s_digit = (uint32_t)b;
      s_rank = rank - acc;
      c_gt += acc;
    }
    __syncthreads();
    prefix |= s_digit << shift;
    rank = s_rank;
    __syncthreads();
  }
  __shared__ uint32_t s_cgt;
  if (tid == 0) s_cgt = c_gt;  // values above T (thread 0 ran the selection walks)
  __syncthreads();
  const uint32_t T = prefix;
  const float vT = fkey_inv(T);
  const int64_t need = a.jpw - (int64_t)s_cgt;
  const unsigned long long lt = (1ull << lane) - 1ull;
  int64_t run = 0;  // values equal to T at lower jobs
  for (int64_t base = 0; base < a.N; base += 1024) {
    const int64_t j = base + tid;
    const bool live = j < a.N;
    const float v = live ? full_value(a, w, j) : 0.f;
    const uint32_t k = live ? fkey(v) : 0u;
    const bool gt = live && k > T, eq = live && k == T;
    const unsigned long long m = __ballot(eq);
    if (lane == 0) wcnt[wv] = (uint32_t)__popcll(m);
    __syncthreads();
    uint32_t below = 0, total = 0;
    for (int q = 0; q < 16; ++q) {
      below += q < wv ? wcnt[q] : 0u;
      total += wcnt[q];
    }
    __syncthreads();
    float bid = 0.f;
    if (gt) bid = (v - vT) + eps;
    else if (eq && run + below + (uint32_t)__popcll(m & lt) < need) bid = (v - vT) + eps;
    if (counter < 100 && live && a.hb[j] == w) bid = eps;
    if (counter > 1000 && w == 0 && live && a.nobid[j]) bid = eps;
    if (bid > 0.f) atomicMax(&a.key[j], ((unsigned long long)__float_as_uint(bid) << 16) | (0xFFFFu - (uint32_t)w));
    run += total;
  }
}

__global__ __launch_bounds__(256) void full_resolve_kernel(FullAuction a, int32_t* __restrict__ out) {
  uint32_t cnt = 0;
  for (int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x; j < a.N; j += (int64_t)gridDim.x * 256) {
    const unsigned long long k = a.key[j];
    a.key[j] = 0ull;
    if (k) {
      const int32_t w = (int32_t)(0xFFFFu - (uint32_t)(k & 0xFFFFu));
      out[j] = w;
      a.hb[j] = w;
      a.nobid[j] = 0;
      a.cost[j] = a.cost[j] + __uint_as_float((uint32_t)(k >> 16));
      ++cnt;
    } else {
      out[j] = -1;
      a.hb[j] = -1;
      a.nobid[j] = 1;
    }
  }
  __shared__ uint32_t wc[4];
  for (int o = 32; o > 0; o >>= 1) cnt += (uint32_t)__shfl_xor((int)cnt, o);
  if ((threadIdx.x & 63) == 0) wc[threadIdx.x >> 6] = cnt;
  __syncthreads();
  if (threadIdx.x == 0 && (wc[0] + wc[1] + wc[2] + wc[3])) atomicAdd(a.have, wc[0] + wc[1] + wc[2] + wc[3]);
}

int64_t full_ws(int64_t n) {
  auto al = [](int64_t b) { return (b + 255) / 256 * 256; };
  return al(n * 4) + al(n * 4) + al(n) + al(n * 8) + 256 + 256;
}
}  // namespace

extern "C" {

int64_t rqsid_auction_full_workspace_bytes(int64_t n_jobs, int32_t n_workers) {
  if (n_jobs < 0 || n_workers <= 0) return -1;
  return full_ws(n_jobs);
}

int rqsid_auction_lap_full(const float* scores_wj, int32_t n_workers, int64_t n_jobs, int32_t max_rounds,
                           int32_t* out_assign, int32_t* out_rounds, void* workspace, int64_t workspace_bytes,
                           void* stream) {
  if (!scores_wj || !out_assign || n_workers <= 0 || n_workers > 65535 || n_jobs <= 0 || n_jobs > INT32_MAX)
    return fail(RQSID_E_ARG, "auction_full: bad arguments (K=%d N=%lld)", n_workers, (long long)n_jobs);
  if (n_workers == 1)  // torch.topk(N + 1) would raise in the reference
    return fail(RQSID_E_ARG, "auction_full: a single worker cannot bid on N + 1 jobs");
  if (!workspace || workspace_bytes < full_ws(n_jobs)) return fail(RQSID_E_WORKSPACE, "auction_full: workspace too small");
  hipStream_t st = (hipStream_t)stream;
  if (out_rounds) *out_rounds = 0;
  if (n_jobs < n_workers) {
    // jobs_per_worker = 0: topk(1) leaves no bid increments, so nothing bids until the leftover rule
    // (:182-183) hands every job to worker 0 in round 1002.  The result is known without the rounds.
    if (max_rounds > 0 && max_rounds < 1002)
      return fail(RQSID_E_LAUNCH, "auction_full: no complete assignment after %d rounds", max_rounds);
    if (fill_async(out_assign, 0, (size_t)n_jobs * 4, st) != hipSuccess)
      return fail(RQSID_E_LAUNCH, "auction_full: memset");
    if (out_rounds) *out_rounds = 1002;
    return RQSID_OK;
  }
  auto al = [](int64_t b) { return (b + 255) / 256 * 256; };
  char* p = (char*)workspace;
  FullAuction a{};
  a.W = scores_wj;
  a.K = n_workers;
  a.N = n_jobs;
  a.jpw = n_jobs / n_workers;
  a.cost = (float*)p;
  p += al(n_jobs * 4);
  a.hb = (int32_t*)p;
  p += al(n_jobs * 4);
  a.nobid = (uint8_t*)p;
  p += al(n_jobs);
  a.key = (unsigned long long*)p;
  p += al(n_jobs * 8);
  a.have = (uint32_t*)p;
  p += 256;
  a.mm = (uint32_t*)p;
  const unsigned gj = grid_cap(cdiv(n_jobs, 256), 4096);
  uint32_t mm_init[2] = {0u, 0xFFFFFFFFu};
  if (hipMemcpyAsync(a.mm, mm_init, 8, hipMemcpyHostToDevice, st) != hipSuccess)
    return fail(RQSID_E_LAUNCH, "auction_full: init");
  hipLaunchKernelGGL(full_init_kernel, dim3(gj), dim3(256), 0, st, a);
  hipLaunchKernelGGL(full_minmax_kernel, dim3(grid_cap(cdiv((int64_t)n_workers * n_jobs, 256), 4096)), dim3(256), 0,
                     st, a);
  uint32_t mm[2];
  int rc = check_launch("auction_full_init");
  if (rc) return rc;
  if (hipMemcpyAsync(mm, a.mm, 8, hipMemcpyDeviceToHost, st) != hipSuccess || hipStreamSynchronize(st) != hipSuccess)
    return fail(RQSID_E_LAUNCH, "auction_full: readback");
  // eps = (max - min) / 50 in fp32, clamped below at fp32(1e-4) (:150-151)
  auto inv = [](uint32_t k) {
    const uint32_t b = (k & 0x80000000u) ? (k & 0x7FFFFFFFu) : ~k;
    float f;
    std::memcpy(&f, &b, 4);
    return f;
  };
  const float spread = inv(mm[0]) - inv(mm[1]);
  float eps = spread / 50.0f;
  if (!(eps >= 1e-4f)) eps = 1e-4f;
  for (int round = 0;; ++round) {
    if (max_rounds > 0 && round >= max_rounds)
      return fail(RQSID_E_LAUNCH, "auction_full: no complete assignment after %d rounds", max_rounds);
    if (fill_async(a.have, 0, 4, st) != hipSuccess) return fail(RQSID_E_LAUNCH, "auction_full: memset");
    hipLaunchKernelGGL(full_bid_kernel, dim3((unsigned)n_workers), dim3(1024), 0, st, a, round, eps);
    hipLaunchKernelGGL(full_resolve_kernel, dim3(gj), dim3(256), 0, st, a, out_assign);
    if ((rc = check_launch("auction_full_round"))) return rc;
    uint32_t have = 0;
    if (hipMemcpyAsync(&have, a.have, 4, hipMemcpyDeviceToHost, st) != hipSuccess ||
        hipStreamSynchronize(st) != hipSuccess)
      return fail(RQSID_E_LAUNCH, "auction_full: readback");
    if ((int64_t)have == n_jobs) {
      if (out_rounds) *out_rounds = round + 1;
      return RQSID_OK;
    }
  }
}

int64_t rqsid_auction_workspace_bytes(int64_t n_jobs, int32_t n_workers) {
  if (n_jobs < 0 || n_workers <= 0) return -1;
  return single_ws(n_jobs, n_workers);
}

// One auction = the segmented auction (auction_seg.hip) over a single segment: the same kernels, the
// same graph-captured round blocks.
int rqsid_auction_lap_half(const uint16_t* scores_wj, int32_t n_workers, int64_t n_jobs, int32_t max_rounds,
                           int32_t* out_assign, int32_t* out_rounds, void* workspace, int64_t workspace_bytes,
                           void* stream) {
  if (!scores_wj || !out_assign || n_workers <= 0 || n_jobs < 0 || n_jobs > INT32_MAX)
    return fail(RQSID_E_ARG, "auction: bad arguments (K=%d N=%lld)", n_workers, (long long)n_jobs);
  if (!workspace || workspace_bytes < single_ws(n_jobs, n_workers))
    return fail(RQSID_E_WORKSPACE, "auction: workspace too small");
  hipStream_t st = (hipStream_t)stream;
  if (out_rounds) *out_rounds = 0;
  if (n_jobs == 0) return RQSID_OK;
  if (n_workers == 1 && n_jobs >= 1)  // torch.topk(N + 1) would raise in the reference
    return fail(RQSID_E_ARG, "auction: a single worker cannot bid on N + 1 jobs");
  const int64_t ch = rqsid_seg_auction_chunk_jobs();
  const int64_t nch = (n_jobs + ch - 1) / ch;
  char* p = (char*)workspace;
  int32_t* seg_off = (int32_t*)p;
  int32_t* chunk_off = (int32_t*)(p + kSmallAlign);
  int32_t* rounds_dev = (int32_t*)(p + 2 * kSmallAlign);
  hipLaunchKernelGGL(single_layout_kernel, dim3(1), dim3(1), 0, st, seg_off, chunk_off, (int32_t)n_jobs,
                     (int32_t)nch);
  int rc = check_launch("auction_layout");
  if (rc) return rc;
  rc = seg_auction_run(scores_wj, n_workers, 1, seg_off, chunk_off, nch, nch > 1 ? 1 : 0, n_jobs, nullptr,
                       max_rounds, out_assign, rounds_dev, p + 3 * kSmallAlign, workspace_bytes - 3 * kSmallAlign,
                       stream, true, /*single_layout=*/true);
  if (rc) return rc;
  int32_t r = 0;
  if (hipMemcpyAsync(&r, rounds_dev, 4, hipMemcpyDeviceToHost, st) != hipSuccess ||
      hipStreamSynchronize(st) != hipSuccess)
    return fail(RQSID_E_LAUNCH, "auction: readback");
  if (out_rounds) *out_rounds = r;
  return RQSID_OK;
}

}  // extern "C"
