// rqsid.hip — MI355X (gfx950 / CDNA4) kernels for hierarchical residual-quantisation K-Means
// semantic IDs, behind the C ABI declared in include/rqsid.h: row bucketing, residuals (A14), group
// weights (A15), the Lloyd centroid update (A10), match-matrix candidate lists and the dense
// distance matrix.  The assignment kernels (A2/A4/A11-A13/A18) live in assign.hip.
#include <hip/hip_runtime.h>

#include <climits>
#include <cmath>
#include <cstdarg>
#include <cstdint>
#include <cstdio>

#include "internal.h"

namespace rqsid {

thread_local char g_err[512] = "";

int fail(int code, const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
  return code;
}

int check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail(RQSID_E_LAUNCH, "%s: %s", what, hipGetErrorString(e));
  return RQSID_OK;
}

namespace {
__global__ __launch_bounds__(256) void fill_words_kernel(uint32_t* __restrict__ p, int64_t n, uint32_t v) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) p[i] = v;
}
__global__ __launch_bounds__(256) void fill_bytes_kernel(uint8_t* __restrict__ p, int64_t n, uint8_t v) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) p[i] = v;
}
}  // namespace

hipError_t fill_async(void* p, int value, size_t bytes, hipStream_t st) {
  static const bool api = [] {
    const char* e = getenv("RQSID_MEMSET_API");
    return e && atoi(e) != 0;
  }();
  if (api) return hipMemsetAsync(p, value, bytes, st);
  if (bytes == 0) return hipSuccess;
  const uint8_t b = (uint8_t)value;
  if (((uintptr_t)p & 3) == 0 && (bytes & 3) == 0) {
    const int64_t n = (int64_t)(bytes / 4);
    hipLaunchKernelGGL(fill_words_kernel, dim3(grid_cap(cdiv(n, 256), 1024)), dim3(256), 0, st, (uint32_t*)p, n,
                       0x01010101u * b);
  } else {
    const int64_t n = (int64_t)bytes;
    hipLaunchKernelGGL(fill_bytes_kernel, dim3(grid_cap(cdiv(n, 256), 1024)), dim3(256), 0, st, (uint8_t*)p, n, b);
  }
  return hipGetLastError();
}

namespace {
constexpr int kAccTileRows = 256;  // rows per centroid-accumulate tile
constexpr int kBucketLdsBins = 16384;
}  // namespace
// ---------------------------------------------------------------------------
// bucketing (counting sort of rows by segment key)
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void bucket_hist_kernel(const int32_t* __restrict__ keys, int64_t n,
                                                          int S, int32_t* __restrict__ counts) {
  extern __shared__ __attribute__((aligned(16))) int32_t lh[];
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  if (S <= kBucketLdsBins) {
    for (int b = threadIdx.x; b < S; b += blockDim.x) lh[b] = 0;
    __syncthreads();
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
      const unsigned k = (unsigned)keys[i];
      if (k < (unsigned)S) atomicAdd(&lh[k], 1);
    }
    __syncthreads();
    for (int b = threadIdx.x; b < S; b += blockDim.x)
      if (lh[b]) atomicAdd(&counts[b], lh[b]);
  } else {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
      const unsigned k = (unsigned)keys[i];
      if (k < (unsigned)S) atomicAdd(&counts[k], 1);
    }
  }
}

// One block: exclusive scans of counts and ceil(counts / tile_rows).  Thread t owns the contiguous run of
// ceil(S / 1024) keys starting at t * run: it sums its run, the block scans the 1024 run sums, and the thread
// writes its run's offsets (one pass of the block scan instead of one per 1024 keys: 160 -> ~5 us at S = 65536).
__global__ __launch_bounds__(1024) void bucket_scan_kernel(const int32_t* __restrict__ counts, int S,
                                                           int tile_rows, int32_t* __restrict__ row_off,
                                                           int32_t* __restrict__ tile_off,
                                                           int32_t* __restrict__ cursor) {
  __shared__ int32_t sa[1024], sb[1024];
  const int t = threadIdx.x;
  const int run = (S + 1023) / 1024;
  const int k0 = t * run < S ? t * run : S, k1 = k0 + run < S ? k0 + run : S;
  int32_t a = 0, b = 0;
  for (int k = k0; k < k1; ++k) {
    const int32_t c = counts[k];
    a += c;
    b += tile_rows > 0 ? (c + tile_rows - 1) / tile_rows : 0;
  }
  sa[t] = a;
  sb[t] = b;
  __syncthreads();
  for (int o = 1; o < 1024; o <<= 1) {
    const int32_t va = t >= o ? sa[t - o] : 0;
    const int32_t vb = t >= o ? sb[t - o] : 0;
    __syncthreads();
    sa[t] += va;
    sb[t] += vb;
    __syncthreads();
  }
  int32_t ea = sa[t] - a, eb = sb[t] - b;
  for (int k = k0; k < k1; ++k) {
    const int32_t c = counts[k];
    row_off[k] = ea;
    if (tile_off) tile_off[k] = eb;
    if (cursor) cursor[k] = ea;
    ea += c;
    eb += tile_rows > 0 ? (c + tile_rows - 1) / tile_rows : 0;
  }
  if (t == 1023) {
    row_off[S] = sa[1023];
    if (tile_off) tile_off[S] = sb[1023];
  }
}

constexpr int kScatterRowsPerBlock = 8192;

// Every row_index write takes its position from a device counter (cursor[k], or the block's LDS copy of it).
// The position is checked against the key's segment [row_off[k], row_off[k+1]) before the store: a count that
// went wrong (a stale cursor, a key changed between the histogram and the scatter) drops the write and raises
// bit kBucketErrScatter of the sticky error word instead of writing outside the segment or past row_index.
constexpr int kBucketErrScatter = 1;
__device__ __forceinline__ void bucket_put(int32_t pos, unsigned k, int64_t i, const int32_t* __restrict__ row_off,
                                           int32_t* __restrict__ row_index, int32_t* __restrict__ err) {
  if (pos >= row_off[k] && pos < row_off[k + 1]) row_index[pos] = (int32_t)i;
  else atomicOr(err, kBucketErrScatter);
}
__global__ __launch_bounds__(256) void bucket_scatter_kernel(const int32_t* __restrict__ keys, int64_t n,
                                                             int S, int32_t* __restrict__ cursor,
                                                             const int32_t* __restrict__ row_off,
                                                             int32_t* __restrict__ row_index, int32_t* __restrict__ err,
                                                             int64_t rows_per_block) {
  extern __shared__ __attribute__((aligned(16))) int32_t lh[];
  if (S <= kBucketLdsBins) {
    const int64_t r0 = (int64_t)blockIdx.x * rows_per_block;
    const int64_t r1 = r0 + rows_per_block < n ? r0 + rows_per_block : n;
    for (int b = threadIdx.x; b < S; b += blockDim.x) lh[b] = 0;
    __syncthreads();
    for (int64_t i = r0 + threadIdx.x; i < r1; i += blockDim.x) {
      const unsigned k = (unsigned)keys[i];
      if (k < (unsigned)S) atomicAdd(&lh[k], 1);
    }
    __syncthreads();
    for (int b = threadIdx.x; b < S; b += blockDim.x) {
      const int32_t c = lh[b];
      if (c) lh[b] = atomicAdd(&cursor[b], c);
    }
    __syncthreads();
    for (int64_t i = r0 + threadIdx.x; i < r1; i += blockDim.x) {
      const unsigned k = (unsigned)keys[i];
      if (k >= (unsigned)S) continue;
      bucket_put(atomicAdd(&lh[k], 1), k, i, row_off, row_index, err);
    }
  } else {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
      const unsigned k = (unsigned)keys[i];
      if (k >= (unsigned)S) continue;
      bucket_put(atomicAdd(&cursor[k], 1), k, i, row_off, row_index, err);
    }
  }
}

// Up to 262144 keys: a count matrix instead of device-wide atomics.  The rows split into B chunks
// (B x S <= 4M words, B <= 256) and the keys into slices of kBucketLdsBins; block (b, s) counts chunk b's keys
// of slice s in LDS and stores them as row b of the matrix (no atomics outside LDS), a column scan turns each
// column into the chunks' exclusive prefixes and the key's total (and sums each 64 keys), the offsets kernel
// scans the totals (each 64-key block adds the sums of the blocks before it: no one-block serial scan), and the
// scatter block (b, s) starts each key of its slice at row_off[k] + prefix[b][k].  The global-atomic form
// (S > 16384) cost 235 + 277 us at 6.25M rows over 65536 keys (the XL last level), plus 160 us of one-block
// scan; the LDS-histogram form flushes ~S global atomics per block.  Blocks of one chunk share an XCD (B is a
// multiple of 8) and so its keys; 1024 threads with kBucketUnroll keys in flight each hide the load latency of
// the few blocks (B x slices).
constexpr int64_t kBucketMatrixWords = int64_t(1) << 22;
constexpr int kBucketUnroll = 8;
// chunks of the count matrix for S keys (S <= 262144; more keys take the global-atomic form): at most
// bucket_max_chunks(S) (the workspace's matrix), and ~32K rows per chunk for small inputs (at least 8 chunks), so
// the column scan of a 100k-row call reads 8 rows of the matrix, not 256
inline int bucket_max_chunks(int S) {
  return S > 262144 ? 0 : (int)std::min<int64_t>(256, kBucketMatrixWords / S) / 8 * 8;
}
inline int bucket_chunks(int64_t n, int S) {
  if (n <= 0) return 0;
  const int64_t want = std::max<int64_t>(8, cdiv(n, 32768) / 8 * 8);
  return (int)std::min<int64_t>(bucket_max_chunks(S), want);
}

__global__ __launch_bounds__(1024) void bucket_chunk_hist_kernel(const int32_t* __restrict__ keys, int64_t n, int S,
                                                                 int64_t chunk_rows, int32_t* __restrict__ mat) {
  extern __shared__ __attribute__((aligned(16))) int32_t lh[];
  const int b0 = blockIdx.y * kBucketLdsBins;
  const int nb = S - b0 < kBucketLdsBins ? S - b0 : kBucketLdsBins;
  for (int j = threadIdx.x; j < nb; j += blockDim.x) lh[j] = 0;
  __syncthreads();
  const int64_t r0 = (int64_t)blockIdx.x * chunk_rows;
  const int64_t r1 = r0 + chunk_rows < n ? r0 + chunk_rows : n;
  for (int64_t i = r0 + threadIdx.x; i < r1; i += (int64_t)blockDim.x * kBucketUnroll) {
    unsigned d[kBucketUnroll];
#pragma unroll
    for (int u = 0; u < kBucketUnroll; ++u) {
      const int64_t r = i + (int64_t)u * blockDim.x;
      d[u] = r < r1 ? (unsigned)keys[r] - (unsigned)b0 : ~0u;  // keys outside [0, S) fall outside every slice
    }
#pragma unroll
    for (int u = 0; u < kBucketUnroll; ++u)
      if (d[u] < (unsigned)nb) atomicAdd(&lh[d[u]], 1);
  }
  __syncthreads();
  int32_t* row = mat + (int64_t)blockIdx.x * S + b0;
  for (int j = threadIdx.x; j < nb; j += blockDim.x) row[j] = lh[j];
}

__device__ __forceinline__ int32_t bucket_wave_sum(int32_t v) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}
__device__ __forceinline__ int32_t bucket_wave_incl_scan(int32_t v, int lane) {
  for (int o = 1; o < 64; o <<= 1) {
    const int32_t u = __shfl_up(v, o);
    if (lane >= o) v += u;
  }
  return v;
}

// Column scan of the [B][S] count matrix: a block takes 64 keys, its 4 waves a quarter of the chunks each (held
// in registers), so the loads of a column are all in flight at once.  counts[k] = the key's total; bsum[blk],
// bsum[nblk + blk] = the block's row and tile totals.
constexpr int kBucketMaxChunks = 256;
__global__ __launch_bounds__(256) void bucket_chunk_scan_kernel(int32_t* __restrict__ mat, int B, int S, int tile_rows,
                                                                int32_t* __restrict__ counts, int32_t* __restrict__ bsum) {
  __shared__ int32_t qs[4][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int k = blockIdx.x * 64 + lane;
  const int q = (B + 3) / 4, c0 = w * q;
  int32_t v[kBucketMaxChunks / 4];
  int32_t sum = 0;
#pragma unroll
  for (int j = 0; j < kBucketMaxChunks / 4; ++j) {
    v[j] = 0;
    if (j < q && c0 + j < B && k < S) v[j] = mat[(int64_t)(c0 + j) * S + k];
    sum += v[j];
  }
  qs[w][lane] = sum;
  __syncthreads();
  int32_t run = 0;
  for (int u = 0; u < w; ++u) run += qs[u][lane];
  if (k < S) {
#pragma unroll
    for (int j = 0; j < kBucketMaxChunks / 4; ++j) {
      if (j < q && c0 + j < B) mat[(int64_t)(c0 + j) * S + k] = run;
      run += v[j];
    }
    if (w == 3) counts[k] = run;
  }
  if (w == 3) {
    const int32_t c = k < S ? run : 0;
    const int32_t a = bucket_wave_sum(c);
    const int32_t t = bucket_wave_sum(tile_rows > 0 ? (c + tile_rows - 1) / tile_rows : 0);
    if (lane == 0) {
      bsum[blockIdx.x] = a;
      bsum[gridDim.x + blockIdx.x] = t;
    }
  }
}

// row_off / tile_off from the key totals: one wave per 64 keys, offset = the sums of the blocks before it.
__global__ __launch_bounds__(64) void bucket_chunk_offsets_kernel(const int32_t* __restrict__ counts,
                                                                  const int32_t* __restrict__ bsum, int S,
                                                                  int tile_rows, int32_t* __restrict__ row_off,
                                                                  int32_t* __restrict__ tile_off) {
  const int lane = threadIdx.x, blk = blockIdx.x, nblk = gridDim.x;
  int32_t a = 0, t = 0;
  for (int j = lane; j < blk; j += 64) {
    a += bsum[j];
    t += bsum[nblk + j];
  }
  a = bucket_wave_sum(a);
  t = bucket_wave_sum(t);
  const int k = blk * 64 + lane;
  const int32_t c = k < S ? counts[k] : 0;
  const int32_t tc = tile_rows > 0 ? (c + tile_rows - 1) / tile_rows : 0;
  const int32_t ia = bucket_wave_incl_scan(c, lane), it = bucket_wave_incl_scan(tc, lane);
  if (k < S) {
    row_off[k] = a + ia - c;
    if (tile_off) tile_off[k] = t + it - tc;
  }
  if (blk == nblk - 1 && lane == 63) {
    row_off[S] = a + ia;
    if (tile_off) tile_off[S] = t + it;
  }
}

__global__ __launch_bounds__(1024) void bucket_chunk_scatter_kernel(const int32_t* __restrict__ keys, int64_t n, int S,
                                                                    int64_t chunk_rows, const int32_t* __restrict__ mat,
                                                                    const int32_t* __restrict__ row_off,
                                                                    int32_t* __restrict__ row_index,
                                                                    int32_t* __restrict__ err) {
  extern __shared__ __attribute__((aligned(16))) int32_t lh[];
  const int b0 = blockIdx.y * kBucketLdsBins;
  const int nb = S - b0 < kBucketLdsBins ? S - b0 : kBucketLdsBins;
  const int32_t* row = mat + (int64_t)blockIdx.x * S + b0;
  for (int j = threadIdx.x; j < nb; j += blockDim.x) lh[j] = row_off[b0 + j] + row[j];
  __syncthreads();
  const int64_t r0 = (int64_t)blockIdx.x * chunk_rows;
  const int64_t r1 = r0 + chunk_rows < n ? r0 + chunk_rows : n;
  for (int64_t i = r0 + threadIdx.x; i < r1; i += (int64_t)blockDim.x * kBucketUnroll) {
    unsigned k[kBucketUnroll];
#pragma unroll
    for (int u = 0; u < kBucketUnroll; ++u) {
      const int64_t r = i + (int64_t)u * blockDim.x;
      k[u] = r < r1 ? (unsigned)keys[r] : ~0u;
    }
#pragma unroll
    for (int u = 0; u < kBucketUnroll; ++u) {
      const unsigned d = k[u] - (unsigned)b0;
      if (d < (unsigned)nb)
        bucket_put(atomicAdd(&lh[d], 1), k[u], i + (int64_t)u * blockDim.x, row_off, row_index, err);
    }
  }
}

// ---------------------------------------------------------------------------
// residual / weights
// ---------------------------------------------------------------------------
constexpr int kMaxGroups = 16;

__global__ __launch_bounds__(256) void residual_kernel(const float* __restrict__ x, int64_t n, int dim,
                                                       const float* __restrict__ centers, int k,
                                                       const int32_t* __restrict__ cid,
                                                       const int32_t* __restrict__ gdims, int G,
                                                       int normalize, float* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  int gend[kMaxGroups];
  int acc_e = 0;
  for (int g = 0; g < kMaxGroups; ++g) {
    if (g < G) acc_e += gdims[g];
    gend[g] = acc_e;
  }
  const int nv = dim / 4;
  for (int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); row < n; row += (int64_t)gridDim.x * 4) {
    const float4* xr = reinterpret_cast<const float4*>(x + row * dim);
    const unsigned ci = (unsigned)cid[row];
    const float4* cr = reinterpret_cast<const float4*>(centers + (int64_t)(ci < (unsigned)k ? ci : 0u) * dim);
    float4* orow = reinterpret_cast<float4*>(out + row * dim);
    if (!normalize) {
      for (int i = lane; i < nv; i += 64) {
        const float4 a = xr[i], c = cr[i];
        orow[i] = make_float4(a.x - c.x, a.y - c.y, a.z - c.z, a.w - c.w);
      }
      continue;
    }
    // first pass: per-group sums of squares in fp64
    double gs[kMaxGroups];
#pragma unroll
    for (int g = 0; g < kMaxGroups; ++g) gs[g] = 0.0;
    for (int i = lane; i < nv; i += 64) {
      const float4 a = xr[i], c = cr[i];
      const float rv[4] = {a.x - c.x, a.y - c.y, a.z - c.z, a.w - c.w};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int d = 4 * i + e;
        int g = 0;
        while (g < G - 1 && d >= gend[g]) ++g;
        const double v = rv[e];
#pragma unroll
        for (int gg = 0; gg < kMaxGroups; ++gg)
          if (gg == g) gs[gg] += v * v;
      }
    }
    float den[kMaxGroups];
#pragma unroll
    for (int g = 0; g < kMaxGroups; ++g) {
      if (g < G) {
        const double t = wave_sum(gs[g]);
        den[g] = (float)sqrt(t) + 1e-8f;
      } else {
        den[g] = 1.f;
      }
    }
    for (int i = lane; i < nv; i += 64) {
      const float4 a = xr[i], c = cr[i];
      float rv[4] = {a.x - c.x, a.y - c.y, a.z - c.z, a.w - c.w};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int d = 4 * i + e;
        int g = 0;
        while (g < G - 1 && d >= gend[g]) ++g;
        float dd = 1.f;
#pragma unroll
        for (int gg = 0; gg < kMaxGroups; ++gg)
          if (gg == g) dd = den[gg];
        rv[e] = rv[e] / dd;
      }
      orow[i] = make_float4(rv[0], rv[1], rv[2], rv[3]);
    }
  }
}

__global__ __launch_bounds__(256) void scale_groups_kernel(const float* __restrict__ x, int64_t n, int dim,
                                                           const int32_t* __restrict__ gdims, int G,
                                                           const float* __restrict__ w,
                                                           float* __restrict__ out) {
  const int64_t total = n * dim;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int d = (int)(i % dim);
    int g = 0, e = gdims[0];
    while (g < G - 1 && d >= e) { ++g; e += gdims[g]; }
    out[i] = x[i] * w[g];
  }
}

// ---------------------------------------------------------------------------
// centroid update
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void centroid_accumulate_kernel(const float* __restrict__ x, int dim,
                                                                  const int32_t* __restrict__ row_index,
                                                                  int S, const int32_t* __restrict__ row_off,
                                                                  const int32_t* __restrict__ tile_off,
                                                                  double* __restrict__ sums) {
  const int b = blockIdx.x;
  if (b >= tile_off[S]) return;
  int lo = 0, hi = S;
  while (hi - lo > 1) {
    const int mid = (lo + hi) >> 1;
    if (tile_off[mid] <= b) lo = mid; else hi = mid;
  }
  const int s = lo;
  const int t0 = row_off[s] + (b - tile_off[s]) * kAccTileRows;
  const int t1 = min(t0 + kAccTileRows, row_off[s + 1]);
  for (int d0 = 0; d0 < dim; d0 += 256) {
    const int d = d0 + threadIdx.x;
    if (d >= dim) break;
    double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
    int i = t0;
    for (; i + 4 <= t1; i += 4) {
      const int r0 = row_index ? row_index[i] : i, r1 = row_index ? row_index[i + 1] : i + 1;
      const int r2 = row_index ? row_index[i + 2] : i + 2, r3 = row_index ? row_index[i + 3] : i + 3;
      a0 += x[(int64_t)r0 * dim + d];
      a1 += x[(int64_t)r1 * dim + d];
      a2 += x[(int64_t)r2 * dim + d];
      a3 += x[(int64_t)r3 * dim + d];
    }
    for (; i < t1; ++i) a0 += x[(int64_t)(row_index ? row_index[i] : i) * dim + d];
    atomicAdd(&sums[(int64_t)s * dim + d], (a0 + a1) + (a2 + a3));
  }
}

__global__ __launch_bounds__(256) void centroid_finalize_kernel(const double* __restrict__ sums,
                                                                const int32_t* __restrict__ row_off, int dim,
                                                                float* __restrict__ centers) {
  const int k = blockIdx.x;
  const int c = row_off[k + 1] - row_off[k];
  if (c <= 0) return;
  for (int d = threadIdx.x; d < dim; d += blockDim.x)
    centers[(int64_t)k * dim + d] = (float)(sums[(int64_t)k * dim + d] / (double)c);
}

// ---------------------------------------------------------------------------
// match matrix -> candidate lists
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void match_count_kernel(const uint8_t* __restrict__ m, int groups, int nc,
                                                          int32_t* __restrict__ cnt, uint8_t* __restrict__ flags) {
  const int lane = threadIdx.x & 63;
  const int g = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (g >= groups) return;
  int c = 0;
  for (int j = lane; j < nc; j += 64) c += m[(int64_t)g * nc + j] != 0;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o);
  if (lane == 0) {
    cnt[g] = c;
    flags[g] = c == 0 ? RQSID_SEG_PENALTY : 0;
  }
}

__global__ __launch_bounds__(256) void match_list_kernel(const uint8_t* __restrict__ m, int groups, int nc,
                                                         const int32_t* __restrict__ base,
                                                         int32_t* __restrict__ idx) {
  const int lane = threadIdx.x & 63;
  const int g = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (g >= groups) return;
  int o = base[g];
  for (int j0 = 0; j0 < nc; j0 += 64) {
    const int j = j0 + lane;
    const bool on = j < nc && m[(int64_t)g * nc + j] != 0;
    const unsigned long long bal = __ballot(on);
    if (on) idx[o + __popcll(bal & ((1ull << lane) - 1ull))] = j;
    o += __popcll(bal);
  }
}

// ---------------------------------------------------------------------------
// dense distance matrix (torch.cdist semantics) for the balanced auction
// ---------------------------------------------------------------------------
constexpr int kPdTile = 64;
// MODE 0: out[n][k] = fp32 distance (torch.cdist, pairwise_distance_full balancekmeans/__init__.py:576-603)
// MODE 1: out16[k][n] = fp16(-distance): the auction's worker-major score matrix (auction_lap_half(-D), :29-43)
// MODE 2: pairwise_distance_half (:536-574) with torch's fp16 arithmetic (ATen _euclidean_dist on half
//         tensors): operands rounded to fp16, |x|^2 = fp16(sum fp16(x_i^2)), d^2 = fp16(-2 x.c + |x|^2 +
//         |c|^2) (exact fp16 products, fp32 accumulation), d = fp16(sqrt(max(d^2, 0))), clamp(min=1e-5);
//         then negated into the worker-major score matrix (oracle.cdist_half)
//
// SEG (modes 1/2 only): segment s owns rows seg_off[s]..seg_off[s+1] and centres s*k .. s*k+k-1; its
// scores go to out16 + k*seg_off[s] as a [k][n_s] worker-major block (the segmented auction's layout).
// Row tiles never straddle segments: blockIdx.x indexes the tile list seg_tile_off (exclusive scan of
// ceil(n_s / 64)).  The arithmetic is the unsegmented kernel's, so each block equals a per-segment call.
__device__ __forceinline__ int seg_of(const int32_t* __restrict__ off, int n_seg, int64_t i) {
  int lo = 0, hi = n_seg - 1;  // last s with off[s] <= i
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if ((int64_t)off[mid] <= i) lo = mid; else hi = mid - 1;
  }
  return lo;
}

template <int MODE, bool SEG = false>
__global__ __launch_bounds__(256) void pairwise_distance_kernel(const float* __restrict__ x, int64_t n, int dim,
                                                                const float* __restrict__ c, int k,
                                                                float* __restrict__ out, uint16_t* __restrict__ out16,
                                                                const int32_t* __restrict__ seg_off = nullptr,
                                                                const int32_t* __restrict__ seg_tile_off = nullptr,
                                                                int n_seg = 0) {
  __shared__ float xs[kPdTile][33];
  __shared__ float cs[kPdTile][33];
  const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
  int64_t r0 = (int64_t)blockIdx.x * kPdTile;
  const int c0 = blockIdx.y * kPdTile;
  int64_t seg_base = 0;
  if (SEG) {
    const int s = seg_of(seg_tile_off, n_seg, blockIdx.x);
    seg_base = seg_off[s];
    r0 = seg_base + (int64_t)(blockIdx.x - seg_tile_off[s]) * kPdTile;
    n = seg_off[s + 1];               // rows end at the segment's end
    c += (int64_t)s * k * dim;         // the segment's own centres
    out16 += (int64_t)k * seg_base;    // its [k][n_s] block
  }
  const int64_t n_s = n - seg_base;   // row stride of the worker-major output
  float acc[4][4] = {};
  float xq[4] = {}, cq[4] = {};
  for (int d0 = 0; d0 < dim; d0 += 32) {
    for (int i = threadIdx.x; i < kPdTile * 32; i += 256) {
      const int rr = i >> 5, dd = i & 31;
      float xv = (r0 + rr < n) ? x[(r0 + rr) * dim + d0 + dd] : 0.f;
      float cv = (c0 + rr < k) ? c[(int64_t)(c0 + rr) * dim + d0 + dd] : 0.f;
      if (MODE == 2) {
        xv = (float)(_Float16)xv;
        cv = (float)(_Float16)cv;
      }
      xs[rr][dd] = xv;
      cs[rr][dd] = cv;
    }
    __syncthreads();
#pragma unroll 8
    for (int dd = 0; dd < 32; ++dd) {
      float a[4], bb[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) a[i] = xs[ty + 16 * i][dd];
#pragma unroll
      for (int j = 0; j < 4; ++j) bb[j] = cs[tx + 16 * j][dd];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        if (MODE == 2) {  // x.pow(2) is an fp16 tensor: every square rounded to fp16 before the sum
          xq[i] += (float)(_Float16)(a[i] * a[i]);
          cq[i] += (float)(_Float16)(bb[i] * bb[i]);
        } else {
          xq[i] = fmaf(a[i], a[i], xq[i]);
          cq[i] = fmaf(bb[i], bb[i], cq[i]);
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = fmaf(a[i], bb[j], acc[i][j]);
      }
    }
    __syncthreads();
  }
  if (MODE == 2) {  // the norms are fp16 tensors
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      xq[i] = (float)(_Float16)xq[i];
      cq[i] = (float)(_Float16)cq[i];
    }
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int64_t rr = r0 + ty + 16 * i;
    if (rr >= n) continue;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int cc = c0 + tx + 16 * j;
      if (cc >= k) continue;
      float d;
      if (MODE == 3) {  // cosine distance 1 - x.c / (|x| |c|) (pairwise_cosine, :625-655)
        d = 1.f - acc[i][j] / (sqrtf(xq[i]) * sqrtf(cq[j]));
      } else {
        const float d2 = MODE == 2 ? (float)(_Float16)((-2.f * acc[i][j] + xq[i]) + cq[j])
                                   : (-2.f * acc[i][j] + xq[i]) + cq[j];
        d = sqrtf(fmaxf(d2, 0.f));
      }
      if (MODE == 3) {
        if (out) out[rr * k + cc] = d;
        if (out16) out16[(int64_t)cc * n_s + (rr - seg_base)] = __builtin_bit_cast(uint16_t, (_Float16)(-d));
      } else if (MODE == 0) {
        out[rr * k + cc] = d;
      } else if (MODE == 1) {
        out16[(int64_t)cc * n_s + (rr - seg_base)] = __builtin_bit_cast(uint16_t, (_Float16)(-d));
      } else {
        const _Float16 dh = (_Float16)d, lo = (_Float16)1e-5f;
        out16[(int64_t)cc * n_s + (rr - seg_base)] = __builtin_bit_cast(uint16_t, (_Float16)(-(dh < lo ? lo : dh)));
      }
    }
  }
}


// ---------------------------------------------------------------------------
// greedy unique-nearest match rows (the match-matrix builders)
// ---------------------------------------------------------------------------
// One block per group g: its sub-centres s = 0..n_g-1 (rows sub_off[g]..sub_off[g+1] of dist, a
// [total_sub][C] distance matrix) take, in order, their nearest still-unused candidate column (lowest
// column on exact ties): hierarchical_rq_kmeans.py:1022-1038, simplified_semantic_id_generator.py:282-291.
// match[g][c] = 1 for the chosen columns; n_sel[g] = how many were chosen (the random fill of the
// reference runs on the host afterwards, in the reference's RNG order).
__global__ __launch_bounds__(256) void greedy_match_kernel(const float* __restrict__ dist, const int32_t* __restrict__ sub_off,
                                                           int C, int max_take, uint8_t* __restrict__ match,
                                                           int32_t* __restrict__ n_sel) {
  extern __shared__ unsigned char used[];
  const int g = blockIdx.x;
  const int s0 = sub_off[g], s1 = sub_off[g + 1];
  const int take = min(s1 - s0, max_take);
  for (int c = threadIdx.x; c < C; c += 256) used[c] = 0;
  __shared__ float bv[4];
  __shared__ int bi[4];
  __syncthreads();
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  for (int s = 0; s < take; ++s) {
    const float* row = dist + (int64_t)(s0 + s) * C;
    float best = INFINITY;
    int bc = INT_MAX;
    for (int c = threadIdx.x; c < C; c += 256) {
      const float v = row[c];
      if (!used[c] && (v < best || (v == best && c < bc) || (bc == INT_MAX && !(v == v)))) {
        best = v;
        bc = c;
      }
    }
    for (int o = 32; o > 0; o >>= 1) {
      const float ov = __shfl_xor(best, o);
      const int oc = __shfl_xor(bc, o);
      if (oc != INT_MAX && (bc == INT_MAX || ov < best || (ov == best && oc < bc))) {
        best = ov;
        bc = oc;
      }
    }
    if (lane == 0) {
      bv[wv] = best;
      bi[wv] = bc;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      float b = bv[0];
      int i = bi[0];
      for (int q = 1; q < 4; ++q)
        if (bi[q] != INT_MAX && (i == INT_MAX || bv[q] < b || (bv[q] == b && bi[q] < i))) {
          b = bv[q];
          i = bi[q];
        }
      if (i != INT_MAX) used[i] = 1;
    }
    __syncthreads();
  }
  int cnt = 0;
  for (int c = threadIdx.x; c < C; c += 256) {
    match[(int64_t)g * C + c] = used[c];
    cnt += used[c];
  }
  for (int o = 32; o > 0; o >>= 1) cnt += __shfl_xor(cnt, o);
  __shared__ int tot[4];
  if (lane == 0) tot[wv] = cnt;
  __syncthreads();
  if (threadIdx.x == 0) n_sel[g] = tot[0] + tot[1] + tot[2] + tot[3];
}

int current_device() {
  int d = -1;
  if (hipGetDevice(&d) != hipSuccess || d < 0 || d >= kMaxDevices) return -1;
  return d;
}

int device_cu_count() {
  static int ncu[kMaxDevices] = {};
  const int d = current_device();
  if (d < 0) return 0;
  if (!ncu[d]) {
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, d) != hipSuccess) return 0;
    ncu[d] = prop.multiProcessorCount;
  }
  return ncu[d];
}

namespace {
bool g_attr_done[kMaxDevices] = {};
int ensure_attrs() {
  const int dev = current_device();
  if (dev < 0) return fail(RQSID_E_LAUNCH, "hipGetDevice failed");
  if (g_attr_done[dev]) return RQSID_OK;
  hipError_t e = hipFuncSetAttribute((const void*)bucket_hist_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                     kBucketLdsBins * 4);
  if (e != hipSuccess) return fail(RQSID_E_LAUNCH, "set smem attr (hist): %s", hipGetErrorString(e));
  e = hipFuncSetAttribute((const void*)bucket_scatter_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                          kBucketLdsBins * 4);
  if (e != hipSuccess) return fail(RQSID_E_LAUNCH, "set smem attr (scatter): %s", hipGetErrorString(e));
  e = hipFuncSetAttribute((const void*)bucket_chunk_hist_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                          kBucketLdsBins * 4);
  if (e != hipSuccess) return fail(RQSID_E_LAUNCH, "set smem attr (chunk hist): %s", hipGetErrorString(e));
  e = hipFuncSetAttribute((const void*)bucket_chunk_scatter_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                          kBucketLdsBins * 4);
  if (e != hipSuccess) return fail(RQSID_E_LAUNCH, "set smem attr (chunk scatter): %s", hipGetErrorString(e));
  g_attr_done[dev] = true;
  return RQSID_OK;
}
}  // namespace
}  // namespace rqsid

using namespace rqsid;

extern "C" {

int rqsid_version(void) { return 1; }

// Timing-probe macros this library was built with (tools/ab_build.sh; such builds return WRONG IDs by design):
// 1 RQSID_AB_MODE, 2 RQSID_AB_HALFROW, 4 RQSID_AB_NOROWDMA, 8 RQSID_AB_EPI, 16 RQSID_STAMPS, 32 RQSID_AB_NO_FLUSH.
// 0 for a product build; the Python loader refuses anything else unless the library was named by RQSID_LIB.
int32_t rqsid_build_flags(void) {
  int32_t f = 0;
#if defined(RQSID_AB_MODE) && RQSID_AB_MODE
  f |= 1;
#endif
#ifdef RQSID_AB_HALFROW
  f |= 2;
#endif
#ifdef RQSID_AB_NOROWDMA
  f |= 4;
#endif
#ifdef RQSID_AB_EPI
  f |= 8;
#endif
#ifdef RQSID_STAMPS
  f |= 16;
#endif
#ifdef RQSID_AB_NO_FLUSH
  f |= 32;
#endif
  return f;
}
const char* rqsid_last_error(void) { return g_err; }

int32_t rqsid_centroid_tile_rows(void) { return kAccTileRows; }

// workspace: counts i32[S] | cursor i32[S] | 64 ints: [0] the sticky error word (zeroed by the caller when it
// allocates the workspace, never by a call: include/rqsid.h) | for S <= 262144 the [B][S] count matrix
// (B x S <= 4M words: 16 MiB, independent of n so that one workspace serves every call with these keys)
int64_t rqsid_bucket_workspace_bytes(int64_t n, int32_t n_segments) {
  (void)n;
  const int64_t B = bucket_max_chunks(n_segments);
  return ((int64_t)n_segments * 2 + 64 + (B ? B * n_segments + 2 * cdiv(n_segments, 64) : 0)) * 4;
}

int rqsid_bucket(const int32_t* keys, int64_t n, int32_t S, int32_t tile_rows, int32_t* seg_row_off,
                 int32_t* seg_tile_off, int32_t* row_index, void* workspace, int64_t workspace_bytes,
                 void* stream) {
  if (S <= 0 || n < 0 || !seg_row_off || (n > 0 && (!keys || !row_index)) || n > INT32_MAX)
    return fail(RQSID_E_ARG, "bucket: bad arguments (n=%lld S=%d)", (long long)n, S);
  if (workspace_bytes < rqsid_bucket_workspace_bytes(n, S) || !workspace)
    return fail(RQSID_E_WORKSPACE, "bucket: workspace too small");
  int rc = ensure_attrs();
  if (rc) return rc;
  hipStream_t st = (hipStream_t)stream;
  int32_t* counts = (int32_t*)workspace;
  int32_t* cursor = counts + S;
  // the count matrix for every S it covers (measured at small S too: 128 keys over 10M rows 0.140 -> 0.080 ms,
  // 256 over 6.25M 0.108 -> 0.061); RQSID_BUCKET_MATRIX=0 keeps the LDS-histogram / global-atomic forms (A/B)
  const char* ebm = getenv("RQSID_BUCKET_MATRIX");
  const int B = ebm && atoi(ebm) == 0 ? 0 : bucket_chunks(n, S);
  if (B > 0) {
    int32_t* mat = cursor + S + 64;
    int32_t* bsum = mat + (int64_t)B * S;
    const int64_t chunk_rows = cdiv(n, B);
    const dim3 grid((unsigned)B, (unsigned)cdiv(S, kBucketLdsBins));
    const size_t lds = (size_t)kBucketLdsBins * 4;
    const unsigned nblk = (unsigned)cdiv(S, 64);
    hipLaunchKernelGGL(bucket_chunk_hist_kernel, grid, dim3(1024), lds, st, keys, n, S, chunk_rows, mat);
    hipLaunchKernelGGL(bucket_chunk_scan_kernel, dim3(nblk), dim3(256), 0, st, mat, B, S, tile_rows, counts, bsum);
    hipLaunchKernelGGL(bucket_chunk_offsets_kernel, dim3(nblk), dim3(64), 0, st, counts, bsum, S, tile_rows,
                       seg_row_off, seg_tile_off);
    hipLaunchKernelGGL(bucket_chunk_scatter_kernel, grid, dim3(1024), lds, st, keys, n, S, chunk_rows, mat,
                       seg_row_off, row_index, cursor + S);
    return check_launch("bucket_chunk");
  }
  if (fill_async(counts, 0, (size_t)S * 4, st) != hipSuccess) return fail(RQSID_E_LAUNCH, "bucket: memset");
  const size_t lds = S <= kBucketLdsBins ? (size_t)S * 4 : 0;
  // rows per LDS-histogram block: every block zeroes its S bins and adds each non-zero bin to the global count
  // (hist) or reserves a cursor range for it (scatter), so many keys take bigger blocks (RQSID_BUCKET_WIDE: the
  // rows per block for S > 4096, A/B)
  const char* ebw = getenv("RQSID_BUCKET_WIDE");
  const int64_t wide_rows = ebw ? std::max<int64_t>(4096, atoll(ebw)) : 32768;
  const bool wide = S > 4096;
  const int64_t hist_rows = wide ? wide_rows : 256 * 16, scat_rows = wide ? wide_rows : kScatterRowsPerBlock;
  if (n > 0) {
    hipLaunchKernelGGL(bucket_hist_kernel, dim3(grid_cap(cdiv(n, hist_rows), 2048)), dim3(256), lds, st, keys, n,
                       S, counts);
    if ((rc = check_launch("bucket_hist"))) return rc;
  }
  hipLaunchKernelGGL(bucket_scan_kernel, dim3(1), dim3(1024), 0, st, counts, S, tile_rows, seg_row_off,
                     seg_tile_off, cursor);
  if ((rc = check_launch("bucket_scan"))) return rc;
  if (n > 0) {
    const unsigned blocks = S <= kBucketLdsBins ? (unsigned)cdiv(n, scat_rows) : grid_cap(cdiv(n, 256 * 16), 2048);
    hipLaunchKernelGGL(bucket_scatter_kernel, dim3(blocks), dim3(256), lds, st, keys, n, S, cursor, seg_row_off,
                       row_index, cursor + S, (int64_t)scat_rows);
    if ((rc = check_launch("bucket_scatter"))) return rc;
  }
  return RQSID_OK;
}


int rqsid_residual(const float* x, int64_t n, int32_t dim, const float* centers, int32_t n_centers,
                   const int32_t* center_id, const int32_t* group_dims, int32_t n_groups, int32_t normalize,
                   float* out, void* stream) {
  if ((n > 0 && (!x || !center_id || !out)) || !centers || dim <= 0 || dim % 4 || n < 0 || n_centers <= 0 ||
      (normalize && (!group_dims || n_groups <= 0 || n_groups > kMaxGroups)))
    return fail(RQSID_E_ARG, "residual: bad arguments (dim=%d groups=%d)", dim, n_groups);
  if (n == 0) return RQSID_OK;
  hipLaunchKernelGGL(residual_kernel, dim3(grid_cap(cdiv(n, 4), 8192)), dim3(256), 0, (hipStream_t)stream, x, n,
                     dim, centers, n_centers, center_id, group_dims, normalize ? n_groups : 1, normalize, out);
  return check_launch("residual");
}

int rqsid_scale_groups(const float* x, int64_t n, int32_t dim, const int32_t* group_dims, int32_t n_groups,
                       const float* weights, float* out, void* stream) {
  if ((n > 0 && (!x || !out)) || !group_dims || !weights || n_groups <= 0 || dim <= 0 || n < 0)
    return fail(RQSID_E_ARG, "scale_groups: bad arguments");
  if (n == 0) return RQSID_OK;
  hipLaunchKernelGGL(scale_groups_kernel, dim3(grid_cap(cdiv(n * dim, 256 * 8), 8192)), dim3(256), 0,
                     (hipStream_t)stream, x, n, dim, group_dims, n_groups, weights, out);
  return check_launch("scale_groups");
}

int rqsid_centroid_accumulate(const float* x, int32_t dim, const int32_t* row_index, int32_t n_segments,
                              const int32_t* seg_row_off, const int32_t* seg_tile_off, int64_t max_tiles,
                              double* sums, void* stream) {
  if (!x || !seg_row_off || !seg_tile_off || !sums || dim <= 0 || n_segments <= 0 || max_tiles < 0 ||
      max_tiles > INT32_MAX)
    return fail(RQSID_E_ARG, "centroid_accumulate: bad arguments");
  if (max_tiles == 0) return RQSID_OK;
  hipLaunchKernelGGL(centroid_accumulate_kernel, dim3((unsigned)max_tiles), dim3(256), 0, (hipStream_t)stream, x,
                     dim, row_index, n_segments, seg_row_off, seg_tile_off, sums);
  return check_launch("centroid_accumulate");
}

int rqsid_centroid_finalize(const double* sums, const int32_t* seg_row_off, int32_t k, int32_t dim, float* centers,
                            void* stream) {
  if (!sums || !seg_row_off || !centers || k <= 0 || dim <= 0)
    return fail(RQSID_E_ARG, "centroid_finalize: bad arguments");
  hipLaunchKernelGGL(centroid_finalize_kernel, dim3((unsigned)k), dim3(256), 0, (hipStream_t)stream, sums,
                     seg_row_off, dim, centers);
  return check_launch("centroid_finalize");
}

int64_t rqsid_match_workspace_bytes(int32_t groups) { return ((int64_t)groups * 2 + 64) * 4; }

int rqsid_match_to_candidates(const uint8_t* match, int32_t groups, int32_t n_cand, int32_t* cand_base,
                              int32_t* cand_count, int32_t* cand_idx, uint8_t* seg_flags, void* workspace,
                              int64_t workspace_bytes, void* stream) {
  if (!match || groups <= 0 || n_cand <= 0 || !cand_base || !cand_count || !cand_idx || !seg_flags)
    return fail(RQSID_E_ARG, "match_to_candidates: bad arguments");
  if (!workspace || workspace_bytes < rqsid_match_workspace_bytes(groups))
    return fail(RQSID_E_WORKSPACE, "match_to_candidates: workspace too small");
  hipStream_t st = (hipStream_t)stream;
  int rc;
  hipLaunchKernelGGL(match_count_kernel, dim3((unsigned)cdiv(groups, 4)), dim3(256), 0, st, match, groups, n_cand,
                     cand_count, seg_flags);
  if ((rc = check_launch("match_count"))) return rc;
  int32_t* off = (int32_t*)workspace;  // groups + 1
  hipLaunchKernelGGL(bucket_scan_kernel, dim3(1), dim3(1024), 0, st, cand_count, groups, 0, off,
                     (int32_t*)nullptr, (int32_t*)nullptr);
  if ((rc = check_launch("match_scan"))) return rc;
  if (hipMemcpyAsync(cand_base, off, (size_t)groups * 4, hipMemcpyDeviceToDevice, st) != hipSuccess)
    return fail(RQSID_E_LAUNCH, "match: copy");
  hipLaunchKernelGGL(match_list_kernel, dim3((unsigned)cdiv(groups, 4)), dim3(256), 0, st, match, groups, n_cand,
                     off, cand_idx);
  return check_launch("match_list");
}

int rqsid_pairwise_distance(const float* x, int64_t n, int32_t dim, const float* centers, int32_t k, float* out,
                            void* stream) {
  if ((n > 0 && (!x || !out)) || !centers || n < 0 || k <= 0 || dim <= 0 || dim % 32)
    return fail(RQSID_E_ARG, "pairwise_distance: bad arguments");
  if (n == 0) return RQSID_OK;
  hipLaunchKernelGGL(pairwise_distance_kernel<0>, dim3((unsigned)cdiv(n, kPdTile), (unsigned)cdiv(k, kPdTile)),
                     dim3(256), 0, (hipStream_t)stream, x, n, dim, centers, k, out, (uint16_t*)nullptr);
  return check_launch("pairwise_distance");
}

int rqsid_pairwise_cosine(const float* x, int64_t n, int32_t dim, const float* centers, int32_t k, float* out,
                          uint16_t* out_wj, void* stream) {
  if ((n > 0 && (!x || (!out && !out_wj))) || !centers || n < 0 || k <= 0 || dim <= 0 || dim % 32)
    return fail(RQSID_E_ARG, "pairwise_cosine: bad arguments");
  if (n == 0) return RQSID_OK;
  hipLaunchKernelGGL(pairwise_distance_kernel<3>, dim3((unsigned)cdiv(n, kPdTile), (unsigned)cdiv(k, kPdTile)),
                     dim3(256), 0, (hipStream_t)stream, x, n, dim, centers, k, out, out_wj);
  return check_launch("pairwise_cosine");
}

int rqsid_auction_scores(const float* x, int64_t n, int32_t dim, const float* centers, int32_t k, int32_t half,
                         uint16_t* out_wj, void* stream) {
  if ((n > 0 && (!x || !out_wj)) || !centers || n < 0 || k <= 0 || dim <= 0 || dim % 32)
    return fail(RQSID_E_ARG, "auction_scores: bad arguments");
  if (n == 0) return RQSID_OK;
  const dim3 g((unsigned)cdiv(n, kPdTile), (unsigned)cdiv(k, kPdTile));
  if (half)
    hipLaunchKernelGGL(pairwise_distance_kernel<2>, g, dim3(256), 0, (hipStream_t)stream, x, n, dim, centers, k,
                       (float*)nullptr, out_wj);
  else
    hipLaunchKernelGGL(pairwise_distance_kernel<1>, g, dim3(256), 0, (hipStream_t)stream, x, n, dim, centers, k,
                       (float*)nullptr, out_wj);
  return check_launch("auction_scores");
}

int rqsid_seg_auction_scores(const float* x, int64_t n, int32_t dim, const float* centers, int32_t k,
                             int32_t n_seg, const int32_t* seg_off, const int32_t* seg_tile_off, int64_t n_tiles,
                             int32_t half, uint16_t* out_wj, void* stream) {
  if ((n > 0 && (!x || !out_wj)) || !centers || !seg_off || !seg_tile_off || n < 0 || k <= 0 || dim <= 0 || dim % 32 ||
      n_seg <= 0 || n_tiles < 0 || n_tiles > INT32_MAX)
    return fail(RQSID_E_ARG, "seg_auction_scores: bad arguments");
  if (n == 0 || n_tiles == 0) return RQSID_OK;
  const dim3 g((unsigned)n_tiles, (unsigned)cdiv(k, kPdTile));
  if (half)
    hipLaunchKernelGGL((pairwise_distance_kernel<2, true>), g, dim3(256), 0, (hipStream_t)stream, x, n, dim, centers,
                       k, (float*)nullptr, out_wj, seg_off, seg_tile_off, n_seg);
  else
    hipLaunchKernelGGL((pairwise_distance_kernel<1, true>), g, dim3(256), 0, (hipStream_t)stream, x, n, dim, centers,
                       k, (float*)nullptr, out_wj, seg_off, seg_tile_off, n_seg);
  return check_launch("seg_auction_scores");
}

int rqsid_greedy_match(const float* dist, const int32_t* sub_off, int32_t groups, int32_t n_cand, int32_t max_take,
                       uint8_t* match, int32_t* n_selected, void* stream) {
  if (!dist || !sub_off || !match || !n_selected || groups < 0 || n_cand <= 0 || n_cand > 65536 || max_take < 0)
    return fail(RQSID_E_ARG, "greedy_match: bad arguments (groups=%d C=%d)", groups, n_cand);
  if (groups == 0) return RQSID_OK;
  // one byte of dynamic LDS per candidate column beside the kernel's static LDS: beyond the default
  // 64 KiB the limit is raised (per device) up to the CU's 160 KiB
  if (n_cand > 32768) {
    static bool raised[kMaxDevices] = {};
    const int dev = current_device();
    if (dev < 0) return fail(RQSID_E_LAUNCH, "greedy_match: hipGetDevice failed");
    if (!raised[dev]) {
      if (hipFuncSetAttribute((const void*)greedy_match_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, 65536) !=
          hipSuccess)
        return fail(RQSID_E_LAUNCH, "greedy_match: cannot raise the dynamic LDS limit");
      raised[dev] = true;
    }
  }
  hipLaunchKernelGGL(greedy_match_kernel, dim3((unsigned)groups), dim3(256), (size_t)n_cand, (hipStream_t)stream, dist,
                     sub_off, n_cand, max_take, match, n_selected);
  return check_launch("greedy_match");
}

}  // extern "C"
