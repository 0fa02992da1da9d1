// rqsid.hip — MI355X (gfx950 / CDNA4) kernels for hierarchical residual-quantisation
// K-Means semantic IDs, behind the C ABI declared in include/rqsid.h.
//
// Hot path: nearest-centre assignment (A2/A4/A11/A12/A13/A18),
// residuals (A14), group weights (A15), the Lloyd centroid update (A10) and the
// row bucketing that replaces the reference's per-parent mask loops.
//
// Design notes (DESIGN.md has the full story):
//  * rqsid_assign is a segmented "grouped GEMM + argmin": a work tile is up to
//    128 rows of ONE segment (a parent cluster / an (l1,l2) group) against that
//    segment's candidate centres.  X·Cᵀ runs on MFMA v_mfma_f32_32x32x16_bf16 with
//    every fp32 operand split into bf16 hi+lo (3 MFMAs: hi·hi + hi·lo + lo·hi);
//    a rigorous per-candidate error bound decides whether the row's nearest centre
//    is already certain.  Rows where the bound admits >1 candidate are appended to
//    a work list and re-scored in fp64 by a second kernel, so the returned IDs are
//    the exact argmin (lowest index on exact ties), independent of summation order.
//  * centres are the MFMA A operand (32 candidates on the M axis) and rows the B
//    operand, so each lane ends up owning ONE row and 16 of its candidates: the
//    argmin is in-register plus one cross-half exchange.
//  * X and centre chunks are staged through LDS (register staging, coalesced
//    128-B line loads) in an XOR-swizzled image that makes every ds_read_b128 of
//    the fragment reads conflict-free.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <climits>
#include <type_traits>

#include "../../include/rqsid.h"

namespace {

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

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef __attribute__((ext_vector_type(4))) unsigned int u32x4;

constexpr int kWaves = 4;
constexpr int kRowsPerWave = 32;
constexpr int kTileRows = kWaves * kRowsPerWave;  // rows per assign work tile
constexpr int kChunk = 32;                         // dims per LDS stage
constexpr int kLdsRow = 128;                       // bytes per LDS image row
constexpr int kXStageBytes = kTileRows * kLdsRow;  // 16 KiB
constexpr int kAccTileRows = 256;                  // rows per centroid-accumulate tile
constexpr int kBucketLdsBins = 16384;

struct WorkItem {
  int32_t row;
  int32_t seg;
  int32_t n;  // >=1: explicit local candidates in cand[]; -1: every candidate of the segment; -2: penalty (all centres)
  int32_t pad;
  int32_t cand[4];
};
static_assert(sizeof(WorkItem) == 32, "work item layout");

struct AssignParams {
  const float* x;
  int32_t dim;
  const int32_t* row_index;
  int32_t n_segments;
  const int32_t* seg_row_off;
  const int32_t* seg_tile_off;
  const float* centers;
  const uint16_t* c_split;
  const float* c_meta;  // float4 per centre: |c|^2, |c|, |c - hi - lo|, |lo|
  int32_t n_centers;
  const int32_t* cand_base;
  const int32_t* cand_count;
  const int32_t* cand_idx;
  const uint8_t* seg_flags;
  int32_t* out_local;
  int32_t* out_global;
  WorkItem* work;
  int32_t* work_count;
  int64_t work_cap;
  float acc_rel;
  // fused residuals (res_levels >= 1)
  const float* ca;
  const int32_t* ca_idx;
  const float* cb;
  const int32_t* cb_idx;
  const float* den_in;
  float* den_out;
};

__device__ __forceinline__ uint16_t bf16_bits(float f) {
  return __builtin_bit_cast(uint16_t, (__bf16)f);
}
__device__ __forceinline__ float bf16_to_f32(uint16_t b) { return __uint_as_float(((uint32_t)b) << 16); }

__device__ __forceinline__ int swz(int row) { return (row >> 1) & 7; }

__device__ __forceinline__ int cand_global(const AssignParams& p, int base, int local) {
  return p.cand_idx ? p.cand_idx[base + local] : base + local;
}

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

// ---------------------------------------------------------------------------
// centre preparation
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void prepare_centers_kernel(const float* __restrict__ c, int64_t k,
                                                              int dim, uint16_t* __restrict__ split,
                                                              float4* __restrict__ meta) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= k) return;
  const float* cr = c + row * dim;
  const int nch = dim / kChunk;
  double s = 0.0, se = 0.0, sl = 0.0;
  for (int i = lane; i < dim; i += 64) {
    const float v = cr[i];
    const uint16_t hb = bf16_bits(v);
    const float rem = v - bf16_to_f32(hb);
    const uint16_t lb = bf16_bits(rem);
    const float ex = rem - bf16_to_f32(lb);
    const int ch = i / kChunk, j = i % kChunk;
    uint16_t* dst = split + (row * nch + ch) * (2 * kChunk);
    dst[j] = hb;
    dst[kChunk + j] = lb;
    s += (double)v * (double)v;
    se += (double)ex * (double)ex;
    sl += (double)rem * (double)rem;
  }
  s = wave_sum(s);
  se = wave_sum(se);
  sl = wave_sum(sl);
  if (lane == 0)  // |c|^2, |c|, |c - hi - lo|, |lo| (norms rounded up slightly for the bound)
    meta[row] = make_float4((float)s, (float)sqrt(s) * 1.0000002f, (float)sqrt(se) * 1.0000002f,
                            (float)sqrt(sl) * 1.0000002f);
}

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

// One block: exclusive scans of counts and ceil(counts / tile_rows).
__global__ __launch_bounds__(1024) void bucket_scan_kernel(const int32_t* __restrict__ counts, int S,
                                                           int tile_rows, int32_t* __restrict__ row_off,
                                                           int32_t* __restrict__ tile_off,
                                                           int32_t* __restrict__ cursor) {
  __shared__ int32_t sa[1024], sb[1024];
  __shared__ int32_t carry[2];
  const int t = threadIdx.x;
  if (t == 0) carry[0] = carry[1] = 0;
  __syncthreads();
  for (int base = 0; base < S; base += 1024) {
    const int i = base + t;
    const int32_t a = i < S ? counts[i] : 0;
    const int32_t b = tile_rows > 0 ? (a + tile_rows - 1) / tile_rows : 0;
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
    const int32_t ea = carry[0] + sa[t] - a, eb = carry[1] + sb[t] - b;
    if (i < S) {
      row_off[i] = ea;
      if (tile_off) tile_off[i] = eb;
      if (cursor) cursor[i] = ea;
    }
    __syncthreads();
    if (t == 1023) {
      carry[0] += sa[1023];
      carry[1] += sb[1023];
    }
    __syncthreads();
  }
  if (t == 0) {
    row_off[S] = carry[0];
    if (tile_off) tile_off[S] = carry[1];
  }
}

constexpr int kScatterRowsPerBlock = 8192;

__global__ __launch_bounds__(256) void bucket_scatter_kernel(const int32_t* __restrict__ keys, int64_t n,
                                                             int S, int32_t* __restrict__ cursor,
                                                             int32_t* __restrict__ row_index) {
  extern __shared__ __attribute__((aligned(16))) int32_t lh[];
  if (S <= kBucketLdsBins) {
    const int64_t r0 = (int64_t)blockIdx.x * kScatterRowsPerBlock;
    const int64_t r1 = r0 + kScatterRowsPerBlock < n ? r0 + kScatterRowsPerBlock : n;
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
      const int32_t pos = atomicAdd(&lh[k], 1);
      row_index[pos] = (int32_t)i;
    }
  } else {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
      const unsigned k = (unsigned)keys[i];
      if (k >= (unsigned)S) continue;
      const int32_t pos = atomicAdd(&cursor[k], 1);
      row_index[pos] = (int32_t)i;
    }
  }
}

// ---------------------------------------------------------------------------
// assignment: bf16x3 MFMA screening (+ fused on-the-fly residuals)
// ---------------------------------------------------------------------------
// Screening error model (DESIGN.md "Screening bound").  Inputs are split
// x = xh + xl + ex with xh = bf16(x), xl = bf16(x - xh); the MFMA computes
// xh.ch + xh.cl + xl.ch.  Representation error (Cauchy-Schwarz, exact per-row /
// per-centre split norms measured on the fly): |ex||c| + |x||ec| + |xl||cl| + |ex||ec|.
// Accumulation: tests/test_mfma_numerics.py shows v_mfma_f32_32x32x16_bf16 does NOT
// sum its products exactly (low bits are dropped while aligning), so the default
// model charges every instruction 17 additions at one ulp (2^-23, truncation) of
// (|C| + sum|products|), i.e. acc_rel = 3*(dim/16)*17*2^-23 of sum|x_i c_i|.  The
// tighter model pinned bit-exactly by test_mfma_emulation (rqsid_set_mfma_model)
// replaces it.
inline float accumulation_rel_pessimistic(int dim) {
  return (float)((3.0 * (dim / 16) * 17.0 + 8.0) * std::ldexp(1.0, -23) * 1.02);
}
float g_acc_rel_override = -1.0f;
inline float accumulation_rel(int dim) {
  return g_acc_rel_override > 0 ? g_acc_rel_override * (3.0f * (dim / 16) + 1.0f) : accumulation_rel_pessimistic(dim);
}

template <int NT>
struct ScreenLayout {
  static constexpr int kCBytes = NT * 32 * kLdsRow;
  static constexpr int kStage = kXStageBytes + kCBytes;
  static constexpr int kMeta = 2 * kStage;             // float2 {|c|^2, |c|} per candidate
  static constexpr int kRatio = kMeta + NT * 32 * 8;   // max over the pass of |ec|/|c|, |cl|/|c|
  static constexpr int kBytes = kRatio + 16;
};

__device__ __forceinline__ void push_work(const AssignParams& p, bool need, int lane, const WorkItem& w) {
  const unsigned long long m = __ballot(need);
  if (!m) return;
  const int leader = __ffsll((long long)m) - 1;
  int base = 0;
  if (lane == leader) base = atomicAdd(p.work_count, __popcll(m));
  base = __shfl(base, leader);
  if (need) {
    const int idx = base + __popcll(m & ((1ull << lane) - 1ull));
    if (idx < p.work_cap) p.work[idx] = w;
  }
}

// RL = residual levels computed on the fly (0: x, 1: x - ca, 2: (x - ca)/n1 - cb),
// NORM = divide by (||.|| + 1e-8) (hierarchical) or not (simplified).
template <int NT, int RL, bool NORM>
__global__ __launch_bounds__(256, 1) void assign_screen_kernel(AssignParams p) {
  using L = ScreenLayout<NT>;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int h = lane >> 5, r = lane & 31;
  const int b = blockIdx.x;
  const int S = p.n_segments;
  if (b >= p.seg_tile_off[S]) return;
  int lo = 0, hi = S;
  while (hi - lo > 1) {
    const int mid = (lo + hi) >> 1;
    if (p.seg_tile_off[mid] <= b) lo = mid; else hi = mid;
  }
  const int s = lo;
  const int t0 = p.seg_row_off[s] + (b - p.seg_tile_off[s]) * kTileRows;
  const int nrows = min(kTileRows, p.seg_row_off[s + 1] - t0);
  const int cnt = p.cand_count[s];
  const int cbase = p.cand_base[s];
  const bool penalty = p.seg_flags && (p.seg_flags[s] & RQSID_SEG_PENALTY);

  const int my_local = wave * kRowsPerWave + r;
  const bool row_valid = my_local < nrows;
  const int pos = t0 + (row_valid ? my_local : 0);
  const int my_row = p.row_index ? p.row_index[pos] : pos;

  if (penalty || cnt <= 0) {
    WorkItem w{};
    w.row = my_row;
    w.seg = s;
    w.n = penalty ? -2 : -3;
    push_work(p, h == 0 && row_valid, lane, w);
    return;
  }

  const int nch = p.dim / kChunk;
  const int q = lane & 7;       // 16-B slot this lane stages
  const int rs = lane >> 3;     // row within an 8-row staging group
  // staging rows as 32-bit ids (64-bit addresses are rebuilt per load to save VGPRs)
  int xrow[4], arow[4], brow[4];
  float inv1[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int rr = 8 * i + rs;
    const int grow = __shfl(my_row, rr);
    xrow[i] = grow;
    if (RL >= 1) arow[i] = p.ca_idx[grow];
    if (RL >= 2) {
      brow[i] = p.cb_idx[grow];
      inv1[i] = NORM ? 1.0f / p.den_in[grow] : 1.0f;
    }
  }
  const int xw_off = wave * (kRowsPerWave * kLdsRow);

  float U = INFINITY, b1 = INFINITY, b2 = INFINITY, b3 = INFINITY;
  int k1 = -1, k2 = -1, k3 = -1;
  double sv2 = 0.0;          // sum v^2 (fp64: the normalising denominator is exact)
  float se2 = 0.f, sl2 = 0.f;  // sum of split residual^2 and lo^2 (bound only)
  float vn = 0.f, en = 0.f, ln = 0.f, inv_den = 1.f, dr = 0.f;
  float2* lds_meta = reinterpret_cast<float2*>(smem + L::kMeta);
  unsigned* lds_ratio = reinterpret_cast<unsigned*>(smem + L::kRatio);
  const f32x16 zero16 = {};

  const int npass = (cnt + NT * 32 - 1) / (NT * 32);
  for (int pass = 0; pass < npass; ++pass) {
    const int pbase = pass * NT * 32;
    int cgi[NT];
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      const int il = j * 32 + wave * 8 + rs;
      const int kl = pbase + il < cnt ? pbase + il : 0;
      cgi[j] = cand_global(p, cbase, kl);
    }
    if (tid < 2) lds_ratio[tid] = 0u;
    __syncthreads();
    if (tid < NT * 32) {
      const int kl = pbase + tid < cnt ? pbase + tid : 0;
      const int cg = cand_global(p, cbase, kl);
      const float4 m = reinterpret_cast<const float4*>(p.c_meta)[cg];
      lds_meta[tid] = make_float2(m.x, m.y);
      const float inv = m.y > 0.f ? 1.0f / m.y : 0.f;
      // positive floats order like their bit patterns
      atomicMax(&lds_ratio[0], __float_as_uint(m.y > 0.f ? m.z * inv * 1.000001f : 0.f));
      atomicMax(&lds_ratio[1], __float_as_uint(m.y > 0.f ? m.w * inv * 1.000001f : 0.f));
    }

    f32x16 acc[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[t] = zero16;

    u32x4 xs[4], cs[NT];
    auto gload = [&](int c) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int64_t off = (int64_t)c * kChunk + q * 4;
        float4 v = *reinterpret_cast<const float4*>(p.x + (int64_t)xrow[i] * p.dim + off);
        if (RL >= 1) {
          const float4 a = *reinterpret_cast<const float4*>(p.ca + (int64_t)arow[i] * p.dim + off);
          v = make_float4(v.x - a.x, v.y - a.y, v.z - a.z, v.w - a.w);  // exact fp32, as the reference
          if (RL >= 2) {
            const float4 cbv = *reinterpret_cast<const float4*>(p.cb + (int64_t)brow[i] * p.dim + off);
            if (NORM) v = make_float4(v.x * inv1[i], v.y * inv1[i], v.z * inv1[i], v.w * inv1[i]);
            v = make_float4(v.x - cbv.x, v.y - cbv.y, v.z - cbv.z, v.w - cbv.w);
          }
        }
        xs[i] = __builtin_bit_cast(u32x4, v);
      }
#pragma unroll
      for (int j = 0; j < NT; ++j)
        cs[j] = *reinterpret_cast<const u32x4*>(p.c_split + ((int64_t)cgi[j] * nch + c) * (2 * kChunk) + q * 8);
    };
    auto swrite = [&](int stage) {
      unsigned char* xb = smem + stage * L::kStage + xw_off;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int rr = 8 * i + rs;
        *reinterpret_cast<u32x4*>(xb + rr * kLdsRow + ((q ^ swz(rr)) << 4)) = xs[i];
      }
      unsigned char* cb = smem + stage * L::kStage + kXStageBytes;
#pragma unroll
      for (int j = 0; j < NT; ++j) {
        const int il = j * 32 + wave * 8 + rs;
        *reinterpret_cast<u32x4*>(cb + il * kLdsRow + ((q ^ swz(il)) << 4)) = cs[j];
      }
    };
    // one chunk = 2 k-steps x NT tiles x 3 MFMAs
    auto chunk = [&](int c) {
      const unsigned char* xb = smem + (c & 1) * L::kStage + xw_off + r * kLdsRow;
      const unsigned char* cb = smem + (c & 1) * L::kStage + kXStageBytes + r * kLdsRow;
      float4 xa[2], xc[2];
      bf16x8 ah[2][NT], al[2][NT];
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const int q0 = 4 * ks + 2 * h;
        xa[ks] = *reinterpret_cast<const float4*>(xb + ((q0 ^ swz(r)) << 4));
        xc[ks] = *reinterpret_cast<const float4*>(xb + (((q0 + 1) ^ swz(r)) << 4));
        const int qh = 2 * ks + h, ql = 4 + 2 * ks + h;
#pragma unroll
        for (int t = 0; t < NT; ++t) {
          const unsigned char* ct = cb + t * 32 * kLdsRow;
          al[ks][t] = *reinterpret_cast<const bf16x8*>(ct + ((ql ^ swz(r)) << 4));
          ah[ks][t] = *reinterpret_cast<const bf16x8*>(ct + ((qh ^ swz(r)) << 4));
        }
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const float xv[8] = {xa[ks].x, xa[ks].y, xa[ks].z, xa[ks].w, xc[ks].x, xc[ks].y, xc[ks].z, xc[ks].w};
        bf16x8 bh, bl;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const __bf16 hv = (__bf16)xv[e];
          const float rem = xv[e] - (float)hv;
          const __bf16 lv = (__bf16)rem;
          bh[e] = hv;
          bl[e] = lv;
          if (pass == 0) {
            const float ex = rem - (float)lv;  // exact: the split residual
            sv2 += (double)xv[e] * (double)xv[e];
            se2 = fmaf(ex, ex, se2);
            sl2 = fmaf(rem, rem, sl2);
          }
        }
#pragma unroll
        for (int t = 0; t < NT; ++t) {
          acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al[ks][t], bh, acc[t], 0, 0, 0);
          acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[ks][t], bl, acc[t], 0, 0, 0);
          acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[ks][t], bh, acc[t], 0, 0, 0);
        }
      }
    };
    gload(0);
    swrite(0);
    __syncthreads();
    for (int c = 0; c < nch; ++c) {
      if (c + 1 < nch) gload(c + 1);
      chunk(c);
      if (c + 1 < nch) swrite((c + 1) & 1);
      __syncthreads();
    }

    if (pass == 0) {
      const double tot = sv2 + __shfl_xor(sv2, 32);
      const float nrm = (float)sqrt(tot);
      const float e2 = se2 + __shfl_xor(se2, 32), l2 = sl2 + __shfl_xor(sl2, 32);
      en = sqrtf(e2) * 1.001f + 1e-30f;
      ln = sqrtf(l2) * 1.001f;
      vn = nrm * 1.0001f;
      if (NORM && RL >= 1) {
        const float den = nrm + 1e-8f;
        inv_den = 1.0f / den;
        if (RL == 1 && h == 0 && row_valid && p.den_out) p.den_out[my_row] = den;
        // |r_ref - v/den| per element: RL1: the reference rounds r_i = u_i/den once;
        // RL2: v was built with a reciprocal multiply (2 ulp of |r1| = 1) and rounded
        dr = RL == 1 ? 2.0f * 5.97e-8f : (4.0f * 2.39e-7f * (1.0f + vn) * inv_den + 4.0f * 5.97e-8f);
      }
    }
    // epilogue: screening bounds and the 3 smallest lower bounds per lane.  Per candidate
    // e_k = K*|c_k| + 2^-22*|c_k|^2 with the row/pass constant
    // K = 2/den*(|ex| + |x| rho_e + |xl| rho_l + |ex| rho_e + acc_rel |x|) + 2 dr + 2^-21 |r|
    // (rho = the pass's largest |ec|/|c|, |cl|/|c|; absolute centre terms scale with |c_k|).
    const float rho_e = __uint_as_float(lds_ratio[0]), rho_l = __uint_as_float(lds_ratio[1]);
    const float vr = vn * inv_den;  // |r| of the row being assigned
    const float K = 2.0f * inv_den * 1.000001f * (en + vn * rho_e + ln * rho_l + en * rho_e + p.acc_rel * vn) +
                    2.0f * dr + 4.8e-7f * vr;
    const float2* meta = lds_meta + 4 * h;
    asm volatile("" : "+v"(meta));
    const int kl_h = pbase + 4 * h;
#pragma unroll
    for (int t = 0; t < NT; ++t) {
#pragma unroll
      for (int v = 0; v < 16; ++v) {
        const int io = t * 32 + (v & 3) + 8 * (v >> 2);
        const int kl = kl_h + io;
        const float2 m = meta[io];  // |c|^2, |c|
        const float sc = m.x - 2.0f * acc[t][v] * inv_den;
        const float e = fmaf(K, m.y, fmaf(2.39e-7f, m.x, 1e-30f));
        const bool ok = kl < cnt;
        const float lb = ok ? sc - e : INFINITY, ub = ok ? sc + e : INFINITY;
        U = fminf(U, ub);
        const bool lt1 = lb < b1, lt2 = lb < b2, lt3 = lb < b3;
        b3 = lt2 ? b2 : (lt3 ? lb : b3);
        k3 = lt2 ? k2 : (lt3 ? kl : k3);
        b2 = lt1 ? b1 : (lt2 ? lb : b2);
        k2 = lt1 ? k1 : (lt2 ? kl : k2);
        b1 = lt1 ? lb : b1;
        k1 = lt1 ? kl : k1;
      }
    }
    __syncthreads();  // meta / staging buffers are rewritten by the next pass
  }

  // Row decision: candidates are the k with lower bound <= U (the least upper bound).  Each
  // lane tracked its 3 smallest lower bounds, so up to 2 per lane are listed exactly; a
  // lane whose 3rd also qualifies may hold more -> re-score the whole segment.
  U = fminf(U, __shfl_xor(U, 32));
  const float b1p = __shfl_xor(b1, 32), b2p = __shfl_xor(b2, 32), b3p = __shfl_xor(b3, 32);
  const int k1p = __shfl_xor(k1, 32), k2p = __shfl_xor(k2, 32);
  const bool q1 = b1 <= U, q2 = b2 <= U, q1p = b1p <= U, q2p = b2p <= U;
  const int ncand = (int)q1 + (int)q2 + (int)q1p + (int)q2p;
  const bool overflow = b3 <= U || b3p <= U || ncand == 0;
  const bool definitive = !overflow && ncand == 1;
  if (h == 0 && row_valid && definitive) {
    const int k = q1 ? k1 : k1p;
    p.out_local[my_row] = k;
    p.out_global[my_row] = cand_global(p, cbase, k);
  }
  WorkItem w{};
  w.row = my_row;
  w.seg = s;
  if (overflow) {
    w.n = -1;
  } else {
    // ascending local index so the re-score keeps the lowest index on exact ties
    int c4[4] = {q1 ? k1 : INT_MAX, q2 ? k2 : INT_MAX, q1p ? k1p : INT_MAX, q2p ? k2p : INT_MAX};
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 3 - i; ++j) {
        const int a = c4[j], bq = c4[j + 1];
        c4[j] = min(a, bq);
        c4[j + 1] = max(a, bq);
      }
    w.n = ncand;
#pragma unroll
    for (int i = 0; i < 4; ++i) w.cand[i] = c4[i];
  }
  push_work(p, h == 0 && row_valid && !definitive, lane, w);
}

// Exact re-score of the rows the screening could not decide: one wave per row.  The
// row's vector is rebuilt with the reference's fp32 operation sequence (x - ca, /n1,
// - cb, /n2 with n = fl(sqrt(sum^2)) + 1e-8) and distances are taken in fp64.
template <int RL, bool NORM>
__global__ __launch_bounds__(256) void assign_rescore_kernel(AssignParams p) {
  const int lane = threadIdx.x & 63;
  const int wid = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int nw = gridDim.x * 4;
  const int64_t nitems_raw = *p.work_count;
  const int64_t nitems = nitems_raw < p.work_cap ? nitems_raw : p.work_cap;
  constexpr int kMaxV = 4;               // float4 per lane: dim <= 1024 keeps the row in registers
  const int nv = p.dim / 4;
  for (int64_t it = wid; it < nitems; it += nw) {
    const WorkItem w = p.work[it];
    const float* xr = p.x + (int64_t)w.row * p.dim;
    float4 v[kMaxV];
    double ss = 0.0;
#pragma unroll
    for (int m = 0; m < kMaxV; ++m) {
      const int i = lane + 64 * m;
      if (i < nv) {
        float4 a = reinterpret_cast<const float4*>(xr)[i];
        if (RL >= 1) {
          const float4 c = reinterpret_cast<const float4*>(p.ca + (int64_t)p.ca_idx[w.row] * p.dim)[i];
          a = make_float4(a.x - c.x, a.y - c.y, a.z - c.z, a.w - c.w);
        }
        if (RL >= 2) {
          if (NORM) {
            const float d1 = p.den_in[w.row];
            a = make_float4(a.x / d1, a.y / d1, a.z / d1, a.w / d1);
          }
          const float4 c = reinterpret_cast<const float4*>(p.cb + (int64_t)p.cb_idx[w.row] * p.dim)[i];
          a = make_float4(a.x - c.x, a.y - c.y, a.z - c.z, a.w - c.w);
        }
        v[m] = a;
        ss += (double)a.x * a.x + (double)a.y * a.y + (double)a.z * a.z + (double)a.w * a.w;
      } else {
        v[m] = make_float4(0.f, 0.f, 0.f, 0.f);
      }
    }
    if (NORM && RL >= 1) {
      float den;
      if (RL == 1 && p.den_out) {
        den = p.den_out[w.row];  // written by the screen for every valid row
      } else {
        den = (float)sqrt(wave_sum(ss)) + 1e-8f;
      }
#pragma unroll
      for (int m = 0; m < kMaxV; ++m)
        v[m] = make_float4(v[m].x / den, v[m].y / den, v[m].z / den, v[m].w / den);
    }
    const bool penalty = w.n == -2;
    const int base = p.cand_base[w.seg];
    int n;
    if (w.n >= 0) n = w.n;
    else if (penalty) n = p.n_centers;
    else if (w.n == -1) n = p.cand_count[w.seg];
    else n = 0;
    double best = INFINITY;
    float bestkey = INFINITY;
    int bestl = -1, bestg = -1;
    for (int j = 0; j < n; ++j) {
      const int kl = w.n >= 0 ? w.cand[j] : j;
      const int g = penalty ? j : cand_global(p, base, kl);
      const float* cr = p.centers + (int64_t)g * p.dim;
      double acc = 0.0;
#pragma unroll
      for (int m = 0; m < kMaxV; ++m) {
        const int i = lane + 64 * m;
        if (i < nv) {
          const float4 c = reinterpret_cast<const float4*>(cr)[i];
          const double d0 = (double)v[m].x - c.x, d1 = (double)v[m].y - c.y, d2 = (double)v[m].z - c.z,
                       d3 = (double)v[m].w - c.w;
          acc += d0 * d0 + d1 * d1 + d2 * d2 + d3 * d3;
        }
      }
      acc = wave_sum(acc);
      if (penalty) {
        // reference: fl32(sqrt(fl32(d^2))) + 10000 in fp32, first index on ties
        const float d = (float)sqrt((double)(float)acc);
        const float key = d + 10000.0f;
        if (key < bestkey) { bestkey = key; bestl = -1; bestg = g; }
      } else if (acc < best) {
        best = acc;
        bestl = kl;
        bestg = g;
      }
    }
    if (bestg < 0 && n > 0) {  // every distance NaN: keep memory-safe ids (first candidate)
      bestl = penalty ? -1 : (w.n >= 0 ? w.cand[0] : 0);
      bestg = penalty ? 0 : cand_global(p, base, w.n >= 0 ? w.cand[0] : 0);
    }
    if (lane == 0) {
      p.out_local[w.row] = bestl;
      p.out_global[w.row] = bestg;
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
__global__ __launch_bounds__(256) void pairwise_distance_kernel(const float* __restrict__ x, int64_t n, int dim,
                                                                const float* __restrict__ c, int k,
                                                                float* __restrict__ out) {
  __shared__ float xs[kPdTile][33];
  __shared__ float cs[kPdTile][33];
  const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
  const int64_t r0 = (int64_t)blockIdx.x * kPdTile;
  const int c0 = blockIdx.y * kPdTile;
  float acc[4][4] = {};
  float xq[4] = {}, cq[4] = {};
  for (int d0 = 0; d0 < dim; d0 += 32) {
    for (int i = threadIdx.x; i < kPdTile * 32; i += 256) {
      const int rr = i >> 5, dd = i & 31;
      xs[rr][dd] = (r0 + rr < n) ? x[(r0 + rr) * dim + d0 + dd] : 0.f;
      cs[rr][dd] = (c0 + rr < k) ? c[(int64_t)(c0 + rr) * dim + d0 + dd] : 0.f;
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
        xq[i] = fmaf(a[i], a[i], xq[i]);
        cq[i] = fmaf(bb[i], bb[i], cq[i]);
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = fmaf(a[i], bb[j], acc[i][j]);
      }
    }
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int64_t rr = r0 + ty + 16 * i;
    if (rr >= n) continue;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int cc = c0 + tx + 16 * j;
      if (cc >= k) continue;
      const float d2 = (-2.f * acc[i][j] + xq[i]) + cq[j];
      out[rr * k + cc] = sqrtf(fmaxf(d2, 0.f));
    }
  }
}


// ---------------------------------------------------------------------------
// MFMA numerics probe: D = A.B + C with ONE v_mfma_f32_32x32x16_bf16 (32x16 A,
// 16x32 B, 32x32 C/D, all row-major).  Used by tests/test_mfma_numerics.py to pin
// the accumulation model the screening error bound relies on.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(64) void mfma_probe_kernel(const uint16_t* __restrict__ a, const uint16_t* __restrict__ b,
                                                        const float* __restrict__ c, float* __restrict__ d) {
  const int l = threadIdx.x, i = l & 31, h = l >> 5;
  bf16x8 av, bv;
  f32x16 acc;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    av[j] = __builtin_bit_cast(__bf16, a[i * 16 + 8 * h + j]);
    bv[j] = __builtin_bit_cast(__bf16, b[(8 * h + j) * 32 + i]);
  }
#pragma unroll
  for (int v = 0; v < 16; ++v) acc[v] = c[((v & 3) + 8 * (v >> 2) + 4 * h) * 32 + i];
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av, bv, acc, 0, 0, 0);
#pragma unroll
  for (int v = 0; v < 16; ++v) d[((v & 3) + 8 * (v >> 2) + 4 * h) * 32 + i] = acc[v];
}

bool g_attr_done = false;
int ensure_attrs() {
  if (g_attr_done) return RQSID_OK;
  hipError_t e;
  {
    const void* ks[] = {(const void*)assign_screen_kernel<4, 0, false>, (const void*)assign_screen_kernel<4, 1, false>,
                        (const void*)assign_screen_kernel<4, 1, true>,  (const void*)assign_screen_kernel<4, 2, false>,
                        (const void*)assign_screen_kernel<4, 2, true>,  (const void*)assign_screen_kernel<8, 0, false>,
                        (const void*)assign_screen_kernel<8, 1, false>, (const void*)assign_screen_kernel<8, 1, true>,
                        (const void*)assign_screen_kernel<8, 2, false>, (const void*)assign_screen_kernel<8, 2, true>};
    for (int i = 0; i < 10; ++i) {
      e = hipFuncSetAttribute(ks[i], hipFuncAttributeMaxDynamicSharedMemorySize,
                              i < 5 ? ScreenLayout<4>::kBytes : ScreenLayout<8>::kBytes);
      if (e != hipSuccess) return fail(RQSID_E_LAUNCH, "set smem attr (screen %d): %s", i, hipGetErrorString(e));
    }
  }
  e = hipFuncSetAttribute((const void*)bucket_hist_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                          kBucketLdsBins * 4);
  if (e != hipSuccess) return fail(RQSID_E_LAUNCH, "set smem attr (hist): %s", hipGetErrorString(e));
  e = hipFuncSetAttribute((const void*)bucket_scatter_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                          kBucketLdsBins * 4);
  if (e != hipSuccess) return fail(RQSID_E_LAUNCH, "set smem attr (scatter): %s", hipGetErrorString(e));
  g_attr_done = true;
  return RQSID_OK;
}

inline int64_t cdiv(int64_t a, int64_t b) { return (a + b - 1) / b; }
inline unsigned grid_cap(int64_t want, int64_t cap) { return (unsigned)(want < 1 ? 1 : (want > cap ? cap : want)); }

template <int NT>
void launch_screen(const AssignParams& p, int rl, bool norm, unsigned grid, hipStream_t st) {
  const size_t lds = ScreenLayout<NT>::kBytes;
  if (rl == 0) hipLaunchKernelGGL((assign_screen_kernel<NT, 0, false>), dim3(grid), dim3(256), lds, st, p);
  else if (rl == 1 && norm) hipLaunchKernelGGL((assign_screen_kernel<NT, 1, true>), dim3(grid), dim3(256), lds, st, p);
  else if (rl == 1) hipLaunchKernelGGL((assign_screen_kernel<NT, 1, false>), dim3(grid), dim3(256), lds, st, p);
  else if (norm) hipLaunchKernelGGL((assign_screen_kernel<NT, 2, true>), dim3(grid), dim3(256), lds, st, p);
  else hipLaunchKernelGGL((assign_screen_kernel<NT, 2, false>), dim3(grid), dim3(256), lds, st, p);
}

}  // namespace

// ===========================================================================
// C ABI
// ===========================================================================
extern "C" {

int rqsid_version(void) { return 1; }
const char* rqsid_last_error(void) { return g_err; }

int rqsid_prepare_centers(const float* centers, int64_t k, int32_t dim, uint16_t* c_split, float* c_meta,
                          void* stream) {
  if (!centers || !c_split || !c_meta || k < 0 || dim <= 0 || dim % kChunk)
    return fail(RQSID_E_ARG, "prepare_centers: bad arguments (k=%lld dim=%d)", (long long)k, dim);
  if (k == 0) return RQSID_OK;
  hipLaunchKernelGGL(prepare_centers_kernel, dim3((unsigned)cdiv(k, 4)), dim3(256), 0, (hipStream_t)stream,
                     centers, k, dim, c_split, reinterpret_cast<float4*>(c_meta));
  return check_launch("prepare_centers");
}

int32_t rqsid_assign_tile_rows(void) { return kTileRows; }
int32_t rqsid_centroid_tile_rows(void) { return kAccTileRows; }

int64_t rqsid_bucket_workspace_bytes(int64_t n, int32_t n_segments) {
  (void)n;
  return ((int64_t)n_segments * 2 + 64) * 4;
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
  if (hipMemsetAsync(counts, 0, (size_t)S * 4, st) != hipSuccess) return fail(RQSID_E_LAUNCH, "bucket: memset");
  const size_t lds = S <= kBucketLdsBins ? (size_t)S * 4 : 0;
  if (n > 0) {
    hipLaunchKernelGGL(bucket_hist_kernel, dim3(grid_cap(cdiv(n, 256 * 16), 2048)), dim3(256), lds, st, keys, n,
                       S, counts);
    if ((rc = check_launch("bucket_hist"))) return rc;
  }
  hipLaunchKernelGGL(bucket_scan_kernel, dim3(1), dim3(1024), 0, st, counts, S, tile_rows, seg_row_off,
                     seg_tile_off, cursor);
  if ((rc = check_launch("bucket_scan"))) return rc;
  if (n > 0) {
    const unsigned blocks = S <= kBucketLdsBins ? (unsigned)cdiv(n, kScatterRowsPerBlock)
                                                : grid_cap(cdiv(n, 256 * 16), 2048);
    hipLaunchKernelGGL(bucket_scatter_kernel, dim3(blocks), dim3(256), lds, st, keys, n, S, cursor, row_index);
    if ((rc = check_launch("bucket_scatter"))) return rc;
  }
  return RQSID_OK;
}

int64_t rqsid_assign_workspace_bytes(int64_t n_rows) { return 256 + (n_rows > 0 ? n_rows : 0) * (int64_t)sizeof(WorkItem); }

int rqsid_assign(const float* x, int64_t n_rows, int32_t dim, const int32_t* row_index, int32_t n_segments,
                 const int32_t* seg_row_off, const int32_t* seg_tile_off, int64_t max_tiles, const float* centers,
                 const uint16_t* c_split, const float* c_meta, int32_t n_centers, const int32_t* cand_base,
                 const int32_t* cand_count, int32_t cand_count_max, const int32_t* cand_idx,
                 const uint8_t* seg_flags, int32_t res_levels, int32_t res_normalize, const float* ca,
                 const int32_t* ca_idx, const float* cb, const int32_t* cb_idx, const float* den_in,
                 float* den_out, int32_t* out_local, int32_t* out_global, void* workspace,
                 int64_t workspace_bytes, void* stream) {
  if (dim <= 0 || dim % kChunk || dim > 1024 || n_rows < 0 || n_segments <= 0 || !seg_row_off ||
      !seg_tile_off || !centers || !c_split || !c_meta || !cand_base || !cand_count || !out_local ||
      !out_global || n_centers <= 0 || cand_count_max < 0 || max_tiles < 0 || n_rows > INT32_MAX ||
      res_levels < 0 || res_levels > 2)
    return fail(RQSID_E_ARG, "assign: bad arguments (n=%lld dim=%d S=%d K=%d levels=%d)", (long long)n_rows, dim,
                n_segments, n_centers, res_levels);
  if ((res_levels >= 1 && (!ca || !ca_idx)) || (res_levels == 2 && (!cb || !cb_idx || (res_normalize && !den_in))))
    return fail(RQSID_E_ARG, "assign: residual inputs missing for res_levels=%d", res_levels);
  if (!workspace || workspace_bytes < rqsid_assign_workspace_bytes(n_rows))
    return fail(RQSID_E_WORKSPACE, "assign: workspace too small");
  if (n_rows == 0 || max_tiles == 0) return RQSID_OK;
  if (max_tiles > INT32_MAX) return fail(RQSID_E_ARG, "assign: too many tiles");
  int rc = ensure_attrs();
  if (rc) return rc;
  hipStream_t st = (hipStream_t)stream;
  AssignParams p{};
  p.x = x;
  p.dim = dim;
  p.row_index = row_index;
  p.n_segments = n_segments;
  p.seg_row_off = seg_row_off;
  p.seg_tile_off = seg_tile_off;
  p.centers = centers;
  p.c_split = c_split;
  p.c_meta = c_meta;
  p.n_centers = n_centers;
  p.cand_base = cand_base;
  p.cand_count = cand_count;
  p.cand_idx = cand_idx;
  p.seg_flags = seg_flags;
  p.out_local = out_local;
  p.out_global = out_global;
  p.work_count = (int32_t*)workspace;
  p.work = (WorkItem*)((char*)workspace + 256);
  p.work_cap = n_rows;
  p.acc_rel = accumulation_rel(dim);
  p.ca = ca;
  p.ca_idx = ca_idx;
  p.cb = cb;
  p.cb_idx = cb_idx;
  p.den_in = den_in;
  p.den_out = den_out;
  const bool norm = res_normalize != 0;
  if (hipMemsetAsync(workspace, 0, 256, st) != hipSuccess) return fail(RQSID_E_LAUNCH, "assign: memset");
  if (cand_count_max <= 128) launch_screen<4>(p, res_levels, norm, (unsigned)max_tiles, st);
  else launch_screen<8>(p, res_levels, norm, (unsigned)max_tiles, st);
  if ((rc = check_launch("assign_screen"))) return rc;
  const dim3 g(grid_cap(cdiv(n_rows, 4), 2048));
  if (res_levels == 0) hipLaunchKernelGGL((assign_rescore_kernel<0, false>), g, dim3(256), 0, st, p);
  else if (res_levels == 1 && norm) hipLaunchKernelGGL((assign_rescore_kernel<1, true>), g, dim3(256), 0, st, p);
  else if (res_levels == 1) hipLaunchKernelGGL((assign_rescore_kernel<1, false>), g, dim3(256), 0, st, p);
  else if (norm) hipLaunchKernelGGL((assign_rescore_kernel<2, true>), g, dim3(256), 0, st, p);
  else hipLaunchKernelGGL((assign_rescore_kernel<2, false>), g, dim3(256), 0, st, p);
  return check_launch("assign_rescore");
}

int rqsid_residual(const float* x, int64_t n, int32_t dim, const float* centers, int32_t n_centers,
                   const int32_t* center_id, const int32_t* group_dims, int32_t n_groups, int32_t normalize,
                   float* out, void* stream) {
  if (!x || !centers || !center_id || !out || dim <= 0 || dim % 4 || n < 0 || n_centers <= 0 ||
      (normalize && (!group_dims || n_groups <= 0 || n_groups > kMaxGroups)))
    return fail(RQSID_E_ARG, "residual: bad arguments (dim=%d groups=%d)", dim, n_groups);
  if (n == 0) return RQSID_OK;
  hipLaunchKernelGGL(residual_kernel, dim3(grid_cap(cdiv(n, 4), 8192)), dim3(256), 0, (hipStream_t)stream, x, n,
                     dim, centers, n_centers, center_id, group_dims, normalize ? n_groups : 1, normalize, out);
  return check_launch("residual");
}

int rqsid_scale_groups(const float* x, int64_t n, int32_t dim, const int32_t* group_dims, int32_t n_groups,
                       const float* weights, float* out, void* stream) {
  if (!x || !group_dims || !weights || !out || n_groups <= 0 || dim <= 0 || n < 0)
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

int rqsid_mfma_probe(const uint16_t* a, const uint16_t* b, const float* c, float* d, void* stream) {
  if (!a || !b || !c || !d) return fail(RQSID_E_ARG, "mfma_probe: null argument");
  hipLaunchKernelGGL(mfma_probe_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, a, b, c, d);
  return check_launch("mfma_probe");
}

int rqsid_pairwise_distance(const float* x, int64_t n, int32_t dim, const float* centers, int32_t k, float* out,
                            void* stream) {
  if (!x || !centers || !out || n < 0 || k <= 0 || dim <= 0 || dim % 32)
    return fail(RQSID_E_ARG, "pairwise_distance: bad arguments");
  if (n == 0) return RQSID_OK;
  hipLaunchKernelGGL(pairwise_distance_kernel, dim3((unsigned)cdiv(n, kPdTile), (unsigned)cdiv(k, kPdTile)),
                     dim3(256), 0, (hipStream_t)stream, x, n, dim, centers, k, out);
  return check_launch("pairwise_distance");
}

}  // extern "C"
