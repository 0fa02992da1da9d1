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

// Rigorous bound of the bf16x3 screening error on x.c relative to |x||c|
// (DESIGN.md §"Screening bound"): split representation 3.1*2^-16 plus the fp32
// accumulation of <= 3*dim/16*(16+1) additions, doubled for the -2 x.c term, with
// 5% slack. Evaluated on the host per dim.
inline float screening_tau(int dim) {
  const double rep = 3.1 * std::ldexp(1.0, -16);
  const double acc = (3.0 * dim / 16.0 * 17.0 + 8.0) * std::ldexp(1.0, -24);
  return (float)(2.0 * (rep + acc) * 1.05);
}

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
  const float* c_sq;
  const float* c_norm;
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
  float tau;
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
                                                              float* __restrict__ csq,
                                                              float* __restrict__ cn) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= k) return;
  const float* cr = c + row * dim;
  const int nch = dim / kChunk;
  double s = 0.0;
  for (int i = lane; i < dim; i += 64) {
    const float v = cr[i];
    const uint16_t hb = bf16_bits(v);
    const uint16_t lb = bf16_bits(v - bf16_to_f32(hb));
    const int ch = i / kChunk, j = i % kChunk;
    uint16_t* dst = split + (row * nch + ch) * (2 * kChunk);
    dst[j] = hb;
    dst[kChunk + j] = lb;
    s += (double)v * (double)v;
  }
  s = wave_sum(s);
  if (lane == 0) {
    csq[row] = (float)s;
    cn[row] = (float)sqrt(s);
  }
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
// assignment: bf16x3 MFMA screening
// ---------------------------------------------------------------------------
template <int NT>
struct ScreenLayout {
  static constexpr int kCBytes = NT * 32 * kLdsRow;
  static constexpr int kStage = kXStageBytes + kCBytes;
  static constexpr int kMeta = 2 * kStage;             // csq[NT*32], cn[NT*32]
  static constexpr int kBytes = kMeta + NT * 32 * 8;
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

template <int NT>
__global__ __launch_bounds__(256, (NT <= 4 ? 2 : 1)) void assign_screen_kernel(AssignParams p) {
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
  // X staging sources: rows 8*i + rs of this wave's 32 rows
  const float* xsrc[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int rr = 8 * i + rs;
    const int grow = __shfl(my_row, rr);
    xsrc[i] = p.x + (int64_t)grow * p.dim + q * 4;
  }
  const int xw_off = wave * (kRowsPerWave * kLdsRow);

  float U = INFINITY, b1 = INFINITY, b2 = INFINITY;
  int k1 = -1, k2 = -1;
  float xsq = 0.f;
  float xn = 0.f;
  float* lds_csq = reinterpret_cast<float*>(smem + L::kMeta);  // float2 {|c|^2, |c|} per candidate

  const int npass = (cnt + NT * 32 - 1) / (NT * 32);
  for (int pass = 0; pass < npass; ++pass) {
    const int pbase = pass * NT * 32;
    // centre staging sources: candidate rows j*32 + wave*8 + rs
    const uint16_t* csrc[NT];
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      const int il = j * 32 + wave * 8 + rs;
      const int kl = pbase + il < cnt ? pbase + il : 0;
      const int cg = cand_global(p, cbase, kl);
      csrc[j] = p.c_split + (int64_t)cg * nch * (2 * kChunk) + q * 8;
    }
    if (tid < NT * 32) {
      const int kl = pbase + tid < cnt ? pbase + tid : 0;
      const int cg = cand_global(p, cbase, kl);
      reinterpret_cast<float2*>(lds_csq)[tid] = make_float2(p.c_sq[cg], p.c_norm[cg]);
    }

    f32x16 acc[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int v = 0; v < 16; ++v) acc[t][v] = 0.f;

    u32x4 xs[4], cs[NT];
    auto gload = [&](int c) {
#pragma unroll
      for (int i = 0; i < 4; ++i) xs[i] = *reinterpret_cast<const u32x4*>(xsrc[i] + c * kChunk);
#pragma unroll
      for (int j = 0; j < NT; ++j) cs[j] = *reinterpret_cast<const u32x4*>(csrc[j] + c * (2 * kChunk));
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

    gload(0);
    swrite(0);
    __syncthreads();
    for (int c = 0; c < nch; ++c) {
      if (c + 1 < nch) gload(c + 1);
      const unsigned char* xb = smem + (c & 1) * L::kStage + xw_off + r * kLdsRow;
      const unsigned char* cb = smem + (c & 1) * L::kStage + kXStageBytes + r * kLdsRow;
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const int q0 = 4 * ks + 2 * h;
        const float4 xa = *reinterpret_cast<const float4*>(xb + ((q0 ^ swz(r)) << 4));
        const float4 xc = *reinterpret_cast<const float4*>(xb + (((q0 + 1) ^ swz(r)) << 4));
        const float xv[8] = {xa.x, xa.y, xa.z, xa.w, xc.x, xc.y, xc.z, xc.w};
        bf16x8 bh, bl;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const __bf16 hv = (__bf16)xv[e];
          bh[e] = hv;
          bl[e] = (__bf16)(xv[e] - (float)hv);
          if (pass == 0) xsq = fmaf(xv[e], xv[e], xsq);
        }
        const int qh = 2 * ks + h, ql = 4 + 2 * ks + h;
#pragma unroll
        for (int t = 0; t < NT; ++t) {
          const unsigned char* ct = cb + t * 32 * kLdsRow;
          const bf16x8 ah = *reinterpret_cast<const bf16x8*>(ct + ((qh ^ swz(r)) << 4));
          const bf16x8 al = *reinterpret_cast<const bf16x8*>(ct + ((ql ^ swz(r)) << 4));
          acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al, bh, acc[t], 0, 0, 0);
          acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bl, acc[t], 0, 0, 0);
          acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bh, acc[t], 0, 0, 0);
        }
      }
      if (c + 1 < nch) swrite((c + 1) & 1);
      __syncthreads();
    }
    if (pass == 0) {
      const float tot = xsq + __shfl_xor(xsq, 32);
      xn = sqrtf(tot) * 1.0001f;
    }
    // epilogue: bounds and top-2 lower bounds per lane.  The per-half base pointer is
    // made opaque so every (t, v) read is base + immediate offset instead of a
    // precomputed address per candidate (which the scheduler otherwise keeps live).
    const float2* meta = reinterpret_cast<const float2*>(lds_csq) + 4 * h;
    asm volatile("" : "+v"(meta));
    const int kl_h = pbase + 4 * h;
#pragma unroll
    for (int t = 0; t < NT; ++t) {
#pragma unroll
      for (int v = 0; v < 16; ++v) {
        const int io = t * 32 + (v & 3) + 8 * (v >> 2);
        const int kl = kl_h + io;
        if (kl < cnt) {
          const float2 m = meta[io];
          const float csq = m.x;
          const float sc = csq - 2.f * acc[t][v];
          const float e = p.tau * xn * m.y + 2.5e-7f * csq + 1e-30f;
          const float lb = sc - e, ub = sc + e;
          U = fminf(U, ub);
          const bool lt1 = lb < b1, lt2 = lb < b2;
          b2 = lt1 ? b1 : (lt2 ? lb : b2);
          k2 = lt1 ? k1 : (lt2 ? kl : k2);
          b1 = lt1 ? lb : b1;
          k1 = lt1 ? kl : k1;
        }
      }
    }
    __syncthreads();  // lds_csq / staging buffers are rewritten by the next pass
  }

  U = fminf(U, __shfl_xor(U, 32));
  const float b1p = __shfl_xor(b1, 32), b2p = __shfl_xor(b2, 32);
  const int k1p = __shfl_xor(k1, 32);
  const bool q1 = b1 <= U, q2 = b2 <= U, q1p = b1p <= U, q2p = b2p <= U;
  const int ncand = (int)q1 + (int)q1p;
  const bool overflow = q2 || q2p || ncand == 0;
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
    w.n = 2;
    w.cand[0] = min(k1, k1p);
    w.cand[1] = max(k1, k1p);
  }
  push_work(p, h == 0 && row_valid && !definitive, lane, w);
}

// fp64 re-score of the rows the screening could not decide: one wave per row.
__global__ __launch_bounds__(256) void assign_rescore_kernel(AssignParams p) {
  const int lane = threadIdx.x & 63;
  const int wid = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int nw = gridDim.x * 4;
  const int64_t nitems_raw = *p.work_count;
  const int64_t nitems = nitems_raw < p.work_cap ? nitems_raw : p.work_cap;
  const int nv = p.dim / 4;  // float4 per row
  for (int64_t it = wid; it < nitems; it += nw) {
    const WorkItem w = p.work[it];
    const float* xr = p.x + (int64_t)w.row * p.dim;
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
      for (int i = lane; i < nv; i += 64) {
        const float4 a = reinterpret_cast<const float4*>(xr)[i];
        const float4 c = reinterpret_cast<const float4*>(cr)[i];
        const double d0 = (double)a.x - c.x, d1 = (double)a.y - c.y, d2 = (double)a.z - c.z,
                     d3 = (double)a.w - c.w;
        acc += d0 * d0 + d1 * d1 + d2 * d2 + d3 * d3;
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

bool g_attr_done = false;
int ensure_attrs() {
  if (g_attr_done) return RQSID_OK;
  hipError_t e;
  e = hipFuncSetAttribute((const void*)assign_screen_kernel<4>, hipFuncAttributeMaxDynamicSharedMemorySize,
                          ScreenLayout<4>::kBytes);
  if (e != hipSuccess) return fail(RQSID_E_LAUNCH, "set smem attr (NT=4): %s", hipGetErrorString(e));
  e = hipFuncSetAttribute((const void*)assign_screen_kernel<8>, hipFuncAttributeMaxDynamicSharedMemorySize,
                          ScreenLayout<8>::kBytes);
  if (e != hipSuccess) return fail(RQSID_E_LAUNCH, "set smem attr (NT=8): %s", hipGetErrorString(e));
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

}  // namespace

// ===========================================================================
// C ABI
// ===========================================================================
extern "C" {

int rqsid_version(void) { return 1; }
const char* rqsid_last_error(void) { return g_err; }

int rqsid_prepare_centers(const float* centers, int64_t k, int32_t dim, uint16_t* c_split, float* c_sqnorm,
                          float* c_norm, void* stream) {
  if (!centers || !c_split || !c_sqnorm || !c_norm || k < 0 || dim <= 0 || dim % kChunk)
    return fail(RQSID_E_ARG, "prepare_centers: bad arguments (k=%lld dim=%d)", (long long)k, dim);
  if (k == 0) return RQSID_OK;
  hipLaunchKernelGGL(prepare_centers_kernel, dim3((unsigned)cdiv(k, 4)), dim3(256), 0, (hipStream_t)stream,
                     centers, k, dim, c_split, c_sqnorm, c_norm);
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
                 const uint16_t* c_split, const float* c_sqnorm, const float* c_norm, int32_t n_centers,
                 const int32_t* cand_base, const int32_t* cand_count, int32_t cand_count_max,
                 const int32_t* cand_idx, const uint8_t* seg_flags, int32_t* out_local, int32_t* out_global,
                 void* workspace, int64_t workspace_bytes, void* stream) {
  if (dim <= 0 || dim % kChunk || n_rows < 0 || n_segments <= 0 || !seg_row_off || !seg_tile_off ||
      !centers || !c_split || !c_sqnorm || !c_norm || !cand_base || !cand_count || !out_local || !out_global ||
      n_centers <= 0 || cand_count_max < 0 || max_tiles < 0 || n_rows > INT32_MAX)
    return fail(RQSID_E_ARG, "assign: bad arguments (n=%lld dim=%d S=%d K=%d)", (long long)n_rows, dim,
                n_segments, n_centers);
  if (!workspace || workspace_bytes < rqsid_assign_workspace_bytes(n_rows))
    return fail(RQSID_E_WORKSPACE, "assign: workspace too small");
  if (n_rows == 0 || max_tiles == 0) return RQSID_OK;
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
  p.c_sq = c_sqnorm;
  p.c_norm = c_norm;
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
  p.tau = screening_tau(dim);
  if (hipMemsetAsync(workspace, 0, 256, st) != hipSuccess) return fail(RQSID_E_LAUNCH, "assign: memset");
  if (max_tiles > INT32_MAX) return fail(RQSID_E_ARG, "assign: too many tiles");
  if (cand_count_max <= 128) {
    hipLaunchKernelGGL(assign_screen_kernel<4>, dim3((unsigned)max_tiles), dim3(256), ScreenLayout<4>::kBytes, st, p);
  } else {
    hipLaunchKernelGGL(assign_screen_kernel<8>, dim3((unsigned)max_tiles), dim3(256), ScreenLayout<8>::kBytes, st, p);
  }
  if ((rc = check_launch("assign_screen"))) return rc;
  hipLaunchKernelGGL(assign_rescore_kernel, dim3(grid_cap(cdiv(n_rows, 4), 2048)), dim3(256), 0, st, p);
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
