// assign.hip — exact segmented nearest-centre assignment for gfx950 (rqsid_assign, rqsid_prepare_centers).
//
// Replaces pairwise_distance_full + torch.argmin (balancekmeans/__init__.py:489-534, 576-603) and the
// masked reassignment / prediction of hierarchical_rq_kmeans.py:839-966, 1146-1305 and
// simplified_semantic_id_generator.py:145-161, 305-331.
//
// Two kernels:
//  1. assign_screen_kernel — a segmented "grouped GEMM + argmin".  A work tile is 128 rows of ONE
//     segment (parent cluster / (l1,l2) group) against that segment's candidate centres.  X·Cᵀ runs on
//     v_mfma_f32_32x32x16_f16 with ONE fp16 term per operand (x rounded to fp16 on the fly, centres
//     pre-rounded by rqsid_prepare_centers).  A rigorous per-(row, candidate) error bound, built from the
//     exact rounding residuals |x - fp16(x)| (measured on the fly) and |c - fp16(c)| (prepared) plus a
//     pessimistic model of the MFMA's internal accumulation, decides whether the row's nearest candidate
//     is certain.  Rows where the bound admits several candidates go to a work list.
//     Data movement: x rows and fp16 centre chunks stream HBM/L2 -> LDS by LDS-DMA
//     (global_load_lds_dwordx4, issued in inline asm so hipcc does not drain it) through an S-stage ring,
//     one barrier per 32-dim chunk; x rows are a per-lane row gather (rows are bucketed by segment).
//     Centres are the MFMA A operand (32 candidates on M) and rows the B operand, so each lane owns ONE
//     row and 16 of its candidates: the argmin is in-register plus one cross-half exchange.
//  2. assign_rescore_kernel — exact fp64 re-score of the listed rows (one wave per row), rebuilding the
//     row's vector with the reference's fp32 operation sequence.  The returned ID is therefore the exact
//     argmin (lowest index on exact ties), independent of any summation order.
//
// Fused residual chain (res_levels 1/2): the vector assigned for row i of segment s is
//     RL0: x_i      RL1: x_i - ca[seg_ca[s]]      RL2: (x_i - ca[seg_ca[s]]) [/ den_in[i]] - cb[seg_cb[s]]
// (NORM additionally divides by ||.|| + 1e-8), i.e. _compute_residuals_with_centers
// (hierarchical_rq_kmeans.py:1088-1128) / simplified :78-96 without materialising residual matrices.
// The residual centres are per-SEGMENT constants (a level's segment determines the parent IDs), so
// they are staged once per tile in LDS.
#include "assign_common.h"

namespace rqsid {
namespace {

// largest |c| of the table as float bits (positive floats order like their bit patterns; a NaN
// sorts above infinity and disables scaling)
__global__ __launch_bounds__(256) void centers_absmax_kernel(const float* __restrict__ c, int64_t n,
                                                             unsigned* __restrict__ out) {
  unsigned m = 0;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
    m = max(m, __float_as_uint(fabsf(c[i])));
  for (int o = 32; o > 0; o >>= 1) m = max(m, (unsigned)__shfl_xor((int)m, o));
  if ((threadIdx.x & 63) == 0) atomicMax(out, m);
}

// ---------------------------------------------------------------------------
// centre preparation
// ---------------------------------------------------------------------------
// c16 [k][dim/32][2][32]: per centre and 32-dim chunk, 32 hi = fp16(c 2^s) then 32 lo = fp16((c 2^s -
// hi) 2^12) (the 3-term screen's second term; scaled by 2^12 so it stays in the fp16 normal range), so
// one chunk's two terms are one 128-B piece (tools/probe/dma_probe2: gathered 128-B pieces stream 9-14 %
// faster than 64-B ones).  meta[k] = {|c|^2, |c|,
// |c - (hi + lo 2^-12) 2^-s|, |c - hi 2^-s|}; meta[k_total].x holds the absmax bits while this runs
// (centers_absmax_kernel) and 2^-s afterwards (centers_scale_kernel).
__global__ __launch_bounds__(256) void prepare_centers_kernel(const float* __restrict__ c, int64_t k, int dim,
                                                              _Float16* __restrict__ c16, float4* __restrict__ meta) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= k) return;
  const int sx = table_scale_exp(reinterpret_cast<const unsigned*>(meta + k)[0]);
  const float* cr = c + row * dim;
  double s = 0.0, s1 = 0.0, s2 = 0.0;
  for (int i = lane; i < dim; i += 64) {
    const float v = cr[i];
    const float vs = ldexpf(v, sx);
    const _Float16 hv = to_f16(vs);
    const float r1 = vs - (float)hv;  // exact (or vs itself when hv was flushed)
    const _Float16 lv = to_f16(r1 * 4096.0f);
    const int64_t o = row * 2 * dim + (i >> 5) * 64 + (i & 31);
    c16[o] = hv;
    c16[o + 32] = lv;
    const double e1 = (double)v - ldexp((double)(float)hv, -sx);  // exact residuals of what the MFMA sees
    const double e2 = e1 - ldexp((double)(float)lv, -sx - 12);
    s += (double)v * (double)v;
    s1 += e1 * e1;
    s2 += e2 * e2;
  }
  s = wave_sum(s);
  s1 = wave_sum(s1);
  s2 = wave_sum(s2);
  if (lane == 0) {  // norms rounded up slightly: they only feed the screening bound
    const float y = (float)sqrt(s) * 1.0000002f, z = (float)sqrt(s2) * 1.0000002f, w = (float)sqrt(s1) * 1.0000002f;
    meta[row] = make_float4((float)s, y, z, w);
    // table-wide collapse constants of the single-pass epilogue (assign_common.h): positive floats
    // order like their bit patterns
    unsigned* tab = reinterpret_cast<unsigned*>(meta + k);
    atomicMax(tab + 1, __float_as_uint(ratio_up(z, y)));
    atomicMax(tab + 2, __float_as_uint(ratio_up(w, y)));
    atomicMax(tab + 3, __float_as_uint(y));
  }
}

__global__ void centers_scale_kernel(float* __restrict__ scale) {
  *scale = ldexpf(1.0f, -table_scale_exp(__float_as_uint(*scale)));
}

// ---------------------------------------------------------------------------
// screening kernel
// ---------------------------------------------------------------------------
#ifndef RQSID_INTERLEAVE  // 1: the ring's DMA ops interleaved with the MFMAs of the compute phase
#define RQSID_INTERLEAVE 0
#endif

constexpr int kSplitDim = 512;  // widest row of the candidate-split form
// CW candidate groups (CW > 1: the candidate-split form, 4 CW waves, see assign_screen_kernel)
template <int NT, int S, bool T3, int CW = 1>
struct ScreenLayout {
  static constexpr int kCHalf = CW * NT * 32 * 64;         // CW*NT*32 candidates x 32 fp16 dims
  static constexpr int kCStage = kCHalf * (T3 ? 2 : 1);     // hi (+ lo) centre images
  static constexpr int kStage = kXStage + kCStage;
  static constexpr int kMeta = S * kStage;       // float4 {|c|^2, |c|, e0, 0} per candidate of the pass
  // CW > 1 (single pass only): meta is the SoA |c|^2, |c| plus the per-wave maxima, and rows are at
  // most kSplitDim wide, so a 3-stage ring of 48-KiB stages fits the 160 KiB of LDS
  static constexpr int kRes = kMeta + (CW > 1 ? 2 * CW * NT * 32 * 4 + 256 : NT * 32 * 16);  // residual rows ca, cb
  // CW > 1: the candidate groups' row exchange (least upper bounds, pass counts, merged lists)
  static constexpr int kXch = kRes + 2 * (CW > 1 ? kSplitDim : kMaxDim) * 4;
  static constexpr int kXchBytes = CW > 1 ? 2 * CW * kTileRows * 4 + kTileRows * kMaxList * 2 : 0;
  static constexpr int bytes(int rl, int dim) { return CW > 1 ? kXch + kXchBytes : kRes + rl * dim * 4; }
  static constexpr int kMaxBytes = kXch + kXchBytes;
  static_assert(kMaxBytes <= 160 * 1024, "LDS budget");
};

// Row decision of the candidate-split form (CW groups of NT*32 candidates, one wave of each group per
// 32 rows): pass_decide over every group's pass bits, exchanged through LDS.  Group g's candidates are
// local positions g*NT*32 .. (g+1)*NT*32 - 1, so the groups' ascending lists concatenate in order.
// k_out >= 0 only in the wave that holds a definitive row's single candidate; w (cand, n) is complete in
// group 0's waves.  Contains two block barriers: every wave of the block calls it.
template <int NW, int CW>
__device__ __forceinline__ bool pass_decide_cw(const uint32_t (&pbits)[NW], int h, int cg, int rowt, int cgbase,
                                               int& k_out, WorkItem& w, unsigned char* xch) {
  int* xn = reinterpret_cast<int*>(xch + CW * kTileRows * 4);                    // [CW][128] counts, -1 overflow
  uint16_t* xl = reinterpret_cast<uint16_t*>(xch + 2 * CW * kTileRows * 4);      // [128][kMaxList]
  int pc = 0;
#pragma unroll
  for (int i = 0; i < NW; ++i) pc += __popc(pbits[i]);
  const int pc_o = __shfl_xor(pc, 32);
  const int nw = pc + pc_o;
  const bool ovf_w = pc > kListPerHalf || pc_o > kListPerHalf;
  uint32_t wv[NW];
#pragma unroll
  for (int i = 0; i < NW; ++i) wv[i] = pbits[i];
  const int k0 = pass_take_first(wv, h);
  const int kw = max(k0, __shfl_xor(k0, 32));  // the group's candidate when nw == 1
  if (h == 0) xn[cg * kTileRows + rowt] = ovf_w ? -1 : nw;
  __syncthreads();
  int total = 0, before = 0;
  bool ovf = false;
#pragma unroll
  for (int g = 0; g < CW; ++g) {
    const int n = xn[g * kTileRows + rowt];
    ovf = ovf || n < 0;
    total += max(n, 0);
    before += g < cg ? max(n, 0) : 0;
  }
  ovf = ovf || total > kMaxList || total == 0;
  const bool definitive = !ovf && total == 1;
  k_out = definitive && nw == 1 ? cgbase + kw : -1;
  w.n = ovf ? -1 : total;
  const bool need_list = !ovf && total > 1;
  if (__builtin_amdgcn_ballot_w64(need_list && nw > 0)) {  // wave-uniform: some row lists candidates here
    int kk[kListPerHalf];
    kk[0] = k0;
#pragma unroll
    for (int j = 1; j < kListPerHalf; ++j) kk[j] = pass_take_first(wv, h);
    int c8[kMaxList];
#pragma unroll
    for (int j = 0; j < kListPerHalf; ++j) {
      const int o = __shfl_xor(kk[j], 32);
      c8[j] = kk[j] >= 0 ? kk[j] : INT_MAX;
      c8[kListPerHalf + j] = o >= 0 ? o : INT_MAX;
    }
#pragma unroll
    for (int i = 0; i < kMaxList; ++i)
#pragma unroll
      for (int j = 0; j < kMaxList - 1 - i; ++j) {
        const int a = c8[j], bq = c8[j + 1];
        c8[j] = min(a, bq);
        c8[j + 1] = max(a, bq);
      }
    if (h == 0 && need_list) {
#pragma unroll
      for (int j = 0; j < kMaxList; ++j)
        if (j < nw) xl[rowt * kMaxList + before + j] = (uint16_t)(cgbase + c8[j]);
    }
  }
  __syncthreads();
  if (cg == 0 && __builtin_amdgcn_ballot_w64(need_list)) {
#pragma unroll
    for (int j = 0; j < kMaxList; ++j) w.cand[j] = j < total ? xl[rowt * kMaxList + j] : (uint16_t)0xFFFF;
  }
  return definitive;
}

// Screening error model (DESIGN.md "Screening bound").  With v the row's vector, vh = fp16(v),
// ex = v - vh, ch = fp16(c), ec = c - ch:
//   |v.c - vh.ch| <= |ex||c| + |vh||ec|                       (Cauchy-Schwarz, exact norms)
//   MFMA accumulation <= acc_rel * |vh||ch|  (model pinned by tests/test_mfma_numerics.py and
//      tools/mfma_model.py: one v_mfma_f32_32x32x16_f16 sums its 16 exact products aligned to the
//      largest one, dropping less than kTrunc * 2^-23 * max|p| (worst seen 2.1 on adversarial
//      mantissas), then adds C rounding to nearest (<= 2^-24 |D|); over N = dim/16 chained
//      instructions: (kTrunc + N/2) 2^-23 sum|p|, sum|p| <= |vh||ch|.  Valid only without
//      subnormal operands: see to_f16.)
// so d^2 = |c|^2 - 2 v.c/den is known to within e_k = A |c_k| + B |ec_k| + 2^-22 |c_k|^2 with the per-row
//   A = 2/den (|ex| + acc_rel |vh|) + 2 dr + 2^-21 |r|,   B = 2/den |vh| (1 + acc_rel)
// (|ch_k| <= |c_k| + |ec_k|; dr = the rounding of the reference's r = v/den).  The centre term is per
// candidate: a near-zero centroid (large RELATIVE fp16 error, tiny absolute error) loosens only its own
// bound.
// Three-term screen (T3): v = vh + vl 2^-12 + ev and c 2^s = ch + cl 2^-12 + ec; the MFMAs sum
// vh.ch (acc) and vl.ch + vh.cl (accl, its own accumulator) and the omitted vl.cl, (vh + vl).ec and
// ev.c terms plus both accumulations are charged per candidate against |c|, |ec2| = |c - (ch + cl
// 2^-12) 2^-s| and |ec1| = |c - ch 2^-s| (see the epilogue's A, B, C).
// Single-pass epilogue (ONE: every segment has <= NT*32 candidates).  The per-candidate centre terms
// collapse onto |c_k| with tile constants: |ec_k| <= gz |c_k|, |ec1_k| <= gw |c_k| (gz, gw = the largest
// ratios over the tile's candidates, rounded up) and e0_k <= 2^-22 |c_k| ymax + 1e-30, so
//   e_k <= A2 |c_k| + 1e-30,   A2 = A + B gz + C gw + 2.39e-7 ymax
// and every candidate costs two packed FMAs for P = |c|^2 - 2 v.c/den and E, two packed adds for
// ub = P + E / lb = P - E (lb overwrites the accumulator) and half a min3 (sweep 1), then a compare
// and two selects (sweep 2: how many candidates have lb <= U, the last two of them).
#ifdef RQSID_STAMPS
__device__ unsigned long long g_stamps_tile[8];
#endif

// Candidate-split form (CW > 1, single-pass segments only): 4 CW waves per block; wave w screens the
// tile's rows 32 (w % 4) .. +31 against candidate group w / 4 (NT*32 candidates), so a segment of up to
// CW*NT*32 candidates (the XL preset's 512 at the last level, 256 3-term at the middle one) is screened
// in ONE pass: the tile's rows stream from HBM once instead of once per 256 / 128-candidate pass.  The
// waves of a row group share the row image (each issues 4/CW of its DMAs) and exchange their least
// upper bounds and pass lists through LDS (pass_decide_cw).
template <int NT, int S, int RL, bool NORM, bool T3, bool ONE, int CW = 1>
__global__ __launch_bounds__(256 * CW, CW > 1 ? 2 : (T3 ? 2 : (S == 2 ? (NT == 4 ? 3 : 2) : ((NT == 4 && S <= 3) ? 2 : 1)))) void assign_screen_kernel(AssignParams p) {
  static_assert(CW == 1 || (ONE && (CW == 2 || CW == 4)), "candidate-split form: single-pass segments");
  using L = ScreenLayout<NT, S, T3, CW>;
  constexpr int kXOps = 4 / CW;  // x-row DMA ops per wave per chunk (a row group's 4 split over its CW waves)
  constexpr int P = kXOps + (NT / 2) * (T3 ? 2 : 1);  // DMA ops per wave per chunk (centres: NT/2 per table)
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  // FP16 (and FP64) denormals flushed: a row value below the fp16 normal range converts to 0 (its
  // value lands in the measured |v - vh|), so no subnormal operand reaches the MFMA (to_f16)
#ifndef RQSID_AB_NO_FLUSH
  asm volatile("s_setreg_imm32_b32 hwreg(HW_REG_MODE, 6, 2), 0");
#endif
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int rg = CW > 1 ? (wave & 3) : wave;   // row group: rows 32 rg .. 32 rg + 31 of the tile
  const int cg = CW > 1 ? (wave >> 2) : 0;     // candidate group: local candidates cg NT 32 ..
  const int h = lane >> 5, r = lane & 31;
  ST(const uint64_t st_begin = ST_NOW(); uint64_t st_wait = 0; uint64_t st_e0 = 0; uint64_t st_issue = 0; uint64_t st_ring = 0;)
  // XCD-aware tile order: blocks b and b+8 share an XCD (and its L2), so give each group of 8 a
  // contiguous run of tiles -> a segment's candidate centres stay hot in one L2 (gridDim.x % 8 == 0)
  const int G = gridDim.x;
  const int b = (blockIdx.x & 7) * (G >> 3) + (blockIdx.x >> 3);
  const int nseg = p.n_segments;
  if (b >= p.seg_tile_off[nseg]) return;
  int s;
  if (p.tile_seg) {  // one load instead of log2(S) dependent ones (14 at the last level)
    s = p.tile_seg[b];
  } else {
    int lo = 0, hi = nseg;
    while (hi - lo > 1) {
      const int mid = (lo + hi) >> 1;
      if (p.seg_tile_off[mid] <= b) lo = mid; else hi = mid;
    }
    s = lo;
  }
  const int t0 = p.seg_row_off[s] + (b - p.seg_tile_off[s]) * kTileRows;
  const int nrows = min(kTileRows, p.seg_row_off[s + 1] - t0);
  const int cnt = p.cand_count[s];
  const int cbase = p.cand_base[s];
  const bool penalty = p.seg_flags && (p.seg_flags[s] & RQSID_SEG_PENALTY);
  const int dim = p.dim;

  const int my_local = rg * kRowsPerWave + r;
  const bool row_valid = my_local < nrows;
  const int pos = t0 + (row_valid ? my_local : 0);
  const int my_row = p.row_index ? p.row_index[pos] : pos;

  if (penalty || cnt <= 0) {  // block-uniform: no barrier below is skipped by part of the block
    WorkItem w{};
    w.row = my_row;
    w.seg = s;
    w.n = penalty ? -2 : -3;
    push_work(p, cg == 0 && h == 0 && row_valid, lane, w);
    return;
  }

  // DMA sources for this wave's x rows: instruction i covers rows 8i + lane/8, 16-B slot lane%8 of the
  // LDS image holding global slot (lane%8) ^ swz(row)  (swz(row) = (row>>1)&7: conflict-free reads);
  // CW > 1: the row group's instructions cg*kXOps .. +kXOps-1
  const float* xsrc[kXOps];
#pragma unroll
  for (int i = 0; i < kXOps; ++i) {
    const int rr = 8 * (cg * kXOps + i) + (lane >> 3);
    const int grow = __shfl(my_row, rr);
    const int slot = (lane & 7) ^ ((rr >> 1) & 7);
    xsrc[i] = p.x + (int64_t)grow * dim + slot * 4;
  }
  // residual rows of this segment -> LDS (staged below, after the ring's first DMAs are in flight)
  float* lds_ca = reinterpret_cast<float*>(smem + L::kRes);
  float* lds_cb = lds_ca + dim;
  float inv1 = 1.0f;
  auto stage_residual_rows = [&]() {
    if (RL >= 1) {
      const float4* a = reinterpret_cast<const float4*>(p.ca + (int64_t)seg_row(p.seg_ca, s) * dim);
      for (int i = tid; i < dim / 4; i += 256 * CW) reinterpret_cast<float4*>(lds_ca)[i] = a[i];
    }
    if (RL >= 2) {
      const float4* a = reinterpret_cast<const float4*>(p.cb + (int64_t)seg_row(p.seg_cb, s) * dim);
      for (int i = tid; i < dim / 4; i += 256 * CW) reinterpret_cast<float4*>(lds_cb)[i] = a[i];
    }
    if (RL >= 2 && NORM) inv1 = 1.0f / p.den_in[my_row];
    asm volatile("" : "+v"(inv1));  // its load completes before the ring's compute starts
  };
  if (!ONE) stage_residual_rows();

  const uint32_t lds0 = lds_addr(smem);
  const int nch = dim / kChunk;
  float U = INFINITY;
  int nlist = 0;
  int lk[kListPerHalf];
  float llb[kListPerHalf];
#pragma unroll
  for (int j = 0; j < kListPerHalf; ++j) {
    lk[j] = -1;
    llb[j] = INFINITY;
  }
  RowSums rs;  // the bound's running sums (row_frag)
  float vn = 0.f, en = 0.f, en2 = 0.f, inv_den = 1.f, dr = 0.f;
  float4* lds_meta = reinterpret_cast<float4*>(smem + L::kMeta);
  const f32x16 zero16 = {};
  const int xsw = (r >> 1) & 7;  // swizzle of this lane's row in the x image
  const int csw = (r >> 2) & 3;  // swizzle of this lane's candidate row in the centre image

  const int npass = ONE ? 1 : (cnt + NT * 32 - 1) / (NT * 32);
  float* m_csq = reinterpret_cast<float*>(smem + L::kMeta);  // ONE: SoA meta |c|^2, |c|, per-wave maxima
  float* m_y = m_csq + CW * NT * 32;
  float* m_red = m_y + CW * NT * 32;
  uint32_t pbits[ONE ? NT / 2 : 1];  // ONE: pass bits, word w = tiles 2w, 2w+1, MSB first
  for (int pass = 0; pass < npass; ++pass) {
    const int pbase = pass * NT * 32;
    // centre DMA sources (c16 row = 2 dim halves, chunk c at 64 c).  1 term: instruction j covers the
    // hi halves of candidates (wave*NT/2 + j)*16 + lane/4 (64 B each, slot lane%4 of the image row
    // k*64 + (slot ^ ((k>>2)&3))*16); T3: instruction j covers the hi+lo pieces of candidates
    // (wave*NT + j)*8 + lane/8 (128 B each, image row k*128 + (slot ^ ((k>>1)&7))*16: hi slots 0-3, lo 4-7)
    constexpr int kCOps = T3 ? NT : NT / 2;
    const _Float16* csrc[kCOps];
#pragma unroll
    for (int j = 0; j < kCOps; ++j) {
      const int il = T3 ? (wave * NT + j) * 8 + (lane >> 3) : (wave * (NT / 2) + j) * 16 + (lane >> 2);
      const int kl = pbase + il < cnt ? pbase + il : cnt - 1;
      const int cg = cand_global(p, cbase, kl);
      const int slot = T3 ? (lane & 7) ^ ((il >> 1) & 7) : (lane & 3) ^ ((il >> 2) & 3);
      csrc[j] = reinterpret_cast<const _Float16*>(p.c16) + (int64_t)cg * 2 * dim + slot * 8;
    }
    constexpr int kCStride = 2 * kChunk;
    // DMA op i of chunk c (x rows 0..3, hi centres, lo centres) into stage c % S
    auto issue_op = [&](int c, int i, bool relaxed) {
      const uint32_t sb = lds0 + (uint32_t)((c % S) * L::kStage);
      if (i < kXOps) {
        const void* src = xsrc[i] + c * kChunk;
        const uint32_t dst = __builtin_amdgcn_readfirstlane(sb + rg * kXWaveBytes + (cg * kXOps + i) * 1024);
        if (relaxed) dma16_nt_r(src, dst); else dma16_nt(src, dst);
      } else {
        const int j = i - kXOps;
        const void* src = csrc[j] + c * kCStride;
        const uint32_t dst = __builtin_amdgcn_readfirstlane(sb + kXStage + (wave * kCOps + j) * 1024);
        if (relaxed) dma16_r(src, dst); else dma16(src, dst);
      }
    };
    auto issue = [&](int c) {
#pragma unroll
      for (int i = 0; i < P; ++i) issue_op(c, i, false);
    };
    if constexpr (ONE) {
      // single pass: the ring's first chunks go out before the tile's remaining header work (residual
      // rows, candidate meta), whose loads then overlap their flight; the barrier below drains both
#pragma unroll
      for (int c = 0; c < S - 1; ++c)
        if (c < nch) issue(c);
      stage_residual_rows();
    } else {
      __syncthreads();
    }
    if constexpr (ONE) {
      float gz = 0.f, gw = 0.f, gy = 0.f;
      if (tid < CW * NT * 32) {
        const bool live = pbase + tid < cnt;
        const int kl = live ? pbase + tid : cnt - 1;
        const float4 m = reinterpret_cast<const float4*>(p.c_meta)[cand_global(p, cbase, kl)];
        m_csq[tid] = live ? m.x : INFINITY;
        m_y[tid] = m.y;
        gz = ratio_up(T3 ? m.z : m.w, m.y);
        gw = T3 ? ratio_up(m.w, m.y) : 0.f;
        gy = m.y;
      }
      gz = wave_max(gz);
      gw = wave_max(gw);
      gy = wave_max(gy);
      if (lane == 0) {
        m_red[wave * 4 + 0] = gz;
        m_red[wave * 4 + 1] = gw;
        m_red[wave * 4 + 2] = gy;
      }
    } else if (tid < NT * 32) {
      const bool live = pbase + tid < cnt;
      const int kl = live ? pbase + tid : cnt - 1;
      const float4 m = reinterpret_cast<const float4*>(p.c_meta)[cand_global(p, cbase, kl)];
      // {|c|^2 (inf for padding candidates), |c|, |ec2| (T3) or |ec1|, |ec1|}
      lds_meta[tid] = make_float4(live ? m.x : INFINITY, m.y, T3 ? m.z : m.w, m.w);
    }
#pragma unroll
    for (int j = 0; j < kCOps; ++j) {
      asm volatile("" : "+v"(csrc[j]));
    }
    __syncthreads();

    f32x16 acc[NT];
    f32x16 accl[T3 ? NT : 1];  // T3: vl.ch + vh.cl in units of 2^-12
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[t] = zero16;
#pragma unroll
    for (int t = 0; t < (T3 ? NT : 1); ++t) accl[t] = zero16;

    // compute chunk c; the P DMA ops of chunk cn (< 0: none) are spread between its 2*NT MFMA groups,
    // so a DMA issue stall (the load path's back-pressure) overlaps MFMAs in flight instead of
    // preceding the whole phase
    auto compute = [&](int c, int cn) {
#if RQSID_AB_MODE >= 3
      if (cn >= 0) issue(cn);
      return;
#endif
      constexpr int NG = 2 * NT;
      const unsigned char* xb = smem + (c % S) * L::kStage + rg * kXWaveBytes + r * 128;
      // centre image row of candidate t*32 + r: 64 B (1 term) or 128 B (T3: hi slots 0-3, lo 4-7)
      const unsigned char* cbp = smem + (c % S) * L::kStage + kXStage + (cg * NT * 32 + r) * (T3 ? 128 : 64);
      const int tsw = (r >> 1) & 7;  // T3 image swizzle (the x image's)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const int q0 = 4 * ks + 2 * h;
        const float4 xa = *reinterpret_cast<const float4*>(xb + ((q0 ^ xsw) << 4));
        const float4 xc = *reinterpret_cast<const float4*>(xb + (((q0 + 1) ^ xsw) << 4));
        const int d0 = c * kChunk + 16 * ks + 8 * h;
        f16x8 bf, bl = {};
        if (pass == 0) row_frag<RL, NORM, T3, true>(xa, xc, lds_ca, lds_cb, d0, inv1, bf, bl, rs);
        else row_frag<RL, NORM, T3, false>(xa, xc, lds_ca, lds_cb, d0, inv1, bf, bl, rs);
        const int qa = T3 ? (2 * ks + h) ^ tsw : (2 * ks + h) ^ csw;
        const int ql = (4 + 2 * ks + h) ^ tsw;
#pragma unroll
        for (int t = 0; t < NT; ++t) {
          const f16x8 af = *reinterpret_cast<const f16x8*>(cbp + t * 32 * (T3 ? 128 : 64) + (qa << 4));
#if RQSID_AB_MODE >= 2
          acc[t][0] += (float)bf[0] + (float)af[0];
          if (false) {
#else
          acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(af, bf, acc[t], 0, 0, 0);
          if (T3) {
#endif
            const f16x8 al = *reinterpret_cast<const f16x8*>(cbp + t * 32 * 128 + (ql << 4));
            accl[t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(af, bl, accl[t], 0, 0, 0);
            accl[t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, bf, accl[t], 0, 0, 0);
          }
#if RQSID_INTERLEAVE
          const int g = ks * NT + t;
#pragma unroll
          for (int i = g * P / NG; i < (g + 1) * P / NG; ++i) {
            RQSID_PIN_MFMA();
            if (cn >= 0) issue_op(cn, i, true);
            RQSID_PIN_MFMA();
          }
#endif
        }
      }
    };

    ST(st_ring = ST_NOW();)
    // S-stage ring: chunks 0..S-2 in flight before the first compute (single pass: issued above)
    if (!ONE) {
#pragma unroll
      for (int c = 0; c < S - 1; ++c)
        if (c < nch) issue(c);
    }
    for (int c = 0; c < nch; ++c) {
      ST(const uint64_t st_w0 = ST_NOW();)
      wait_chunks<S, P>(min(S - 2, nch - 1 - c));  // chunk c landed (every wave), chunk c-1 fully read
      ST(st_wait += ST_NOW() - st_w0;)
      const int cn = c + S - 1 < nch ? c + S - 1 : -1;  // into the stage chunk c-1 used
#if !RQSID_INTERLEAVE
      ST(const uint64_t st_i0 = ST_NOW();)
      if (cn >= 0) issue(cn);
      ST(st_issue += ST_NOW() - st_i0;)
      compute(c, -1);
#else
      compute(c, cn);
#endif
    }

    ST(st_e0 = ST_NOW();)
    if (pass == 0) {
      const float se2 = rs.se2v.x + rs.se2v.y, sf2 = rs.sf2v.x + rs.sf2v.y;
      const float e2 = se2 + __shfl_xor(se2, 32);
      en = sqrtf(e2) * 1.001f + 1e-30f;
      if (T3) {
        const float l2 = rs.se2l.x + rs.se2l.y;
        en2 = sqrtf(l2 + __shfl_xor(l2, 32)) * (1.001f / 4096.0f) + 1e-30f;
      }
      float nrm;
      if (NORM && RL >= 1) {
        if (RL == 1) {  // exact: written to den_out
          const double t2 = rs.sv2 + rs.sv2b;
          nrm = (float)sqrt(t2 + __shfl_xor(t2, 32));
        } else {  // fp32 sums: |nrm - |v|| <= den_eps |v| (chains of dim/4 + 2 terms, sqrt's half ulp)
          nrm = sqrtf(sf2 + __shfl_xor(sf2, 32));
        }
        const float den = nrm + 1e-8f;
        inv_den = 1.0f / den;
        if (RL == 1 && cg == 0 && h == 0 && row_valid && p.den_out) p.den_out[my_row] = den;
        // |r_ref - v/den| per element: RL1: the reference rounds r_i = u_i/den once;
        // RL2: v was built with a reciprocal multiply (2 ulp of |r1| = 1) and rounded
        // RL2 also: the fp32 denominator's error, |v/den' - v/den| <= den_eps |v| / den'
        const float den_eps = (0.125f * (float)(p.dim) + 3.0f) * 5.97e-8f;
        dr = RL == 1 ? 2.0f * 5.97e-8f
                     : (4.0f * 2.39e-7f * (1.0f + nrm) * inv_den + 4.0f * 5.97e-8f + 1.01f * den_eps * nrm * inv_den);
      } else {
        nrm = sqrtf(sf2 + __shfl_xor(sf2, 32));
      }
      vn = nrm * 1.0001f + 1e-30f;
    }
#if RQSID_AB_MODE >= 1
    {  // A/B timing build: no epilogue (results are wrong; tools/ab_sweep only)
      float sink = 0.f;
#pragma unroll
      for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int v = 0; v < 16; ++v) sink += acc[t][v] + (T3 ? accl[t < (T3 ? NT : 1) ? t : 0][v] : 0.f);
      if (sink == -1.2345e38f) p.out_local[my_row] = 7;
      __syncthreads();
      continue;
    }
#endif
    // epilogue.  Sweep 1: the least upper bound U over the row's candidates so far.  Sweep 2: list
    // (ascending) the candidates whose lower bound is <= U, up to kListPerHalf per lane half; U only
    // shrinks over passes, so earlier listings are re-filtered at the end.
    const float hn = vn + en;       // >= |vh|
    const float vr = vn * inv_den;  // |r| of the row being assigned
    // ar: the main accumulator (dim/16 instructions); ar2 = 2 ar: the T3 second one (twice as many)
    const float ar = p.acc_rel, ar2 = 2.0f * p.acc_rel, k2 = 2.0f * inv_den * 1.000001f;
    // e_k = A |c_k| + B m.z + C |ec1_k| + e0(|c_k|^2): 1-term m.z = |ec1| and C = 0; T3 m.z = |ec2|
    const float A = T3 ? k2 * (en2 + ar * hn + ar2 * (en + en2)) + 2.0f * dr + 7.2e-7f * vr
                       : k2 * (en + ar * hn) + 2.0f * dr + 4.8e-7f * vr;
    const float B = T3 ? k2 * (hn * (1.0f + ar2) + 2.0f * (en + en2)) : k2 * hn * (1.0f + ar);
    const float C = T3 ? k2 * ((en + en2) + ar * hn + ar2 * (hn + en + en2)) : 0.0f;
    // the MFMA sums are in units of 2^s of the centre table (rqsid_prepare_centers; exact power of two)
    const float m2 = -2.0f * inv_den *
                     __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(p.c_meta[4 * p.n_centers])));
    if constexpr (ONE) {
      float gz = 0.f, gw = 0.f, gy = 0.f;
#pragma unroll
      for (int w = 0; w < kWaves * CW; ++w) {
        gz = fmaxf(gz, m_red[w * 4 + 0]);
        gw = fmaxf(gw, m_red[w * 4 + 1]);
        gy = fmaxf(gy, m_red[w * 4 + 2]);
      }
      const float A2 = (A + B * gz + C * gw + 2.39e-7f * gy) * 1.000001f;
      const f2 m2v = {m2, m2}, a2v = {A2, A2}, epsv = {1e-30f, 1e-30f};
      // sweep 1: ub / lb per candidate (lb kept in the accumulator), U = least ub
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const float4 cs = *reinterpret_cast<const float4*>(m_csq + (cg * NT + t) * 32 + 8 * g + 4 * h);
          const float4 yy = *reinterpret_cast<const float4*>(m_y + (cg * NT + t) * 32 + 8 * g + 4 * h);
#pragma unroll
          for (int e = 0; e < 2; ++e) {
            const int v = 4 * g + 2 * e;
            f2 d = {acc[t][v], acc[t][v + 1]};
            if (T3) d = f2{accl[T3 ? t : 0][v], accl[T3 ? t : 0][v + 1]} * 0x1p-12f + d;
            const f2 P = m2v * d + (e ? f2{cs.z, cs.w} : f2{cs.x, cs.y});
            const f2 E = a2v * (e ? f2{yy.z, yy.w} : f2{yy.x, yy.y}) + epsv;
            const f2 ub = P + E, lb = P - E;
            U = fminf(U, fminf(ub.x, ub.y));
            acc[t][v] = lb.x;
            acc[t][v + 1] = lb.y;
          }
        }
      }
      U = fminf(U, __shfl_xor(U, 32));
      if constexpr (CW > 1) {  // the row's least upper bound over every candidate group
        // lb materialised here: otherwise hipcc sinks lb = P - E past the barrier, keeping P and E
        // both live (256 VGPRs -> spills)
#pragma unroll
        for (int t = 0; t < NT; ++t) asm volatile("" : "+v"(acc[t]));
        float* xu = reinterpret_cast<float*>(smem + L::kXch);
        if (h == 0) xu[cg * kTileRows + my_local] = U;
        __syncthreads();
#pragma unroll
        for (int g = 0; g < CW; ++g) U = fminf(U, xu[g * kTileRows + my_local]);
      }
      // sweep 2: one bit per candidate, lb <= U, i.e. the sign of lb - Up with Up > U by >= 2 ulp (a
      // candidate admitted by rounding is only re-scored); v_alignbit shifts the sign into the word.
      // v = 0..15 is ascending in candidate order, so word w holds tile 2w's candidates from bit 31
      // down, then tile 2w+1's.
      const float Up = fmaf(fabsf(U), 0x1p-22f, U) + 1.2e-38f;
      const f2 upv = {Up, Up};
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        __builtin_amdgcn_sched_barrier(0);
        uint32_t b = (t & 1) ? pbits[t >> 1] : 0u;
#pragma unroll
        for (int v = 0; v < 16; v += 2) {
          const f2 d = f2{acc[t][v], acc[t][v + 1]} - upv;
          b = __builtin_amdgcn_alignbit(b, __float_as_uint(d.x), 31);
          b = __builtin_amdgcn_alignbit(b, __float_as_uint(d.y), 31);
        }
        pbits[t >> 1] = b;
      }
      continue;  // npass == 1
    }
    const float4* meta = lds_meta + 4 * h;
    const int kl_h = pbase + 4 * h;
    // sweep 1: U = least upper bound.  The scheduling barriers stop hipcc from hoisting every
    // tile's meta reads at once (256 VGPRs -> spills at 2 waves/SIMD).
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int v = 0; v < 16; ++v) {
        const int io = t * 32 + (v & 3) + 8 * (v >> 2);
        const float4 m = meta[io];
        const float dot = T3 ? fmaf(0x1p-12f, accl[t][v], acc[t][v]) : acc[t][v];
        const float sc = fmaf(m2, dot, m.x);
        const float e0 = fmaf(2.39e-7f, m.x, 1e-30f);  // the fp32 epilogue's own rounding
        U = fminf(U, sc + fmaf(A, m.y, fmaf(B, m.z, T3 ? fmaf(C, m.w, e0) : e0)));
      }
    }
    U = fminf(U, __shfl_xor(U, 32));
    // sweep 2: list the candidates whose lower bound (recomputed) is <= U, ascending
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int v = 0; v < 16; ++v) {
        const int kl = kl_h + t * 32 + (v & 3) + 8 * (v >> 2);
        const float4 m = meta[t * 32 + (v & 3) + 8 * (v >> 2)];
        const float dot = T3 ? fmaf(0x1p-12f, accl[t][v], acc[t][v]) : acc[t][v];
        const float e0 = fmaf(2.39e-7f, m.x, 1e-30f);
        const float lb = fmaf(m2, dot, m.x) - fmaf(A, m.y, fmaf(B, m.z, T3 ? fmaf(C, m.w, e0) : e0));
        const bool q = lb <= U && kl < cnt;
        if (__builtin_amdgcn_ballot_w64(q)) {  // wave-uniform skip: most candidates qualify for no row
#pragma unroll
          for (int j = 0; j < kListPerHalf; ++j) {
            const bool take = q && nlist == j;
            lk[j] = take ? kl : lk[j];
            llb[j] = take ? lb : llb[j];
          }
          nlist += q ? 1 : 0;
        }
      }
    }
    __syncthreads();  // meta / ring are rewritten by the next pass
  }

#if RQSID_AB_MODE >= 1
  if (h == 0 && row_valid) {  // hashed ids keep the next level's segment mix realistic
    const int k = (int)(((uint32_t)my_row * 2654435761u) >> 8) % cnt;
    p.out_local[my_row] = cand_local(p, cbase, k);
    p.out_global[my_row] = cand_global(p, cbase, k);
  }
  return;
#endif
  if constexpr (ONE) {
    WorkItem w{};
    w.row = my_row;
    w.seg = s;
    int k = -1;
    bool definitive;
    if constexpr (CW > 1) definitive = pass_decide_cw<NT / 2, CW>(pbits, h, cg, my_local, cg * NT * 32, k, w, smem + L::kXch);
    else definitive = pass_decide(pbits, h, k, w);
    if (h == 0 && row_valid && definitive && k >= 0) {
      p.out_local[my_row] = cand_local(p, cbase, k);
      p.out_global[my_row] = cand_global(p, cbase, k);
    }
    push_work(p, cg == 0 && h == 0 && row_valid && !definitive, lane, w);
#ifdef RQSID_STAMPS
    if (tid == 0) {
      const uint64_t now = ST_NOW();
      atomicAdd(&g_stamps_tile[0], (unsigned long long)(now - st_begin));
      atomicAdd(&g_stamps_tile[1], (unsigned long long)st_wait);
      atomicAdd(&g_stamps_tile[2], (unsigned long long)(now - st_e0));
      atomicAdd(&g_stamps_tile[3], (unsigned long long)st_issue);
      atomicAdd(&g_stamps_tile[4], (unsigned long long)(st_ring - st_begin));
    }
#endif
    return;
  }
  // Row decision: keep the listed candidates still within the final U; a half that listed more
  // than kListPerHalf overflows -> re-score every candidate of the segment.
  bool ovf = nlist > kListPerHalf || cnt > 65535;
  int nh = 0;
  int kk[kListPerHalf];
#pragma unroll
  for (int j = 0; j < kListPerHalf; ++j) {
    const bool keep = j < nlist && llb[j] <= U;
    kk[j] = keep ? lk[j] : -1;
    nh += keep ? 1 : 0;
  }
  const bool ovf_p = __shfl_xor((int)ovf, 32) != 0;
  const int nh_p = __shfl_xor(nh, 32);
  int kp[kListPerHalf];
#pragma unroll
  for (int j = 0; j < kListPerHalf; ++j) kp[j] = __shfl_xor(kk[j], 32);
  const int ncand = nh + nh_p;
  const bool overflow = ovf || ovf_p || ncand == 0;
  const bool definitive = !overflow && ncand == 1;
  if (h == 0 && row_valid && definitive) {
    int k = -1;
#pragma unroll
    for (int j = 0; j < kListPerHalf; ++j) k = max(k, max(kk[j], kp[j]));
    p.out_local[my_row] = cand_local(p, cbase, k);
    p.out_global[my_row] = cand_global(p, cbase, k);
  }
  WorkItem w{};
  w.row = my_row;
  w.seg = s;
  if (overflow) {
    w.n = -1;
  } else {
    // ascending candidate list (empty slots sort last); static indexing only
    int c8[kMaxList];
#pragma unroll
    for (int j = 0; j < kListPerHalf; ++j) {
      c8[j] = kk[j] >= 0 ? kk[j] : INT_MAX;
      c8[kListPerHalf + j] = kp[j] >= 0 ? kp[j] : INT_MAX;
    }
#pragma unroll
    for (int i = 0; i < kMaxList; ++i)
#pragma unroll
      for (int j = 0; j < kMaxList - 1 - i; ++j) {
        const int a = c8[j], bq = c8[j + 1];
        c8[j] = min(a, bq);
        c8[j + 1] = max(a, bq);
      }
#pragma unroll
    for (int j = 0; j < kMaxList; ++j) w.cand[j] = (uint16_t)(c8[j] == INT_MAX ? 0xFFFF : c8[j]);
    const int n = ncand;
    w.n = n;
  }
  push_work(p, h == 0 && row_valid && !definitive, lane, w);
}

// ---------------------------------------------------------------------------
// exact re-score
// ---------------------------------------------------------------------------
// One wave per listed row.  The row's vector is rebuilt with the reference's fp32 operation sequence
// (x - ca, / n1, - cb, / n2 with n = fl(sqrt(sum^2)) + 1e-8) and held in registers, lanes over dims;
// candidates are scored 8 at a time (coalesced 2 KB centre-row reads, fp64 sums of (v - c)^2, one
// batched cross-lane reduction), so explicit lists cost one batch and "every candidate" / penalty rows
// cost ceil(n/8) batches.  The winner is the lexicographic minimum (distance, local index).
constexpr int kRescoreMaxV = kMaxDim / 256;  // float4 per lane
constexpr int kBatch = 8;

template <int RL, bool NORM>
__global__ __launch_bounds__(256) void assign_rescore_kernel(AssignParams p) {
  const int lane = threadIdx.x & 63;
  const int wid = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int nw = gridDim.x * 4;
  const int64_t nitems_raw = *p.work_count;
  const int64_t nitems = nitems_raw < p.work_cap ? nitems_raw : p.work_cap;
  const int nv = p.dim / 4;
  // Items are strided over every wave of the grid: the "every candidate" rows cluster in a few
  // segments (duplicated centres), and striding spreads them evenly over the waves.
  for (int64_t it = wid; it < nitems; it += nw) {
    const WorkItem w = p.work[p.work_idx ? p.work_idx[it] : it];
    const float* xr = p.x + (int64_t)w.row * p.dim;
    const float* car = RL >= 1 ? p.ca + (int64_t)seg_row(p.seg_ca, w.seg) * p.dim : nullptr;
    const float* cbr = RL >= 2 ? p.cb + (int64_t)seg_row(p.seg_cb, w.seg) * p.dim : nullptr;
    const bool screened = w.n >= 1 || w.n == -1;  // the screen wrote den_out for these rows
    float4 v[kRescoreMaxV];
    double ss = 0.0;
#pragma unroll
    for (int m = 0; m < kRescoreMaxV; ++m) {
      const int i = lane + 64 * m;
      if (i < nv) {
        float4 a = reinterpret_cast<const float4*>(xr)[i];
        if (RL >= 1) {
          const float4 c = reinterpret_cast<const float4*>(car)[i];
          a = make_float4(a.x - c.x, a.y - c.y, a.z - c.z, a.w - c.w);
        }
        if (RL >= 2) {
          if (NORM) {
            const float d1 = p.den_in[w.row];
            a = make_float4(a.x / d1, a.y / d1, a.z / d1, a.w / d1);
          }
          const float4 c = reinterpret_cast<const float4*>(cbr)[i];
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
      if (RL == 1 && p.den_out && screened) den = p.den_out[w.row];
      else den = (float)sqrt(wave_sum(ss)) + 1e-8f;
      if (RL == 1 && p.den_out && !screened && lane == 0) p.den_out[w.row] = den;
#pragma unroll
      for (int m = 0; m < kRescoreMaxV; ++m)
        v[m] = make_float4(v[m].x / den, v[m].y / den, v[m].z / den, v[m].w / den);
    }
    const bool penalty = w.n == -2;
    const bool listed = w.n >= 1;
    const int base = p.cand_base[w.seg];
    const int n = listed ? w.n : (penalty ? p.n_centers : (w.n == -1 ? p.cand_count[w.seg] : 0));
    double best = INFINITY;  // penalty rows compare fl32(sqrt(fl32(d^2))) + 10000 in fp32, as the reference
    int bj = INT_MAX;
    for (int j0 = 0; j0 < n; j0 += kBatch) {
      double acc[kBatch];
      int loc[kBatch];
#pragma unroll
      for (int jj = 0; jj < kBatch; ++jj) {
        const int j = j0 + jj;
        acc[jj] = 0.0;
        loc[jj] = j < n ? (listed ? (int)w.cand[jj] : j) : INT_MAX;
        if (j < n) {
          const int g = penalty ? loc[jj] : cand_global(p, base, loc[jj]);
          const float4* cr = reinterpret_cast<const float4*>(p.centers + (int64_t)g * p.dim);
#pragma unroll
          for (int m = 0; m < kRescoreMaxV; ++m) {
            const int i = lane + 64 * m;
            if (i < nv) {
              const float4 c = cr[i];
              const double d0 = (double)v[m].x - c.x, d1 = (double)v[m].y - c.y, d2 = (double)v[m].z - c.z,
                           d3 = (double)v[m].w - c.w;
              acc[jj] += d0 * d0 + d1 * d1 + d2 * d2 + d3 * d3;
            }
          }
        }
      }
      // halving cross-lane reduction: 4 + 2 + 1 exchanges leave lane l holding the wave total of
      // candidate jj(l) = 4*(l>>5) + 2*((l>>4)&1) + ((l>>3)&1) summed over its 8-lane group; 3 more
      // exchanges finish it.  10 shuffles for 8 sums instead of 48.
      double r4[4], r2[2], r1;
      const bool b5 = lane & 32, b4 = lane & 16, b3 = lane & 8;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const double send = b5 ? acc[j] : acc[j + 4];
        const double keep = b5 ? acc[j + 4] : acc[j];
        r4[j] = keep + __shfl_xor(send, 32);
      }
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const double send = b4 ? r4[j] : r4[j + 2];
        const double keep = b4 ? r4[j + 2] : r4[j];
        r2[j] = keep + __shfl_xor(send, 16);
      }
      {
        const double send = b3 ? r2[0] : r2[1];
        const double keep = b3 ? r2[1] : r2[0];
        r1 = keep + __shfl_xor(send, 8);
      }
      r1 += __shfl_xor(r1, 4);
      r1 += __shfl_xor(r1, 2);
      r1 += __shfl_xor(r1, 1);
      const int my_jj = 4 * (lane >> 5) + 2 * ((lane >> 4) & 1) + ((lane >> 3) & 1);
      int my_loc = INT_MAX;
#pragma unroll
      for (int jj = 0; jj < kBatch; ++jj) my_loc = my_jj == jj ? loc[jj] : my_loc;
      double key = r1;
      if (penalty) key = (double)((float)sqrt((double)(float)key) + 10000.0f);
      // lexicographic (distance, index) minimum over the batch (lanes) and the running best; a NaN
      // distance never displaces a real one
#pragma unroll
      for (int o = 8; o < 64; o <<= 1) {
        const double ok = __shfl_xor(key, o);
        const int ol = __shfl_xor(my_loc, o);
        const bool kn = key != key, okn = ok != ok;
        const bool take = ol != INT_MAX && (my_loc == INT_MAX || (!okn && (kn || ok < key || (ok == key && ol < my_loc))));
        key = take ? ok : key;
        my_loc = take ? ol : my_loc;
      }
      {
        const bool kn = key != key, bn = best != best;
        const bool take = my_loc != INT_MAX &&
                          (bj == INT_MAX || (!kn && (bn || key < best || (key == best && my_loc < bj))));
        if (take) {
          best = key;
          bj = my_loc;
        }
      }
    }
    if (lane == 0) {
      const bool found = bj != INT_MAX;
      p.out_local[w.row] = found && !penalty ? cand_local(p, base, bj) : -1;
      p.out_global[w.row] = found ? (penalty ? bj : cand_global(p, base, bj)) : -1;
    }
  }
}

// Two listed rows per wave (rows of at most kHalfDim dims): lanes 32 hh .. 32 hh + 31 re-score item
// 2 wid + hh of the pass with 4 float4 of the row per lane; the same arithmetic, candidate batches and
// (distance, index) rule as assign_rescore_kernel, with every reduction kept inside the half.  The
// re-score is bound by its dependent-load chain (item -> row, residual rows -> candidate rows), not by
// bytes, and a wave now carries two chains at the same register count.
constexpr int kHalfDim = 512;
__device__ __forceinline__ double half_sum(double v) {
#pragma unroll
  for (int o = 16; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

// mode 0: every work item; after the fp32 re-screen the items it left "every candidate" (n = -1: a true
// cluster of > kMaxList candidates, e.g. near-equal distances of a zero residual row) go to their own pass
// instead: mode 1 takes the other items, mode 2 the n = -1 items in overflow-list order, where a block's 8
// consecutive items are rows of one segment walking the same candidates, so a candidate row is read from
// L2 once per block rather than once per row (the per-row arithmetic is the same code)
constexpr int kOvfSlot = 56;  // workspace header int: overflow item count
// workspace header int 60: sticky error word of the counter-driven list writes (NOT cleared by a call: the
// caller zeroes it when it allocates the workspace; ops.AssignWorkspace.error() / RQEncoder.errors() read it).  Each index such a write takes from a device counter is
// checked against its slot's capacity; a write that would fall outside is dropped and its bit raised, so
// a wrong count can only produce a reported error, never a store outside the workspace.
// (kErrSlot and its bits: assign_common.h)
template <int RL, bool NORM>
__global__ __launch_bounds__(256) void assign_rescore_half_kernel(AssignParams p, const int32_t* __restrict__ ovf_list,
                                                                  int mode) {
  constexpr int kV = kHalfDim / 128;  // float4 per lane
  const int lane = threadIdx.x & 63, hl = lane & 31, hh = lane >> 5;
  const int wid = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int nw = gridDim.x * 4;
  const int64_t nitems_raw = mode == 2 ? p.work_count[kOvfSlot] : *p.work_count;
  const int64_t nitems = nitems_raw < p.work_cap ? nitems_raw : p.work_cap;
  const int nv = p.dim / 4;
  for (int64_t it0 = 2 * (int64_t)wid; it0 < nitems; it0 += 2 * (int64_t)nw) {
    const int64_t it = it0 + hh < nitems ? it0 + hh : it0;
    const WorkItem w = p.work[mode == 2 ? ovf_list[it] : (p.work_idx ? p.work_idx[it] : it)];
    // an idle half (past the end, or an item of the other pass) repeats the work and writes nothing
    const bool active = it0 + hh < nitems && (mode == 0 || (mode == 1 ? w.n != -1 : w.n == -1));
    const float* xr = p.x + (int64_t)w.row * p.dim;
    const float* car = RL >= 1 ? p.ca + (int64_t)seg_row(p.seg_ca, w.seg) * p.dim : nullptr;
    const float* cbr = RL >= 2 ? p.cb + (int64_t)seg_row(p.seg_cb, w.seg) * p.dim : nullptr;
    const bool screened = w.n >= 1 || w.n == -1;  // the screen wrote den_out for these rows
    float4 v[kV];
    double ss = 0.0;
#pragma unroll
    for (int m = 0; m < kV; ++m) {
      const int i = hl + 32 * m;
      if (i < nv) {
        float4 a = reinterpret_cast<const float4*>(xr)[i];
        if (RL >= 1) {
          const float4 c = reinterpret_cast<const float4*>(car)[i];
          a = make_float4(a.x - c.x, a.y - c.y, a.z - c.z, a.w - c.w);
        }
        if (RL >= 2) {
          if (NORM) {
            const float d1 = p.den_in[w.row];
            a = make_float4(a.x / d1, a.y / d1, a.z / d1, a.w / d1);
          }
          const float4 c = reinterpret_cast<const float4*>(cbr)[i];
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
      if (RL == 1 && p.den_out && screened) den = p.den_out[w.row];
      else den = (float)sqrt(half_sum(ss)) + 1e-8f;
      if (RL == 1 && p.den_out && !screened && hl == 0 && active) p.den_out[w.row] = den;
#pragma unroll
      for (int m = 0; m < kV; ++m)
        v[m] = make_float4(v[m].x / den, v[m].y / den, v[m].z / den, v[m].w / den);
    }
    const bool penalty = w.n == -2;
    const bool listed = w.n >= 1;
    const int base = p.cand_base[w.seg];
    const int n = !active ? 0 : listed ? w.n : (penalty ? p.n_centers : (w.n == -1 ? p.cand_count[w.seg] : 0));
    const int nmax = max(n, __shfl_xor(n, 32));  // both halves run the same batches
    double best = INFINITY;
    int bj = INT_MAX;
    for (int j0 = 0; j0 < nmax; j0 += kBatch) {
      double acc[kBatch];
      int loc[kBatch];
#pragma unroll
      for (int jj = 0; jj < kBatch; ++jj) {
        const int j = j0 + jj;
        acc[jj] = 0.0;
        loc[jj] = j < n ? (listed ? (int)w.cand[jj] : j) : INT_MAX;
        if (j < n) {
          const int g = penalty ? loc[jj] : cand_global(p, base, loc[jj]);
          const float4* cr = reinterpret_cast<const float4*>(p.centers + (int64_t)g * p.dim);
#pragma unroll
          for (int m = 0; m < kV; ++m) {
            const int i = hl + 32 * m;
            if (i < nv) {
              const float4 c = cr[i];
              const double d0 = (double)v[m].x - c.x, d1 = (double)v[m].y - c.y, d2 = (double)v[m].z - c.z,
                           d3 = (double)v[m].w - c.w;
              acc[jj] += d0 * d0 + d1 * d1 + d2 * d2 + d3 * d3;
            }
          }
        }
      }
      // halving reduction inside the half: 4 + 2 + 1 exchanges leave lane hl holding candidate
      // jj(hl) = 4*((hl>>4)&1) + 2*((hl>>3)&1) + ((hl>>2)&1) summed over its 4-lane group; 2 more finish it
      double r4[4], r2[2], r1;
      const bool b4 = hl & 16, b3 = hl & 8, b2 = hl & 4;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const double send = b4 ? acc[j] : acc[j + 4];
        const double keep = b4 ? acc[j + 4] : acc[j];
        r4[j] = keep + __shfl_xor(send, 16);
      }
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const double send = b3 ? r4[j] : r4[j + 2];
        const double keep = b3 ? r4[j + 2] : r4[j];
        r2[j] = keep + __shfl_xor(send, 8);
      }
      {
        const double send = b2 ? r2[0] : r2[1];
        const double keep = b2 ? r2[1] : r2[0];
        r1 = keep + __shfl_xor(send, 4);
      }
      r1 += __shfl_xor(r1, 2);
      r1 += __shfl_xor(r1, 1);
      const int my_jj = 4 * ((hl >> 4) & 1) + 2 * ((hl >> 3) & 1) + ((hl >> 2) & 1);
      int my_loc = INT_MAX;
#pragma unroll
      for (int jj = 0; jj < kBatch; ++jj) my_loc = my_jj == jj ? loc[jj] : my_loc;
      double key = r1;
      if (penalty) key = (double)((float)sqrt((double)(float)key) + 10000.0f);
#pragma unroll
      for (int o = 4; o < 32; o <<= 1) {
        const double ok = __shfl_xor(key, o);
        const int ol = __shfl_xor(my_loc, o);
        const bool kn = key != key, okn = ok != ok;
        const bool take = ol != INT_MAX && (my_loc == INT_MAX || (!okn && (kn || ok < key || (ok == key && ol < my_loc))));
        key = take ? ok : key;
        my_loc = take ? ol : my_loc;
      }
      {
        const bool kn = key != key, bn = best != best;
        const bool take = my_loc != INT_MAX &&
                          (bj == INT_MAX || (!kn && (bn || key < best || (key == best && my_loc < bj))));
        if (take) {
          best = key;
          bj = my_loc;
        }
      }
    }
    if (hl == 0 && active) {
      const bool found = bj != INT_MAX;
      p.out_local[w.row] = found && !penalty ? cand_local(p, base, bj) : -1;
      p.out_global[w.row] = found ? (penalty ? bj : cand_global(p, base, bj)) : -1;
    }
  }
}

// ---------------------------------------------------------------------------
// fp32 re-screen of overflowing rows
// ---------------------------------------------------------------------------
// A row whose fp16 screen admits more than kMaxList candidates is marked "every candidate" (n = -1)
// and the fp64 re-score would score its whole segment: against the 2560 / 5120 candidates of a last
// level, or K = 1280 centres of a training-time nearest, on diffuse residual data that is most rows
// and 100s of ms per launch (VERDICT r3 "re-score cliff").  The re-screen gives those rows a list
// first: every candidate's squared distance in fp32 (sum of fl32((v_i - c_i)^2), all terms >= 0, so
// any summation order is within gamma_{dim+2} of the exact d^2), lower / upper bounds
// S (1 -/+ e) with e = (dim + 4) 2^-24 (1 + 2^-10) — ~60x tighter than the fp16 screen's — and the
// running least upper bound U; a candidate is kept while its lower bound is <= U (the list is
// compacted against the current U when it fills, so only a true cluster of > kMaxList candidates
// within the bound, e.g. duplicated centres, stays an overflow).  The exact fp64 re-score then scores
// the list; it contains every candidate the fp64 argmin can return, so IDs are unchanged.
// Block layout: 8 half-waves take 8 consecutive overflow items and walk the candidates together, so
// rows of one segment read each candidate row from L1 / L2 once per block, not once per row.
__global__ __launch_bounds__(256) void overflow_list_kernel(AssignParams p, int32_t* __restrict__ ovf_list) {
  const int64_t nitems_raw = *p.work_count;
  const int64_t nitems = nitems_raw < p.work_cap ? nitems_raw : p.work_cap;
  for (int64_t it = (int64_t)blockIdx.x * 256 + threadIdx.x; it < nitems; it += (int64_t)gridDim.x * 256) {
    const int32_t idx = p.work_idx ? p.work_idx[it] : (int32_t)it;
    if ((uint32_t)idx >= (uint32_t)p.work_cap) {  // a list entry outside work[]: never dereferenced
      atomicOr(p.work_count + kErrSlot, kErrWorkIdx);
      continue;
    }
    if (p.work[idx].n == -1) {
      const int pos = atomicAdd(p.work_count + kOvfSlot, 1);
      if (pos < p.work_cap) ovf_list[pos] = idx;
      else atomicOr(p.work_count + kErrSlot, kErrOvfList);
    }
  }
}

template <int RL, bool NORM>
__global__ __launch_bounds__(256) void assign_rescreen_kernel(AssignParams p, const int32_t* __restrict__ ovf_list) {
  constexpr int kV = kHalfDim / 128;  // float4 per lane of a half
  const int lane = threadIdx.x & 63, hl = lane & 31, hh = lane >> 5;
  const int wid = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int nw = gridDim.x * 4;
  const int64_t nov = p.work_count[kOvfSlot];
  const int nv = p.dim / 4;
  const float eps = (float)(p.dim + 4) * 0x1p-24f * 1.001f;
  for (int64_t it0 = 2 * (int64_t)wid; it0 < nov; it0 += 2 * (int64_t)nw) {
    const bool active = it0 + hh < nov;  // an idle half repeats its partner's item and writes nothing
    const int32_t idx = ovf_list[active ? it0 + hh : it0];
    WorkItem w = p.work[idx];
    const float* xr = p.x + (int64_t)w.row * p.dim;
    const float* car = RL >= 1 ? p.ca + (int64_t)seg_row(p.seg_ca, w.seg) * p.dim : nullptr;
    const float* cbr = RL >= 2 ? p.cb + (int64_t)seg_row(p.seg_cb, w.seg) * p.dim : nullptr;
    // the row as the re-score rebuilds it (the reference's fp32 operation sequence)
    float4 v[kV];
    double ss = 0.0;
#pragma unroll
    for (int m = 0; m < kV; ++m) {
      const int i = hl + 32 * m;
      if (i < nv) {
        float4 a = reinterpret_cast<const float4*>(xr)[i];
        if (RL >= 1) {
          const float4 c = reinterpret_cast<const float4*>(car)[i];
          a = make_float4(a.x - c.x, a.y - c.y, a.z - c.z, a.w - c.w);
        }
        if (RL >= 2) {
          if (NORM) {
            const float d1 = p.den_in[w.row];
            a = make_float4(a.x / d1, a.y / d1, a.z / d1, a.w / d1);
          }
          const float4 c = reinterpret_cast<const float4*>(cbr)[i];
          a = make_float4(a.x - c.x, a.y - c.y, a.z - c.z, a.w - c.w);
        }
        v[m] = a;
        ss += (double)a.x * a.x + (double)a.y * a.y + (double)a.z * a.z + (double)a.w * a.w;
      } else {
        v[m] = make_float4(0.f, 0.f, 0.f, 0.f);
      }
    }
    if (NORM && RL >= 1) {
      // the screen wrote den_out for every listed row at RL = 1; level 2 recomputes its own divisor
      const float den = (RL == 1 && p.den_out) ? p.den_out[w.row] : (float)sqrt(half_sum(ss)) + 1e-8f;
#pragma unroll
      for (int m = 0; m < kV; ++m)
        v[m] = make_float4(v[m].x / den, v[m].y / den, v[m].z / den, v[m].w / den);
    }
    const int base = p.cand_base[w.seg];
    const int n = p.cand_count[w.seg];
    const int nmax = max(n, __shfl_xor(n, 32));  // both halves walk the same batches
    bool ovf = n > 65535;
    float U = INFINITY;
    int cnt = 0;
    int lk[kMaxList];
    float llb[kMaxList];
#pragma unroll
    for (int k = 0; k < kMaxList; ++k) {
      lk[k] = -1;
      llb[k] = INFINITY;
    }
    for (int j0 = 0; j0 < nmax; j0 += kBatch) {
      float acc[kBatch];
#pragma unroll
      for (int jj = 0; jj < kBatch; ++jj) {
        const int j = j0 + jj;
        acc[jj] = 0.f;
        if (j < n) {
          const float4* cr = reinterpret_cast<const float4*>(p.centers + (int64_t)cand_global(p, base, j) * p.dim);
#pragma unroll
          for (int m = 0; m < kV; ++m) {
            const int i = hl + 32 * m;
            if (i < nv) {
              const float4 c = cr[i];
              const float d0 = v[m].x - c.x, d1 = v[m].y - c.y, d2 = v[m].z - c.z, d3 = v[m].w - c.w;
              acc[jj] = fmaf(d0, d0, fmaf(d1, d1, fmaf(d2, d2, fmaf(d3, d3, acc[jj]))));
            }
          }
        }
      }
      // the re-score's halving reduction inside the half (fp32): lane hl ends with candidate
      // jj(hl) = 4*((hl>>4)&1) + 2*((hl>>3)&1) + ((hl>>2)&1) summed over the half
      float r4[4], r2[2], r1;
      const bool b4 = hl & 16, b3 = hl & 8, b2 = hl & 4;
#pragma unroll
      for (int j = 0; j < 4; ++j) r4[j] = (b4 ? acc[j + 4] : acc[j]) + __shfl_xor(b4 ? acc[j] : acc[j + 4], 16);
#pragma unroll
      for (int j = 0; j < 2; ++j) r2[j] = (b3 ? r4[j + 2] : r4[j]) + __shfl_xor(b3 ? r4[j] : r4[j + 2], 8);
      r1 = (b2 ? r2[1] : r2[0]) + __shfl_xor(b2 ? r2[0] : r2[1], 4);
      r1 += __shfl_xor(r1, 2);
      r1 += __shfl_xor(r1, 1);
      const int my_j = j0 + 4 * ((hl >> 4) & 1) + 2 * ((hl >> 3) & 1) + ((hl >> 2) & 1);
      const bool real = my_j < n;
      const float lb = real ? r1 - r1 * eps : INFINITY;
      float ub = real ? fmaf(r1, eps, r1) + 1e-30f : INFINITY;
      ovf = ovf || (real && r1 != r1);  // a NaN distance: the fp64 pass applies its NaN rule
      ub = fminf(ub, __shfl_xor(ub, 4));
      ub = fminf(ub, __shfl_xor(ub, 8));
      ub = fminf(ub, __shfl_xor(ub, 16));
      U = fminf(U, ub);
#pragma unroll
      for (int jj = 0; jj < kBatch; ++jj) {
        const int src = (hh << 5) | (16 * ((jj >> 2) & 1) + 8 * ((jj >> 1) & 1) + 4 * (jj & 1));
        const float lbj = __shfl(lb, src);
        const bool q = lbj <= U;
        if (q && cnt == kMaxList) {  // full: drop entries the current U already excludes (rare)
          int pos = 0;
          int nk[kMaxList];
          float nl[kMaxList];
#pragma unroll
          for (int t = 0; t < kMaxList; ++t) {
            nk[t] = -1;
            nl[t] = INFINITY;
          }
#pragma unroll
          for (int k = 0; k < kMaxList; ++k) {
            const bool keep = llb[k] <= U;
#pragma unroll
            for (int t = 0; t < kMaxList; ++t) {
              const bool put = keep && pos == t;
              nk[t] = put ? lk[k] : nk[t];
              nl[t] = put ? llb[k] : nl[t];
            }
            pos += keep ? 1 : 0;
          }
#pragma unroll
          for (int t = 0; t < kMaxList; ++t) {
            lk[t] = nk[t];
            llb[t] = nl[t];
          }
          cnt = pos;
          ovf = ovf || cnt == kMaxList;
        }
        const bool ins = q && cnt < kMaxList;
#pragma unroll
        for (int k = 0; k < kMaxList; ++k) {
          const bool put = ins && k == cnt;
          lk[k] = put ? j0 + jj : lk[k];
          llb[k] = put ? lbj : llb[k];
        }
        cnt += ins ? 1 : 0;
      }
    }
    // a NaN distance seen by any lane of the half (each lane checks only its own candidate) sends the
    // whole row to the fp64 pass, which applies the reference's NaN rule
#pragma unroll
    for (int o = 1; o < 32; o <<= 1) ovf = ovf || __shfl_xor((int)ovf, o) != 0;
    // the final list: entries still within the final U, ascending candidate order
    int m = 0;
    uint16_t outc[kMaxList];
#pragma unroll
    for (int t = 0; t < kMaxList; ++t) outc[t] = 0xFFFF;
#pragma unroll
    for (int k = 0; k < kMaxList; ++k) {
      const bool keep = k < cnt && llb[k] <= U;
#pragma unroll
      for (int t = 0; t < kMaxList; ++t) outc[t] = (keep && m == t) ? (uint16_t)lk[k] : outc[t];
      m += keep ? 1 : 0;
    }
    if (hl == 0 && active && !ovf && m >= 1) {
      w.n = m;
#pragma unroll
      for (int t = 0; t < kMaxList; ++t) w.cand[t] = outc[t];
      p.work[idx] = w;
    }
  }
}

// tile -> segment map of the per-tile screen (one thread per tile, binary search of seg_tile_off)
__global__ __launch_bounds__(256) void tile_seg128_kernel(const int32_t* __restrict__ seg_tile_off, int nseg,
                                                          int64_t cap, int32_t* __restrict__ tile_seg) {
  const int ntiles = seg_tile_off[nseg];
  for (int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x; t < ntiles && t < cap; t += (int64_t)gridDim.x * 256) {
    int lo = 0, hi = nseg;
    while (hi - lo > 1) {
      const int mid = (lo + hi) >> 1;
      if (seg_tile_off[mid] <= t) lo = mid; else hi = mid;
    }
    tile_seg[t] = lo;
  }
}

// Stream-path compaction: rows whose out_global is the re-score sentinel (-2) -> work_idx list.
// One atomic per block: the block counts the sentinels of its 16K-row range, reserves, then lists
// (the row order inside the list is irrelevant).  A per-wave atomic serialises on the one counter.
constexpr int kCompactRows = 16384;
__global__ __launch_bounds__(256) void sentinel_compact_kernel(const int32_t* __restrict__ out_global, int64_t n,
                                                               int32_t* __restrict__ work_count,
                                                               int32_t* __restrict__ work_idx, int64_t cap) {
  __shared__ int wcount[4], wbase[4];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t r0 = (int64_t)blockIdx.x * kCompactRows, r1 = min(n, r0 + kCompactRows);
  int cnt = 0;
  for (int64_t i = r0 + threadIdx.x; i < r1; i += 256) cnt += out_global[i] == -2 ? 1 : 0;
  for (int o = 32; o > 0; o >>= 1) cnt += __shfl_xor(cnt, o);
  if (lane == 0) wcount[wave] = cnt;
  __syncthreads();
  if (threadIdx.x == 0) {
    const int tot = wcount[0] + wcount[1] + wcount[2] + wcount[3];
    const int base = tot ? atomicAdd(work_count, tot) : 0;
    wbase[0] = base;
    wbase[1] = base + wcount[0];
    wbase[2] = wbase[1] + wcount[1];
    wbase[3] = wbase[2] + wcount[2];
  }
  __syncthreads();
  if (!wcount[wave]) return;
  int pos = wbase[wave];
  // each wave lists the sentinels of the rows it counted (same strided walk, in order)
  for (int64_t i0 = r0 + wave * 64; i0 < r1; i0 += 256) {
    const int64_t i = i0 + lane;
    const bool need = i < r1 && out_global[i] == -2;
    const unsigned long long m = __ballot(need);
    if (need) {
      const int64_t q = (int64_t)pos + __popcll(m & ((1ull << lane) - 1ull));
      if (q < cap) work_idx[q] = (int32_t)i;
      else atomicOr(work_count + kErrSlot, kErrCompact);
    }
    pos += __popcll(m);
  }
}

// ---------------------------------------------------------------------------
// MFMA numerics probe: D = A.B + C with ONE v_mfma_f32_32x32x16_{bf16,f16} (32x16 A, 16x32 B,
// 32x32 C/D, row-major).  tests/test_mfma_numerics.py uses it to pin the accumulation model the
// screening bound relies on.
// ---------------------------------------------------------------------------
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
template <bool F16>
__global__ __launch_bounds__(64) void mfma_probe_kernel(const uint16_t* __restrict__ a, const uint16_t* __restrict__ b,
                                                        const float* __restrict__ c, float* __restrict__ d) {
  const int l = threadIdx.x, i = l & 31, hh = l >> 5;
  f32x16 acc;
#pragma unroll
  for (int v = 0; v < 16; ++v) acc[v] = c[((v & 3) + 8 * (v >> 2) + 4 * hh) * 32 + i];
  if (F16) {
    f16x8 av, bv;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      av[j] = __builtin_bit_cast(_Float16, a[i * 16 + 8 * hh + j]);
      bv[j] = __builtin_bit_cast(_Float16, b[(8 * hh + j) * 32 + i]);
    }
    acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(av, bv, acc, 0, 0, 0);
  } else {
    bf16x8 av, bv;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      av[j] = __builtin_bit_cast(__bf16, a[i * 16 + 8 * hh + j]);
      bv[j] = __builtin_bit_cast(__bf16, b[(8 * hh + j) * 32 + i]);
    }
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av, bv, acc, 0, 0, 0);
  }
#pragma unroll
  for (int v = 0; v < 16; ++v) d[((v & 3) + 8 * (v >> 2) + 4 * hh) * 32 + i] = acc[v];
}

// fp8 (OCP e4m3) form, groundwork for a level-1 correction MFMA: D = A.B + C with ONE
// v_mfma_scale_f32_32x32x64_f8f6f4 (unit scales), A 32x64 and B 64x32 as bytes.  Lane half hh holds K = 32 hh ..
// 32 hh + 31 of its row (A) / column (B); a dot product is invariant to any K order applied to both operands
// alike, so A.B + C comes out exactly iff the instruction maps the two operands' registers to K the same way.
typedef __attribute__((ext_vector_type(8))) int i32x8;
__global__ __launch_bounds__(64) void mfma_probe_f8_kernel(const uint8_t* __restrict__ a, const uint8_t* __restrict__ b,
                                                           const float* __restrict__ c, float* __restrict__ d) {
  const int l = threadIdx.x, i = l & 31, hh = l >> 5;
  f32x16 acc;
#pragma unroll
  for (int v = 0; v < 16; ++v) acc[v] = c[((v & 3) + 8 * (v >> 2) + 4 * hh) * 32 + i];
  i32x8 av, bv;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    uint32_t wa = 0, wb = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int k = 32 * hh + 4 * j + q;
      wa |= (uint32_t)a[i * 64 + k] << (8 * q);
      wb |= (uint32_t)b[k * 32 + i] << (8 * q);
    }
    av[j] = (int)wa;
    bv[j] = (int)wb;
  }
  acc = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(av, bv, acc, 0, 0, 0, 127, 0, 127);
#pragma unroll
  for (int v = 0; v < 16; ++v) d[((v & 3) + 8 * (v >> 2) + 4 * hh) * 32 + i] = acc[v];
}

// the hi terms of the interleaved table, contiguous per centre: each 32-dim chunk of c16 is 4 16-B pieces of hi
// terms then 4 of lo terms, so hi piece i is c16 piece 8 (i / 4) + i % 4
__global__ __launch_bounds__(256) void centers_hi_kernel(const uint4* __restrict__ c16, int64_t n, uint4* __restrict__ hi) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
    hi[i] = c16[(i >> 2) * 8 + (i & 3)];
}

// ---------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------
template <int NT, int S, bool T3, bool ONE, int CW = 1>
void set_attrs(bool* ok) {
  const int bytes = ScreenLayout<NT, S, T3, CW>::kMaxBytes;
  const void* ks[] = {(const void*)assign_screen_kernel<NT, S, 0, false, T3, ONE, CW>,
                      (const void*)assign_screen_kernel<NT, S, 1, false, T3, ONE, CW>,
                      (const void*)assign_screen_kernel<NT, S, 1, true, T3, ONE, CW>,
                      (const void*)assign_screen_kernel<NT, S, 2, false, T3, ONE, CW>,
                      (const void*)assign_screen_kernel<NT, S, 2, true, T3, ONE, CW>};
  for (const void* k : ks)
    if (hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, bytes) != hipSuccess) *ok = false;
}

// screen variant (tuning / A-B tests): 0 default (per level: see rqsid_assign); 1: per-tile kernel
// only; 2: per-tile kernel with the multi-sweep list epilogue on single-pass segments; 5: the
// persistent streamed kernels (assign_stream.hip, RQSID_STREAM_SHAPE) where they apply; 6: the
// centre-resident screen; 7: no candidate split; 8: the row-resident screen (assign_rows.hip,
// RQSID_ROWS_SHAPE)
int screen_variant() {  // read per call: tests switch it within one process
  const char* e = getenv("RQSID_SCREEN_VARIANT");
  return e ? atoi(e) : 0;
}

// ring depth of the candidate-split form (one block per CU).  S = 3 (96 KiB in flight per CU instead of
// 48) measured no faster on the XL levels (L2 15.3 vs 14.8 ms), so the smaller ring stays
#ifndef RQSID_SPLIT_S
#define RQSID_SPLIT_S 2
#endif
constexpr int kSplitS = RQSID_SPLIT_S;

bool g_attr_done[kMaxDevices] = {};
int ensure_attrs() {
  const int dev = current_device();
  if (dev < 0) return fail(RQSID_E_LAUNCH, "assign: hipGetDevice failed");
  if (g_attr_done[dev]) return RQSID_OK;
  bool ok = true;
  set_attrs<4, 2, false, true>(&ok);
  set_attrs<8, 2, false, true>(&ok);
  set_attrs<4, 2, true, true>(&ok);
  set_attrs<4, 2, false, false>(&ok);
  set_attrs<8, 2, false, false>(&ok);
  set_attrs<4, 2, true, false>(&ok);
  set_attrs<8, kSplitS, false, true, 2>(&ok);
  set_attrs<4, kSplitS, true, true, 2>(&ok);
  if (!ok) return fail(RQSID_E_LAUNCH, "assign: cannot raise the dynamic LDS limit");
  g_attr_done[dev] = true;
  return RQSID_OK;
}

template <int NT, int S, bool T3, bool ONE, int CW = 1>
void launch_screen(const AssignParams& p, int rl, bool norm, unsigned grid, hipStream_t st) {
  const size_t lds = ScreenLayout<NT, S, T3, CW>::bytes(rl, p.dim);
  const dim3 blk(256 * CW);
  if (rl == 0) hipLaunchKernelGGL((assign_screen_kernel<NT, S, 0, false, T3, ONE, CW>), dim3(grid), blk, lds, st, p);
  else if (rl == 1 && norm) hipLaunchKernelGGL((assign_screen_kernel<NT, S, 1, true, T3, ONE, CW>), dim3(grid), blk, lds, st, p);
  else if (rl == 1) hipLaunchKernelGGL((assign_screen_kernel<NT, S, 1, false, T3, ONE, CW>), dim3(grid), blk, lds, st, p);
  else if (norm) hipLaunchKernelGGL((assign_screen_kernel<NT, S, 2, true, T3, ONE, CW>), dim3(grid), blk, lds, st, p);
  else hipLaunchKernelGGL((assign_screen_kernel<NT, S, 2, false, T3, ONE, CW>), dim3(grid), blk, lds, st, p);
}
template <int NT, int S, bool T3>
void launch_screen2(const AssignParams& p, int rl, bool norm, unsigned grid, bool one, hipStream_t st) {
  if (one) launch_screen<NT, S, T3, true>(p, rl, norm, grid, st);
  else launch_screen<NT, S, T3, false>(p, rl, norm, grid, st);
}

}  // namespace
}  // namespace rqsid

using namespace rqsid;

extern "C" {

int rqsid_prepare_centers(const float* centers, int64_t k, int32_t dim, uint16_t* c16, float* c_meta,
                          void* stream) {
  if (!centers || !c16 || !c_meta || k < 0 || dim <= 0 || dim % kChunk || dim > kMaxDim)
    return fail(RQSID_E_ARG, "prepare_centers: bad arguments (k=%lld dim=%d)", (long long)k, dim);
  if (k == 0) return RQSID_OK;
  hipStream_t st = (hipStream_t)stream;
  float* scale = c_meta + 4 * k;  // row k of meta
  if (fill_async(scale, 0, 4 * sizeof(float), st) != hipSuccess)
    return fail(RQSID_E_LAUNCH, "prepare_centers: hipMemsetAsync failed");
  const int64_t n = k * dim;
  const unsigned g = (unsigned)(cdiv(n, 256 * 16) < 2048 ? cdiv(n, 256 * 16) : 2048);
  hipLaunchKernelGGL(centers_absmax_kernel, dim3(g), dim3(256), 0, st, centers, n, reinterpret_cast<unsigned*>(scale));
  hipLaunchKernelGGL(prepare_centers_kernel, dim3((unsigned)cdiv(k, 4)), dim3(256), 0, st,
                     centers, k, dim, reinterpret_cast<_Float16*>(c16), reinterpret_cast<float4*>(c_meta));
  hipLaunchKernelGGL(centers_scale_kernel, dim3(1), dim3(1), 0, st, scale);
  return check_launch("prepare_centers");
}

int rqsid_prepare_centers_hi(const uint16_t* c16, int64_t k, int32_t dim, uint16_t* c16_hi, void* stream) {
  if (!c16 || !c16_hi || k < 0 || dim <= 0 || dim % kChunk || dim > kMaxDim)
    return fail(RQSID_E_ARG, "prepare_centers_hi: bad arguments (k=%lld dim=%d)", (long long)k, dim);
  if (k == 0) return RQSID_OK;
  const int64_t n = k * dim / 8;  // 16-B pieces of the hi table
  hipLaunchKernelGGL(centers_hi_kernel, dim3((unsigned)grid_cap(cdiv(n, 256), 8192)), dim3(256), 0, (hipStream_t)stream,
                     reinterpret_cast<const uint4*>(c16), n, reinterpret_cast<uint4*>(c16_hi));
  return check_launch("prepare_centers_hi");
}

int32_t rqsid_assign_tile_rows(void) { return kTileRows; }

// workspace: [0,256) counters and store sinks | WorkItem[n_rows] | tile->segment map i32[n_rows]
// (tiles <= rows) | compact row list i32[n_rows] (resident screen: 32-row tile offsets per segment) |
// resident screen tile descriptors int4[n_rows] | overflow item list i32[n_rows] (fp32 re-screen)
int64_t rqsid_assign_workspace_bytes(int64_t n_rows) {
  const int64_t n = n_rows > 0 ? n_rows : 0;
  return 256 + n * (int64_t)sizeof(WorkItem) + 3 * ((n * 4 + 255) / 256 * 256) + resident_desc_bytes(n);
}

int rqsid_assign(const float* x, int64_t n_rows, int32_t dim, const int32_t* row_index, int32_t n_segments,
                 const int32_t* seg_row_off, const int32_t* seg_tile_off, int64_t max_tiles, const float* centers,
                 const uint16_t* c16, const uint16_t* c16_hi, const float* c_meta, int32_t n_centers,
                 const int32_t* cand_base,
                 const int32_t* cand_count, int32_t cand_count_max, const int32_t* cand_idx,
                 const int32_t* cand_lid, const uint8_t* seg_flags, int32_t res_levels, int32_t res_normalize, const float* ca,
                 const int32_t* seg_ca, const float* cb, const int32_t* seg_cb, const float* den_in,
                 float* den_out, int32_t* out_local, int32_t* out_global, int32_t screen_terms, void* workspace,
                 int64_t workspace_bytes, void* stream) {
  if (dim <= 0 || dim % kChunk || dim > kMaxDim || n_rows < 0 || n_segments <= 0 || !seg_row_off ||
      !seg_tile_off || !centers || !c16 || !c_meta || !cand_base || !cand_count || (n_rows > 0 && (!out_local || !out_global)) ||
      n_centers <= 0 || cand_count_max < 0 || max_tiles < 0 || n_rows > INT32_MAX || res_levels < 0 ||
      res_levels > 2 || (screen_terms != 0 && screen_terms != 1 && screen_terms != 3))
    return fail(RQSID_E_ARG, "assign: bad arguments (n=%lld dim=%d S=%d K=%d levels=%d)", (long long)n_rows, dim,
                n_segments, n_centers, res_levels);
  if ((res_levels >= 1 && !ca) || (res_levels == 2 && (!cb || !seg_cb || (res_normalize && n_rows > 0 && !den_in))))
    return fail(RQSID_E_ARG, "assign: residual inputs missing for res_levels=%d", res_levels);
  if (!workspace || workspace_bytes < rqsid_assign_workspace_bytes(n_rows))
    return fail(RQSID_E_WORKSPACE, "assign: workspace too small");
  if (n_rows == 0 || max_tiles == 0) return RQSID_OK;
  if (max_tiles > INT32_MAX - 8) return fail(RQSID_E_ARG, "assign: too many tiles");
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
  p.c16 = c16;
  p.c16h = c16_hi;
  p.c_meta = c_meta;
  p.n_centers = n_centers;
  p.cand_base = cand_base;
  p.cand_count = cand_count;
  p.cand_idx = cand_idx;
  p.cand_lid = cand_lid;
  p.seg_flags = seg_flags;
  p.out_local = out_local;
  p.out_global = out_global;
  p.work_count = (int32_t*)workspace;
  p.work = (WorkItem*)((char*)workspace + 256);
  p.work_cap = n_rows;
  p.work_idx = nullptr;
  int32_t* tile_seg = (int32_t*)((char*)workspace + 256 + n_rows * (int64_t)sizeof(WorkItem));
  int32_t* work_idx = tile_seg + (n_rows * 4 + 255) / 256 * 64;
  p.acc_rel = accumulation_rel(dim);
  p.ca = ca;
  p.seg_ca = seg_ca;
  p.cb = cb;
  p.seg_cb = seg_cb;
  p.den_in = den_in;
  p.den_out = den_out;
  const bool norm = res_normalize != 0;
  // header ints [0, 60) per call; [60, 64) hold the sticky error word (kErrSlot), zeroed by the allocator
  if (fill_async(workspace, 0, 4 * kErrSlot, st) != hipSuccess) return fail(RQSID_E_LAUNCH, "assign: memset");
  const unsigned grid = (unsigned)((max_tiles + 7) / 8 * 8);  // XCD remap needs a multiple of 8
  // Measured on MI355X (tools/screen_sweep.py): independent blocks per CU beat ring depth: NT4 with
  // S=2 runs 3 blocks/CU, NT8 with S=2 runs 2 blocks/CU (RQSID_SCREEN_VARIANT=1/3 select the older
  // deeper-ring single-block configurations for comparison).
  // Terms: the 3-term screen (rounding residuals of both operands summed by two more MFMAs) shrinks
  // the bound ~5x at 2 blocks/CU; auto picks it for residual levels with <= 128 candidates, where
  // trained codebooks leave the most rows inside the 1-term bound ("Screen terms").
  // (The 8-tile form has no 3-term build: its second accumulator set does not fit 256 VGPRs.)
  // ONE: single-pass segments take the collapsed-bound epilogue (RQSID_SCREEN_VARIANT=2: the
  // per-candidate two-sweep list epilogue, for comparison).
  // Wider first-residual levels (the XL preset's middle level: 256 candidates per parent) take the
  // 3-term screen in two 128-candidate passes: the 1-term bound leaves ~2/3 of those rows to the fp64
  // re-score (measured: 4.1 M of 6.25 M rows, 14.3 ms).
  const bool t3 = (cand_count_max <= 128 && (screen_terms == 3 || (screen_terms == 0 && res_levels >= 1))) ||
                  (cand_count_max <= 256 && (screen_terms == 3 || (screen_terms == 0 && res_levels == 1)));
  p.terms = t3 ? 3 : 1;
  const bool legacy = screen_variant() == 2;
  // the persistent streamed kernel (assign_stream.hip): 512-d rows, single-pass segments, no local-id
  // remap, den_out present whenever it normalises a first-level residual
  const int nt = t3 || cand_count_max <= 128 ? 4 : 8;
  const bool stream_ok = dim == 512 && cand_count_max <= 256 && !cand_lid && (res_levels != 1 || !norm || den_out) &&
                         n_rows >= 64 * 256 && (int64_t)n_segments + 1 <= n_rows &&
                         stream_supported(nt, t3, res_levels, norm);
  // Default (variant 0): the ping-pong form for 1-term 256-candidate RESIDUAL levels (gathered rows;
  // measured L2 of the bench 7.58 vs 7.92 ms), the per-tile kernel elsewhere (L0 3.37 vs 3.99, L1 6.04 vs
  // 6.54 ms; the XL preset's 256-candidate level 0 on contiguous rows 3.03 vs 3.62-3.65 ms).
  // Variant 1 forces the per-tile kernel, variant 5 the stream forms (RQSID_STREAM_SHAPE).
  const int variant = screen_variant();
  const int shape = variant == 5 ? 0 : (variant == 0 && nt == 8 && !t3 && res_levels >= 1 ? 88 : -1);
  const bool use_stream = stream_ok && shape >= 0 && variant != 6;
  // the centre-resident screen (assign_resident.hip): variant 6 forces it wherever it applies (1-term,
  // <= 256 candidates).  Not the default yet: measured L2 of the bench 8.0-9.1 ms against the ping-pong
  // form's 7.6 ms ('Centre-resident screen')
  const bool res_ok = resident_supported(dim, cand_count_max, t3, res_levels) && (int64_t)n_segments + 1 <= n_rows &&
                      (res_levels != 1 || !norm || den_out);
  const bool use_res = res_ok && variant == 6;
  // the row-resident screen (assign_rows.hip): variant 8 forces it wherever it applies (1-term levels of
  // 512-d rows with <= 512 candidates)
  // default for 1-term residual levels wider than 256 candidates (the XL preset's 512-candidate last level:
  // 7.0 vs 14.8 ms for the candidate-split screen, profiles/r4_xl_rows_ab.txt); the 256-candidate PROD level
  // keeps the ping-pong form (7.4 vs 7.6-7.8 ms)
  const bool use_rows = (variant == 8 || (variant == 0 && res_levels >= 1 && cand_count_max > 256)) &&
                        rows_supported(dim, cand_count_max, t3, res_levels, norm) && (int64_t)n_segments + 1 <= n_rows;
  // the producer/consumer screen (assign_pc.hip): the default for the residual levels it covers (PROD level 1,
  // 3-term <= 128 candidates, and level 2, 1-term <= 256); RQSID_PC=0 keeps the older
  // dispatch above for A/B, variant 9 forces it wherever it applies
  const char* pce = getenv("RQSID_PC");
  const bool pc_ok = pc_supported(dim, cand_count_max, t3, res_levels) &&
                     (res_levels != 1 || !norm || den_out) && (int64_t)n_segments + 1 <= n_rows &&
                     pc_desc_bytes(n_rows, n_segments) <= resident_desc_bytes(n_rows);
  // (default: the 1-term levels; RQSID_PC=2 takes the 3-term ones too, RQSID_PC=0 none)
  const int pc_mode = pce ? atoi(pce) : 1;
  const bool use_pc = pc_ok && (variant == 9 || (variant == 0 && (pc_mode >= 2 || (pc_mode == 1 && !t3))));
  if (use_pc) {
    // R-row tile offsets in the compact-list area, the tile map in the tile_seg slot, the tile descriptors in
    // the resident screen's descriptor area; a failed launch returns before the compaction and re-score
    int4* desc = reinterpret_cast<int4*>(work_idx + (n_rows * 4 + 255) / 256 * 64);
    if ((rc = launch_pc_screen(p, t3, res_levels, norm, tile_seg, work_idx, desc, n_rows, st))) return rc;
    if ((rc = check_launch("assign_pc"))) return rc;
    hipLaunchKernelGGL(sentinel_compact_kernel, dim3((unsigned)cdiv(n_rows, kCompactRows)), dim3(256), 0, st, out_global,
                       n_rows, p.work_count, work_idx, n_rows);
    p.work_idx = work_idx;
  } else if (use_rows) {
    // R-row tile offsets in the compact-list area, the tile map in the tile_seg slot; compact work list
    if ((rc = launch_rows_screen(p, res_levels, norm, tile_seg, work_idx, n_rows, st))) return rc;
  } else if (use_res) {
    p.err = p.work_count + 48;  // zeroed with the workspace header above
    const char* fc = getenv("RQSID_TEST_FORCE_SPIN_CAP");
    p.force_cap = fc && atoi(fc) ? 1 : 0;
    int4* desc = reinterpret_cast<int4*>(work_idx + (n_rows * 4 + 255) / 256 * 64);
    // tile_seg's slot holds the segment of each ambiguous row
    if ((rc = launch_resident_screen(p, t3, res_levels, norm, desc, work_idx, tile_seg, n_rows, st))) return rc;
    // re-score rows carry the sentinel -2 and their pass masks at work[row] (the 32-row tile offsets in
    // the compact-list area are dead by now); the expand pass makes them work items
    hipLaunchKernelGGL(sentinel_compact_kernel, dim3((unsigned)cdiv(n_rows, kCompactRows)), dim3(256), 0, st, out_global,
                       n_rows, p.work_count, work_idx, n_rows);
    p.work_idx = work_idx;
    launch_resident_expand(p, tile_seg, t3, n_rows, st);
  } else if (use_stream) {
    // the 256-row tile offsets live in the compact-list area until the compaction pass
    // a failed stream launch returns its status here: the compaction and re-score below must never run
    // over an out_global the screen did not write
    if ((rc = launch_stream_screen(p, nt, t3, res_levels, norm, tile_seg, work_idx, n_rows, shape, st))) return rc;
    if ((rc = check_launch("assign_stream"))) return rc;
    hipLaunchKernelGGL(sentinel_compact_kernel, dim3((unsigned)cdiv(n_rows, kCompactRows)), dim3(256), 0, st, out_global,
                       n_rows, p.work_count, work_idx, n_rows);
    p.work_idx = work_idx;
  } else {
    if (n_segments > 1) {  // (tiles <= rows: the map fits its workspace slot)
      hipLaunchKernelGGL(tile_seg128_kernel, dim3(grid_cap(cdiv(max_tiles, 256), 4096)), dim3(256), 0, st, seg_tile_off,
                         n_segments, n_rows, tile_seg);
      p.tile_seg = tile_seg;
    }
  }
  // candidate-split single pass (CW = 2) for segments wider than one wave's tiles: 3-term <= 256
  // candidates, 1-term <= 512 (the XL preset's middle and last levels); RQSID_SCREEN_VARIANT=7 (or 2)
  // keeps the multi-pass screen for comparison
  const bool split = !legacy && variant != 7 && dim <= kSplitDim;
  if (use_pc || use_stream || use_res || use_rows) {
  } else if (t3 && cand_count_max > 128 && split) launch_screen<4, kSplitS, true, true, 2>(p, res_levels, norm, grid, st);
  else if (t3) launch_screen2<4, 2, true>(p, res_levels, norm, grid, !legacy && cand_count_max <= 128, st);
  else if (cand_count_max <= 128) launch_screen2<4, 2, false>(p, res_levels, norm, grid, !legacy, st);
  else if (cand_count_max <= 256) launch_screen2<8, 2, false>(p, res_levels, norm, grid, !legacy, st);
  else if (cand_count_max <= 512 && split) launch_screen<8, kSplitS, false, true, 2>(p, res_levels, norm, grid, st);
  else launch_screen<8, 2, false, false>(p, res_levels, norm, grid, st);
  if ((rc = check_launch("assign_screen"))) return rc;
  const dim3 g(4096);  // multiple of 8 (XCD-grouped work runs)
  // two rows per wave for rows of <= 512 dims (RQSID_RESCORE_FULL=1: one row per wave, for A/B)
  const char* ef = getenv("RQSID_RESCORE_FULL");
  const bool half = dim <= kHalfDim && !(ef && atoi(ef));
  // rows the screen left with "every candidate" get an fp32 list first (RQSID_NO_RESCREEN=1: off, A/B)
  const char* nr = getenv("RQSID_NO_RESCREEN");
  int32_t* ovf_list = nullptr;
  if (dim <= kHalfDim && !(nr && atoi(nr)) && cand_count_max > kMaxList) {
    ovf_list = reinterpret_cast<int32_t*>(reinterpret_cast<char*>(work_idx) + (n_rows * 4 + 255) / 256 * 256 +
                                          resident_desc_bytes(n_rows));
    hipLaunchKernelGGL(overflow_list_kernel, dim3(grid_cap(cdiv(n_rows, 256), 1024)), dim3(256), 0, st, p, ovf_list);
#define RQ_RSC(RL, NORM) hipLaunchKernelGGL((assign_rescreen_kernel<RL, NORM>), dim3(2048), dim3(256), 0, st, p, ovf_list)
    if (res_levels == 0) RQ_RSC(0, false);
    else if (res_levels == 1 && norm) RQ_RSC(1, true);
    else if (res_levels == 1) RQ_RSC(1, false);
    else if (norm) RQ_RSC(2, true);
    else RQ_RSC(2, false);
#undef RQ_RSC
    if ((rc = check_launch("assign_rescreen"))) return rc;
  }
#define RQ_RS(RL, NORM)                                                                                       \
  do {                                                                                                        \
    if (half && ovf_list) {                                                                                   \
      hipLaunchKernelGGL((assign_rescore_half_kernel<RL, NORM>), g, dim3(256), 0, st, p, ovf_list, 1);          \
      hipLaunchKernelGGL((assign_rescore_half_kernel<RL, NORM>), g, dim3(256), 0, st, p, ovf_list, 2);          \
    } else if (half) {                                                                                        \
      hipLaunchKernelGGL((assign_rescore_half_kernel<RL, NORM>), g, dim3(256), 0, st, p, (const int32_t*)nullptr, 0); \
    } else {                                                                                                  \
      hipLaunchKernelGGL((assign_rescore_kernel<RL, NORM>), g, dim3(256), 0, st, p);                          \
    }                                                                                                         \
  } while (0)
  if (res_levels == 0) RQ_RS(0, false);
  else if (res_levels == 1 && norm) RQ_RS(1, true);
  else if (res_levels == 1) RQ_RS(1, false);
  else if (norm) RQ_RS(2, true);
  else RQ_RS(2, false);
#undef RQ_RS
  if ((rc = check_launch("assign_rescore"))) return rc;
  if (use_res) {
    // the resident screen's role waits are capped (assign_resident.hip): a wave that gave up waiting
    // left wrong IDs behind, so the call fails instead of returning them (one readback, opt-in path)
    int32_t err = 0;
    if (hipMemcpyAsync(&err, p.err, 4, hipMemcpyDeviceToHost, st) != hipSuccess || hipStreamSynchronize(st) != hipSuccess)
      return fail(RQSID_E_LAUNCH, "assign: error word readback");
    if (err) return fail(RQSID_E_LAUNCH, "assign: a resident-screen wait reached its spin cap (error word %d)", err);
  }
  return RQSID_OK;
}

#ifdef RQSID_STAMPS
int rqsid_debug_stamps_tile(unsigned long long* out8) {
  if (hipMemcpyFromSymbol(out8, HIP_SYMBOL(g_stamps_tile), 8 * sizeof(unsigned long long)) != hipSuccess) return -1;
  const unsigned long long z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  return hipMemcpyToSymbol(HIP_SYMBOL(g_stamps_tile), z, sizeof(z)) == hipSuccess ? 0 : -1;
}
#endif

int rqsid_mfma_probe(int32_t f16, const uint16_t* a, const uint16_t* b, const float* c, float* d, void* stream) {
  if (!a || !b || !c || !d) return fail(RQSID_E_ARG, "mfma_probe: null argument");
  if (f16 == 2)
    hipLaunchKernelGGL(mfma_probe_f8_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream,
                       reinterpret_cast<const uint8_t*>(a), reinterpret_cast<const uint8_t*>(b), c, d);
  else if (f16) hipLaunchKernelGGL(mfma_probe_kernel<true>, dim3(1), dim3(64), 0, (hipStream_t)stream, a, b, c, d);
  else hipLaunchKernelGGL(mfma_probe_kernel<false>, dim3(1), dim3(64), 0, (hipStream_t)stream, a, b, c, d);
  return check_launch("mfma_probe");
}

}  // extern "C"
