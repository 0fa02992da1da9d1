// assign_resident.hip — the centre-resident screen: rqsid_assign's path for 512-d rows whose segments
// hold <= 256 candidates (one fp16 term) or <= 128 (three terms).
//
// Same arithmetic as assign.hip's single-pass screen (fp16 MFMA X·Cᵀ with a rigorous per-candidate
// error bound, pass-bit masks, the exact fp64 re-score of ambiguous rows), different data movement.
// The per-tile kernel re-streams a segment's candidate centres through LDS for every 128-row tile
// (1-2 KiB of centre traffic per row at levels 1 and 2); here the centres stay in registers:
//  * One persistent 8-wave block per CU walks an XCD-contiguous run of 32-row tiles (a segment's
//    tiles are consecutive, so the block meets each segment once).  Every wave holds 32 candidates as
//    the MFMA's A operand for the whole segment: 32 k-steps x f16x8 = 128 VGPRs per lane.  1 term:
//    8 waves x 32 = 256 candidates.  3 terms: waves 0-3 hold the hi terms of 4 x 32 = 128 candidates
//    and compute vh.ch and vl.ch, waves 4-7 hold the lo terms of the same candidates and compute
//    vh.cl; the two partial second-term sums meet in LDS.
//  * The rows are produced ONCE: each wave loads 4 rows of the next tile (fp32, 2 x 1 KiB coalesced
//    loads per row, non-temporal), builds the reference's residual chain in fp32, rounds to fp16 (and
//    the fp16 rounding residual, 3 terms) and writes the MFMA B operand image of the tile to LDS
//    (double buffered, XOR-swizzled: conflict-free 8-B writes and 16-B fragment reads); the per-row
//    bound statistics (|v - fp16(v)|, |v|, the normalising denominator) are reduced across the wave.
//  * Waves 0-3 produce tile j+1 and then multiply tile j; waves 4-7 multiply first and produce after,
//    so on every SIMD one wave's VALU work runs beside the other's MFMAs.
//  * Epilogue per tile: per-candidate upper / lower bounds (the single-pass collapsed bound of
//    assign.hip), the least upper bound across the candidate waves through LDS, one pass mask word per
//    (row, candidate wave), and per row: one passing candidate -> final ID, else a work item for the
//    re-score.  Three barriers per tile (two with one term).
// Segment changes reload the centre registers (from L2: a segment's table is 128-256 KiB) right after
// the last MFMA of the old segment, so the load overlaps the epilogue and the next tile's production.
#include <type_traits>

#include "assign_common.h"

#ifdef RQSID_STAMPS
// diagnostic build: per role (wave 0: produce first, wave 4: multiply first) cycles of
// {loop, segment change, produce, MFMA, epilogue 1 + barrier(s), epilogue 2 + barrier, decisions, tiles}
__device__ unsigned long long g_rstamps[32];
#define RS_NOW() ((uint32_t)__builtin_amdgcn_s_memtime())
#define RS(...) __VA_ARGS__
#else
#define RS(...)
#endif

namespace rqsid {
namespace {

#ifndef RQ_PF
#define RQ_PF 2  // fragment prefetch distance (k-steps)
#endif
#ifndef RQ_ILV
#define RQ_ILV 0  // A/B: VALU instructions pinned after each MFMA of the fused block (0: compiler's order)
#endif
constexpr int kRD = 512;                 // row width of this kernel
constexpr int kRT = 32;                  // rows per tile (the MFMA's N)
constexpr int kKS = kRD / 16;            // k-steps of v_mfma_f32_32x32x16_f16
constexpr int kGS = (kRT + 1) * 16;      // bytes per eight-dim group: 32 rows x 16 B + 16 B pad
constexpr int kImg = kRD / 8 * kGS;      // one fp16 image: 64 eight-dim groups (33 KiB)

__device__ __forceinline__ int runi(int v) { return __builtin_amdgcn_readfirstlane(v); }

// image slot of eight-dim group kh (= dims 8kh .. 8kh+7) of tile row n.  The 16-B pad per group
// shifts consecutive groups by 4 banks, so a producer write (fixed n, kh = lane/2: 8 groups per
// 16-lane group) is conflict-free, a fragment read (fixed kh per half-wave, n = 0..31) is 512
// contiguous bytes, and a lane's reads over the k-steps are one base + immediate offsets
__device__ __forceinline__ int img_off(int kh, int n) { return kh * kGS + n * 16; }

template <bool T3, int RL>
struct ResLayout {
  static constexpr int NCW = T3 ? 4 : 8;                 // candidate waves (32 candidates each)
  static constexpr int NC = NCW * 32;                    // candidate capacity
  static constexpr int kBuf = kImg * (T3 ? 2 : 1);       // vh [+ vl] images of one tile
  static constexpr int kStat = 2 * kBuf;                 // [2 bufs][32 rows] float4 {en, en2, |v|, 1/den}
  static constexpr int kStat2 = kStat + 2 * kRT * 16;    // [2 bufs][32 rows] {dr, row id}
  static constexpr int kCsq = kStat2 + 2 * kRT * 8;      // [2 slots][NC] |c|^2 (inf: padding)
  static constexpr int kCy = kCsq + 2 * NC * 4;          // [2 slots][NC] |c|
  static constexpr int kCred = kCy + 2 * NC * 4;         // [2 slots][8 waves][4] segment maxima
  static constexpr int kCid = kCred + 2 * 8 * 16;        // [2 slots][NC] global centre id of list position
  static constexpr int kClid = kCid + 2 * NC * 4;        // [2 slots][NC] local id reported for it
  static constexpr int kEX = NCW + 1;                    // exchange row stride in float4 (padded: conflict-free)
  static constexpr int kExch = kClid + 2 * NC * 4;       // [2 bufs][32 rows][kEX] float4 per-wave row summaries
  static constexpr int kXacc = kExch + 2 * kRT * kEX * 16;  // T3: [4 waves][4][64 lanes] float4 (vh.cl)
  static constexpr int kRes = kXacc + (T3 ? 4 * 4 * 64 * 16 : 0);  // [RL rows] residual centres
  static constexpr int kBytes = kRes + RL * kRD * 4;
  static_assert(kBytes <= 160 * 1024, "LDS budget");
};

struct ResSeg {  // wave-uniform
  int s, cnt, cbase, ca, cb, pen;  // pen: 0, 2 (penalty segment), 3 (no candidates): work item n = -pen
};

__device__ __forceinline__ ResSeg res_seg(const AssignParams& p, int s) {
  ResSeg g;
  g.s = s;
  g.cnt = runi(p.cand_count[s]);
  g.cbase = runi(p.cand_base[s]);
  const bool flag = p.seg_flags && (runi(p.seg_flags[s]) & RQSID_SEG_PENALTY);
  g.pen = flag ? 2 : (g.cnt <= 0 ? 3 : 0);
  g.ca = p.seg_ca ? runi(p.seg_ca[s]) : s;
  g.cb = p.seg_cb ? runi(p.seg_cb[s]) : s;
  return g;
}

// one k-step of the MFMA loop as a schedule group: N fragment reads then N MFMAs, so hipcc cannot
// hoist all 32 steps' reads ahead of the MFMAs (128 extra VGPRs beside the resident centres)
#define RQ_PAIR(N)                                   \
  do {                                               \
    __builtin_amdgcn_sched_group_barrier(0x100, N, 0); \
    __builtin_amdgcn_sched_group_barrier(0x008, N, 0); \
  } while (0)

__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// wave sums of four rows' per-lane partials: lanes 16r .. 16r+15 end with the total of row r
template <typename T>
__device__ __forceinline__ T red4(const T (&v)[4], int lane) {
  const bool b5 = lane & 32, b4 = lane & 16;
  const T t0 = (b5 ? v[2] : v[0]) + __shfl_xor(b5 ? v[0] : v[2], 32);
  const T t1 = (b5 ? v[3] : v[1]) + __shfl_xor(b5 ? v[1] : v[3], 32);
  T t = (b4 ? t1 : t0) + __shfl_xor(b4 ? t0 : t1, 16);
  t += __shfl_xor(t, 8);
  t += __shfl_xor(t, 4);
  t += __shfl_xor(t, 2);
  t += __shfl_xor(t, 1);
  return t;
}

template <int RL, bool NORM, bool T3>
__global__ __launch_bounds__(512, 1) void assign_resident_kernel(AssignParams p, const int4* __restrict__ desc,
                                                                 const int32_t* __restrict__ seg_tile32,
                                                                 int32_t* __restrict__ seg_of_row) {
  using L = ResLayout<T3, RL>;
  constexpr int NCW = L::NCW;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  // FP16 (and FP64) denormals flushed: no subnormal operand reaches the MFMA (to_f16, assign.hip)
  asm volatile("s_setreg_imm32_b32 hwreg(HW_REG_MODE, 6, 2), 0");
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = runi(tid >> 6);
  const int h = lane >> 5, n = lane & 31;
  const int cw = T3 ? (wave & 3) : wave;       // candidate group of this wave
  const bool lo_wave = T3 && wave >= 4;        // 3 terms: holds the lo centre terms
  const int T = runi(seg_tile32[p.n_segments]);
  const int G = gridDim.x;
  const int xb = (blockIdx.x & 7) * (G >> 3) + (blockIdx.x >> 3);  // XCD-contiguous tile runs
  const int tb = (int)((int64_t)T * xb / G), te = (int)((int64_t)T * (xb + 1) / G);
  if (tb >= te) return;

  const float tscale = __int_as_float(runi(__float_as_int(p.c_meta[4 * p.n_centers])));
  const float ar = p.acc_rel, ar2 = 2.0f * p.acc_rel;
  const float den_eps = (0.125f * (float)kRD + 3.0f) * 5.97e-8f;

  float* const st_base = reinterpret_cast<float*>(smem + L::kStat);
  float* const csq_base = reinterpret_cast<float*>(smem + L::kCsq);
  float* const cy_base = reinterpret_cast<float*>(smem + L::kCy);
  float* const cred_base = reinterpret_cast<float*>(smem + L::kCred);
  int32_t* const cid_base = reinterpret_cast<int32_t*>(smem + L::kCid);
  int32_t* const clid_base = reinterpret_cast<int32_t*>(smem + L::kClid);
  float4* const exch = reinterpret_cast<float4*>(smem + L::kExch);

  // ---- per-segment register state
  f16x8 a[kKS];                 // this wave's 32 candidates (A operand), the MFMA segment's
  auto load_centres = [&](const ResSeg& g) __attribute__((always_inline)) {
    const int m = min(32 * cw + n, g.cnt - 1);
    const int cg = cand_global(p, g.cbase, m);
    const _Float16* src = reinterpret_cast<const _Float16*>(p.c16) + (int64_t)cg * (2 * kRD) + 8 * h + (lo_wave ? 32 : 0);
#pragma unroll
    for (int ks = 0; ks < kKS; ++ks) a[ks] = *reinterpret_cast<const f16x8*>(src + (ks >> 1) * 64 + (ks & 1) * 16);
  };
  // residual centre rows of the producer segment g -> LDS (one copy: the caller barriers before the
  // producers read it, and every producer of the previous segment has passed the tile barriers)
  auto load_res_rows = [&](const ResSeg& g) __attribute__((always_inline)) {
    float4* dst = reinterpret_cast<float4*>(smem + L::kRes);
    if (RL >= 1 && tid < kRD / 4) dst[tid] = reinterpret_cast<const float4*>(p.ca + (int64_t)g.ca * kRD)[tid];
    if (RL >= 2 && tid >= kRD / 4 && tid < kRD / 2)
      dst[tid] = reinterpret_cast<const float4*>(p.cb + (int64_t)g.cb * kRD)[tid - kRD / 4];
  };
  // candidate |c|^2, |c| and the segment maxima of the collapsed bound -> LDS slot sl
  auto write_cmeta = [&](const ResSeg& g, int sl) __attribute__((always_inline)) {
    float gz = 0.f, gw = 0.f, gy = 0.f;
    if (tid < L::NC && g.cnt > 0) {
      const bool live = tid < g.cnt;
      const int kl = live ? tid : g.cnt - 1;
      const float4 m = reinterpret_cast<const float4*>(p.c_meta)[cand_global(p, g.cbase, kl)];
      csq_base[sl * L::NC + tid] = live ? m.x : INFINITY;
      cy_base[sl * L::NC + tid] = m.y;
      cid_base[sl * L::NC + tid] = cand_global(p, g.cbase, kl);
      clid_base[sl * L::NC + tid] = cand_local(p, g.cbase, kl);
      gz = ratio_up(T3 ? m.z : m.w, m.y);
      gw = T3 ? ratio_up(m.w, m.y) : 0.f;
      gy = m.y;
    }
    gz = wave_max(gz);
    gw = wave_max(gw);
    gy = wave_max(gy);
    if (lane == 0) {
      cred_base[(sl * 8 + wave) * 4 + 0] = gz;
      cred_base[(sl * 8 + wave) * 4 + 1] = gw;
      cred_base[(sl * 8 + wave) * 4 + 2] = gy;
    }
  };

  // ---- row pipeline: R = the 4 rows (this wave's tile rows 4w..4w+3) of the next tile to produce
  typedef __attribute__((ext_vector_type(4))) float f4v;
  f4v R[4][2];
  float dvr[4] = {1.f, 1.f, 1.f, 1.f};  // RL 2 NORM: den_in of the R rows
  int rrow[4] = {0, 0, 0, 0};           // row ids of the R rows (wave-uniform)
  int prow[4] = {0, 0, 0, 0};           // row ids of the rows being produced
  // descriptors travel the pipeline as loaded (VGPRs) and become wave-uniform (readfirstlane) only
  // where used, iterations later: a readfirstlane at the load would wait for it, and with it for every
  // row load in flight
  auto desc_of = [&](int t) __attribute__((always_inline)) { return desc[t]; };
  auto U4 = [&](const int4& d) __attribute__((always_inline)) { return make_int4(runi(d.x), runi(d.y), runi(d.z), 0); };
  auto load_rids = [&](const int4& d) __attribute__((always_inline)) {  // lanes: row id of tile row 4w + (lane & 3)
    const int pos = d.y + min(4 * wave + (lane & 3), d.z - 1);
    return p.row_index ? p.row_index[pos] : pos;
  };
  // R[r] <- row r of tile d (its id in lane r of rid)
  // Unconditional: padding rows load the tile's last row (load_rids clamps) and the pipeline runs past
  // the block's last tile on clamped descriptors, so every iteration issues the same loads in the same
  // order and hipcc's counted waits stay exact (a conditional load makes it wait for vmcnt(0)).
  auto issue_row = [&](int rid, int r) __attribute__((always_inline)) {
    rrow[r] = __builtin_amdgcn_readlane(rid, r);
    const f4v* xr = reinterpret_cast<const f4v*>(p.x + (int64_t)rrow[r] * kRD);
    R[r][0] = __builtin_nontemporal_load(xr + lane);
    R[r][1] = __builtin_nontemporal_load(xr + 64 + lane);
    if (RL >= 2 && NORM) dvr[r] = p.den_in[rrow[r]];
  };

  // produce row r of the next tile from R[r] into image buffer bf: the reference's residual chain in
  // fp32, fp16 rounding (+ the second term), the per-lane partial sums of the bound's statistics
  float s_ex[4], s_el[4], s_v[4];
  double s_v64[4];
  auto produce_row = [&](int r, int bf) __attribute__((always_inline)) {
    unsigned char* img = smem + bf * L::kBuf;
    const int tr = 4 * wave + r;  // tile row
    prow[r] = rrow[r];
    float inv1 = 1.0f;
    if (RL >= 2 && NORM) inv1 = 1.0f / dvr[r];
    float v[8] = {R[r][0].x, R[r][0].y, R[r][0].z, R[r][0].w, R[r][1].x, R[r][1].y, R[r][1].z, R[r][1].w};
    const float4* res = reinterpret_cast<const float4*>(smem + L::kRes);
    if (RL >= 1) {
      const float4 caA = res[lane], caB = res[64 + lane];
      const float c[8] = {caA.x, caA.y, caA.z, caA.w, caB.x, caB.y, caB.z, caB.w};
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = v[e] - c[e];
    }
    if (RL >= 2) {
      const float4 cbA = res[kRD / 4 + lane], cbB = res[kRD / 4 + 64 + lane];
      const float c[8] = {cbA.x, cbA.y, cbA.z, cbA.w, cbB.x, cbB.y, cbB.z, cbB.w};
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = (NORM ? v[e] * inv1 : v[e]) - c[e];
    }
    h2 hh[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) hh[e] = __builtin_convertvector(f2{v[2 * e], v[2 * e + 1]}, h2);
    float ex[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) ex[e] = (e & 1) ? sub_f16<1>(v[e], hh[e >> 1]) : sub_f16<0>(v[e], hh[e >> 1]);
    // dims 4l..4l+3 -> group kh = l/2, byte (l&1)*8; dims 256+4l.. -> group 32 + l/2
    const int o0 = img_off(lane >> 1, tr) + (lane & 1) * 8, o1 = img_off(32 + (lane >> 1), tr) + (lane & 1) * 8;
    typedef __attribute__((ext_vector_type(4))) _Float16 h4;
    *reinterpret_cast<h4*>(img + o0) = __builtin_shufflevector(hh[0], hh[1], 0, 1, 2, 3);
    *reinterpret_cast<h4*>(img + o1) = __builtin_shufflevector(hh[2], hh[3], 0, 1, 2, 3);
    float se = 0.f, sl = 0.f, sv = 0.f;
    double sv64 = 0.0;
    if (T3) {
      h2 lh[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) lh[e] = __builtin_convertvector(f2{ex[2 * e] * 4096.0f, ex[2 * e + 1] * 4096.0f}, h2);
      *reinterpret_cast<h4*>(img + kImg + o0) = __builtin_shufflevector(lh[0], lh[1], 0, 1, 2, 3);
      *reinterpret_cast<h4*>(img + kImg + o1) = __builtin_shufflevector(lh[2], lh[3], 0, 1, 2, 3);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float ev = fmaf(ex[e], 4096.0f, -(float)lh[e >> 1][e & 1]);  // exact
        sl = fmaf(ev, ev, sl);
      }
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      se = fmaf(ex[e], ex[e], se);
      if (fp64_norm(RL, NORM)) sv64 = fma((double)v[e], (double)v[e], sv64);
      else sv = fmaf(v[e], v[e], sv);
    }
    s_ex[r] = se;
    s_el[r] = sl;
    s_v[r] = sv;
    s_v64[r] = sv64;
  };
  // wave totals of the four produced rows -> row statistics of tile d in buffer bf (+ den_out)
  auto finish_rows = [&](const int4& d, int bf, bool live) __attribute__((always_inline)) {
    const float e2 = red4(s_ex, lane);
    const float l2 = T3 ? red4(s_el, lane) : 0.f;
    float nrm;
    if (fp64_norm(RL, NORM)) nrm = (float)sqrt(red4(s_v64, lane));
    else nrm = sqrtf(red4(s_v, lane));
    if ((lane & 15) == 0) {
      const int r = lane >> 4;
      const int tr = 4 * wave + r;
      const bool valid = live && tr < d.z;
      const int row = r == 0 ? prow[0] : (r == 1 ? prow[1] : (r == 2 ? prow[2] : prow[3]));
      const float en = sqrtf(e2) * 1.001f + 1e-30f;
      const float en2 = T3 ? sqrtf(l2) * (1.001f / 4096.0f) + 1e-30f : 0.f;
      float inv_den = 1.f, dr = 0.f;
      if (NORM && RL >= 1) {
        const float den = nrm + 1e-8f;
        inv_den = 1.0f / den;
        if (RL == 1 && valid && p.den_out) p.den_out[row] = den;
        dr = RL == 1 ? 2.0f * 5.97e-8f
                     : (4.0f * 2.39e-7f * (1.0f + nrm) * inv_den + 4.0f * 5.97e-8f + 1.01f * den_eps * nrm * inv_den);
      }
      const float vn = nrm * 1.0001f + 1e-30f;
      reinterpret_cast<float4*>(smem + L::kStat)[bf * kRT + tr] = make_float4(en, en2, vn, inv_den);
      reinterpret_cast<float2*>(smem + L::kStat2)[bf * kRT + tr] = make_float2(dr, __int_as_float(valid ? row : -1));
    }
  };

  // ---- prologue: tile tb produced into buffer 0, tile tb+1's rows in flight, centres of tile tb loaded
  int4 d0 = U4(desc_of(tb));
  ResSeg g0 = res_seg(p, d0.x);
  int slot0 = 0;
  int4 d1 = U4(desc_of(min(tb + 1, te - 1)));
  int4 d2 = U4(desc_of(min(tb + 2, te - 1)));
  int4 d3raw = desc_of(min(tb + 3, te - 1));
  {
    const int rid0 = load_rids(d0);
    load_res_rows(g0);
    lds_barrier();
#pragma unroll
    for (int r = 0; r < 4; ++r) issue_row(rid0, r);
    write_cmeta(g0, 0);
#pragma unroll
    for (int r = 0; r < 4; ++r) produce_row(r, 0);
    finish_rows(d0, 0, true);
  }
  {
    const int rid1 = load_rids(d1);
#pragma unroll
    for (int r = 0; r < 4; ++r) issue_row(rid1, r);
  }
  int rid2 = load_rids(d2);
  if (g0.cnt > 0) load_centres(g0);
#pragma unroll
  for (int ks = 0; ks < kKS; ++ks) asm volatile("" : "+v"(a[ks]));  // complete before the loop (see its end)
  lds_barrier();

  // Waves 0-3 produce their rows of tile j+1 before multiplying tile j, waves 4-7 after: on every SIMD
  // one wave's VALU work runs beside the other's MFMAs.  (One loop body for both roles, a wave-uniform
  // guard per phase: two loop instances in one kernel exhaust hipcc's register allocation.)
  RS(uint32_t rs_acc[16] = {}; uint32_t rs_t = RS_NOW(); const uint32_t rs_0 = rs_t;)
#define RS_MARK(k) RS({ const uint32_t t_ = RS_NOW(); rs_acc[k] += t_ - rs_t; rs_t = t_; })
  for (int j = tb; j < te; ++j) {
    RS(rs_acc[7] += 1;)
    const int b = (j - tb) & 1;
    const bool has1 = j + 1 < te;
    // segment of the tile to produce
    ResSeg g1 = g0;
    int slot1 = slot0;
    const bool newseg = has1 && d1.x != d0.x;
    if (newseg) {
      g1 = res_seg(p, d1.x);
      slot1 = slot0 ^ 1;
      load_res_rows(g1);
      write_cmeta(g1, slot1);
      lds_barrier();  // (rare: segment changes) the rows are read by every wave's producer below
    }
    RS_MARK(1);
    // Tile j's MFMAs interleaved with producing this wave's four rows of tile j+1 (and re-filling their R
    // registers with tile j+2) in ONE straight-line block: the matrix pipe runs under the producer's
    // VALU / LDS work of the same wave, and the fragment reads have the producer's work to hide behind.
    f32x16 acc = {}, accl = {};
    const unsigned char* ib = smem + b * L::kBuf + img_off(h, n);  // + 2 kGS per k-step
    const unsigned char* il = ib + kImg;
    // B fragments are read RQ_PF k-steps ahead of their MFMA (an LDS round trip is several MFMA issue
    // slots; a read issued just before its MFMA stalls the chain)
    auto fused = [&](auto lo_tag) __attribute__((always_inline)) {
      constexpr bool LO = decltype(lo_tag)::value;
      constexpr bool TWO = T3 && !LO;  // vh and vl fragments
      f16x8 fb[RQ_PF], fl[TWO ? RQ_PF : 1];
#pragma unroll
      for (int i = 0; i < RQ_PF; ++i) {
        fb[i] = *reinterpret_cast<const f16x8*>(ib + 2 * kGS * i);
        if (TWO) fl[i] = *reinterpret_cast<const f16x8*>(il + 2 * kGS * i);
      }
#pragma unroll
      for (int ks = 0; ks < kKS; ++ks) {
        const f16x8 bf = fb[ks % RQ_PF];
        const f16x8 bl = fl[TWO ? ks % RQ_PF : 0];
        if (ks + RQ_PF < kKS) {
          fb[ks % RQ_PF] = *reinterpret_cast<const f16x8*>(ib + 2 * kGS * (ks + RQ_PF));
          if (TWO) fl[ks % RQ_PF] = *reinterpret_cast<const f16x8*>(il + 2 * kGS * (ks + RQ_PF));
        }
        if (LO) {
          accl = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[ks], bf, accl, 0, 0, 0);
        } else {
          acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[ks], bf, acc, 0, 0, 0);
          if (T3) accl = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[ks], bl, accl, 0, 0, 0);
        }
        if (ks % (kKS / 4) == kKS / 4 - 1) {
          produce_row(ks / (kKS / 4), b ^ 1);
          issue_row(rid2, ks / (kKS / 4));
        }
      }
#if RQ_ILV > 0
      // interleave: every MFMA followed by RQ_ILV VALU instructions of the producer (and one fragment
      // read), so the matrix pipe runs under the producer within the wave
#pragma unroll
      for (int i = 0; i < kKS * (TWO ? 2 : 1); ++i) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x002, RQ_ILV, 0);
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      }
#endif
    };
#ifdef RQSID_STAMPS
    asm volatile("" ::"v"(R[0][0]), "v"(R[0][1]), "v"(R[1][0]), "v"(R[1][1]), "v"(R[2][0]), "v"(R[2][1]), "v"(R[3][0]), "v"(R[3][1]));
    RS_MARK(8);  // waiting for the rows of tile j+1
#endif
    if (T3 && lo_wave) fused(std::true_type{});
    else fused(std::false_type{});
    finish_rows(d1, b ^ 1, has1);
    RS_MARK(2);
    // the next segment's centres, completed in the same block: hipcc's wait counting is path-insensitive
    // and a load left pending here would put a wait before every MFMA of the common path.  The stall is
    // one L2 round trip per segment change.
    if (newseg && g1.cnt > 0) {
      load_centres(g1);
#pragma unroll
      for (int ks = 0; ks < kKS; ++ks) asm volatile("" : "+v"(a[ks]));
    }
    RS_MARK(3);
    // the pipeline behind: row ids of tile j+3, descriptor of tile j+4 (clamped to the last tile)
    const int4 d3 = U4(d3raw);  // loaded an iteration ago
    rid2 = load_rids(d3);
    const int4 d4raw = desc_of(min(j + 4, te - 1));

    // ---- epilogue of tile j (segment g0, statistics buffer b, candidate meta slot0)
    if (T3) {  // waves 4-7 hand their vh.cl sums to waves 0-3
      float4* xa = reinterpret_cast<float4*>(smem + L::kXacc) + cw * 4 * 64 + lane;
      if (lo_wave) {
#pragma unroll
        for (int g = 0; g < 4; ++g) xa[g * 64] = make_float4(accl[4 * g], accl[4 * g + 1], accl[4 * g + 2], accl[4 * g + 3]);
      }
      lds_barrier();
      if (!lo_wave) {
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const float4 o = xa[g * 64];
          accl[4 * g] += o.x;
          accl[4 * g + 1] += o.y;
          accl[4 * g + 2] += o.z;
          accl[4 * g + 3] += o.w;
        }
      }
    }
    // One exchange per tile.  Each candidate wave posts, per row, a summary of its 32 candidates: U_w
    // (least upper bound), the lower bound of the candidate attaining it and L_w (least lower bound of
    // the others).  With U = min_w U_w the row is definitive iff exactly one candidate has lb < U' (the
    // pass rule of assign.hip), i.e. no L_w passes and exactly one of the posted lower bounds does;
    // that candidate's wave writes the ID.  Other rows get every wave's pass mask in work[row] (the
    // expand pass turns them into work items for the fp64 re-score).
    int row_id = -1, my_cid = 0, my_clid = 0;
    if (!lo_wave) {
      const float4 s0 = reinterpret_cast<const float4*>(smem + L::kStat)[b * kRT + n];
      const float2 s1 = reinterpret_cast<const float2*>(smem + L::kStat2)[b * kRT + n];
      row_id = __float_as_int(s1.y);
      const float en = s0.x, en2 = s0.y, vn = s0.z, inv_den = s0.w, dr = s1.x;
      const float hn = vn + en;       // >= |vh|
      const float vr = vn * inv_den;  // |r| of the row being assigned
      const float k2 = 2.0f * inv_den * 1.000001f;
      const float A = T3 ? k2 * (en2 + ar * hn + ar2 * (en + en2)) + 2.0f * dr + 7.2e-7f * vr
                         : k2 * (en + ar * hn) + 2.0f * dr + 4.8e-7f * vr;
      const float B = T3 ? k2 * (hn * (1.0f + ar2) + 2.0f * (en + en2)) : k2 * hn * (1.0f + ar);
      const float C = T3 ? k2 * ((en + en2) + ar * hn + ar2 * (hn + en + en2)) : 0.0f;
      const float m2 = -2.0f * inv_den * tscale;
      float gz = 0.f, gw = 0.f, gy = 0.f;
#pragma unroll
      for (int w = 0; w < L::NC / 64; ++w) {
        const float4 c = reinterpret_cast<const float4*>(cred_base)[slot0 * 8 + w];
        gz = fmaxf(gz, c.x);
        gw = fmaxf(gw, c.y);
        gy = fmaxf(gy, c.z);
      }
      const float A2 = (A + B * gz + C * gw + 2.39e-7f * gy) * 1.000001f;
      const float* csq = csq_base + slot0 * L::NC + 32 * cw + 4 * h;
      const float* cy = cy_base + slot0 * L::NC + 32 * cw + 4 * h;
      float U = INFINITY, lbk = INFINITY, Lo = INFINITY;
      int kv = 0;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        __builtin_amdgcn_sched_barrier(0);  // one group's meta at a time (register pressure)
        const float4 cs = *reinterpret_cast<const float4*>(csq + 8 * g);
        const float4 yy = *reinterpret_cast<const float4*>(cy + 8 * g);
        const float csv[4] = {cs.x, cs.y, cs.z, cs.w}, yv[4] = {yy.x, yy.y, yy.z, yy.w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int v = 4 * g + e;
          const float dd = T3 ? fmaf(0x1p-12f, accl[v], acc[v]) : acc[v];
          const float P = fmaf(m2, dd, csv[e]);
          const float E = fmaf(A2, yv[e], 1e-30f);
          const float ub = P + E, lb = P - E;
          const bool nm = ub < U;
          Lo = fminf(Lo, nm ? lbk : lb);
          lbk = nm ? lb : lbk;
          kv = nm ? v : kv;
          U = nm ? ub : U;
          acc[v] = lb;  // kept for the pass masks of an ambiguous row
        }
      }
      // combine the two lane halves of the row (16 candidates each)
      int kpos = 32 * cw + (kv & 3) + 8 * (kv >> 2) + 4 * h;
      const float oU = __shfl_xor(U, 32), olb = __shfl_xor(lbk, 32), oL = __shfl_xor(Lo, 32);
      const int ok = __shfl_xor(kpos, 32);
      const bool take = oU < U || (oU == U && ok < kpos);
      Lo = take ? fminf(fminf(Lo, lbk), oL) : fminf(fminf(Lo, olb), oL);
      lbk = take ? olb : lbk;
      kpos = take ? ok : kpos;
      U = take ? oU : U;
      if (h == 0) exch[(b * kRT + n) * L::kEX + cw] = make_float4(U, lbk, Lo, 0.f);
      // this wave's candidate ids, read before the barrier: after it a faster wave may rewrite the slot
      my_cid = cid_base[slot0 * L::NC + kpos];
      my_clid = clid_base[slot0 * L::NC + kpos];
    }
    RS_MARK(9);  // epilogue 1 compute
    lds_barrier();
    RS_MARK(4);
    if (!lo_wave) {
      float U = INFINITY;
#pragma unroll
      for (int w = 0; w < NCW; ++w) U = fminf(U, exch[(b * kRT + n) * L::kEX + w].x);
      // pass: lb < Up, Up above U by >= 2 ulp (a candidate admitted by rounding is only re-scored)
      const float Up = fmaf(fabsf(U), 0x1p-22f, U) + 1.2e-38f;
      int cnt = 0, win = 0;
      bool many = false;
#pragma unroll
      for (int w = 0; w < NCW; ++w) {
        const float4 e = exch[(b * kRT + n) * L::kEX + w];
        const bool pk = (__float_as_uint(e.y - Up) >> 31) != 0;
        cnt += pk ? 1 : 0;
        win = pk ? w : win;
        many = many || (__float_as_uint(e.z - Up) >> 31) != 0;
      }
      const bool valid = row_id >= 0;
      const bool definitive = !g0.pen && !many && cnt == 1;
#ifndef RQ_AB_NOSTORE
      if (h == 0 && valid && definitive && win == cw) {
        p.out_local[row_id] = my_clid;
        p.out_global[row_id] = my_cid;
      }
#endif
      // ambiguous rows (a few per cent): every candidate wave stores its pass mask in work[row]
      // (word cw); wave 0 marks the row (sentinel -2, segment in seg_of_row, ~segment for a row of
      // a penalty / empty segment).  Behind a wave-uniform branch: the common tile skips it.
      const bool amb = valid && !definitive;
      if (__builtin_amdgcn_ballot_w64(amb)) {
        uint32_t mk = 0;
#pragma unroll
        for (int v = 0; v < 16; ++v) mk |= (__float_as_uint(acc[v] - Up) >> 31) << ((v & 3) + 8 * (v >> 2) + 4 * h);
        mk |= __shfl_xor(mk, 32);
        if (h == 0 && amb) {
          reinterpret_cast<uint32_t*>(p.work + row_id)[cw] = mk;
          if (cw == 0) {
            p.out_global[row_id] = -2;
            seg_of_row[row_id] = g0.pen ? ~g0.s : g0.s;
          }
        }
      }
    }
    RS_MARK(5);
    // rotate the pipeline
    d0 = d1;
    d1 = d2;
    d2 = d3;
    d3raw = d4raw;
    g0 = g1;
    slot0 = slot1;
    RS_MARK(6);
  }
#ifdef RQSID_STAMPS
  if (lane == 0 && (wave == 0 || wave == 4)) {
    rs_acc[0] = RS_NOW() - rs_0;
    for (int k = 0; k < 16; ++k) atomicAdd(&g_rstamps[(wave >> 2) * 16 + k], (unsigned long long)rs_acc[k]);
  }
#endif
#undef RS_MARK
}

// 32-row tiling of the segments: seg_tile32[s] = sum_{s' < s} ceil(rows(s') / 32) (one block)
__global__ __launch_bounds__(1024) void res_tiles_kernel(const int32_t* __restrict__ seg_row_off, int nseg,
                                                         int32_t* __restrict__ seg_tile32) {
  __shared__ int part[1024];
  const int tid = threadIdx.x;
  const int per = (nseg + 1023) / 1024, s0 = min(nseg, tid * per), s1 = min(nseg, s0 + per);
  int sum = 0;
  for (int s = s0; s < s1; ++s) sum += (seg_row_off[s + 1] - seg_row_off[s] + kRT - 1) / kRT;
  part[tid] = sum;
  __syncthreads();
  for (int o = 1; o < 1024; o <<= 1) {  // inclusive Hillis-Steele scan
    const int v = tid >= o ? part[tid - o] : 0;
    __syncthreads();
    part[tid] += v;
    __syncthreads();
  }
  int run = part[tid] - sum;
  for (int s = s0; s < s1; ++s) {
    seg_tile32[s] = run;
    run += (seg_row_off[s + 1] - seg_row_off[s] + kRT - 1) / kRT;
  }
  if (tid == 1023) seg_tile32[nseg] = part[1023];
}

// tile descriptors {segment, first row position, rows} (one thread per tile)
__global__ __launch_bounds__(256) void res_desc_kernel(const int32_t* __restrict__ seg_row_off,
                                                       const int32_t* __restrict__ seg_tile32, int nseg, int64_t cap,
                                                       int4* __restrict__ desc) {
  const int ntiles = seg_tile32[nseg];
  for (int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x; t < ntiles && t < cap; t += (int64_t)gridDim.x * 256) {
    int lo = 0, hi = nseg;  // last segment whose first tile is <= t (skips empty segments)
    while (hi - lo > 1) {
      const int mid = (lo + hi) >> 1;
      if (seg_tile32[mid] <= t) lo = mid; else hi = mid;
    }
    const int t0 = seg_row_off[lo] + ((int)t - seg_tile32[lo]) * kRT;
    desc[t] = make_int4(lo, t0, min(kRT, seg_row_off[lo + 1] - t0), 0);
  }
}

struct DevState {
  int ncu = 0;
  bool attr[2][3][2] = {};  // [T3][RL][NORM]
};
DevState g_dev[64];

template <int RL, bool NORM, bool T3>
int launch_res(const AssignParams& p, const int4* desc, const int32_t* seg_tile32, int32_t* seg_of_row, hipStream_t st) {
  using L = ResLayout<T3, RL>;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return fail(RQSID_E_LAUNCH, "assign: hipGetDevice");
  DevState& ds = g_dev[dev];
  if (!ds.ncu) {
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, dev) != hipSuccess) return fail(RQSID_E_LAUNCH, "assign: device properties");
    ds.ncu = prop.multiProcessorCount;
  }
  const void* k = (const void*)assign_resident_kernel<RL, NORM, T3>;
  if (!ds.attr[T3][RL][NORM]) {
    if (hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, L::kBytes) != hipSuccess)
      return fail(RQSID_E_LAUNCH, "assign: cannot raise the dynamic LDS limit (resident screen)");
    ds.attr[T3][RL][NORM] = true;
  }
  const unsigned g = (unsigned)(ds.ncu >= 8 ? ds.ncu / 8 * 8 : 8);  // one persistent block per CU
  hipLaunchKernelGGL((assign_resident_kernel<RL, NORM, T3>), dim3(g), dim3(512), L::kBytes, st, p, desc, seg_tile32,
                     seg_of_row);
  return check_launch("assign_resident");
}

// Ambiguous rows of the resident screen -> work items for assign_rescore_kernel (after the sentinel
// compaction listed them): work[row] holds one pass-mask word per candidate wave (bit j of word q =
// list position 32 q + j); seg_of_row[row] the segment (~segment for a penalty / empty segment).
__global__ __launch_bounds__(256) void res_expand_kernel(AssignParams p, const int32_t* __restrict__ seg_of_row,
                                                         int ncw) {
  const int64_t cnt_raw = *p.work_count;
  const int64_t cnt = cnt_raw < p.work_cap ? cnt_raw : p.work_cap;
  for (int64_t it = (int64_t)blockIdx.x * 256 + threadIdx.x; it < cnt; it += (int64_t)gridDim.x * 256) {
    const int row = p.work_idx[it];
    const int s = seg_of_row[row];
    WorkItem w{};
    w.row = row;
#pragma unroll
    for (int k = 0; k < kMaxList; ++k) w.cand[k] = 0xFFFF;
    if (s < 0) {
      w.seg = ~s;
      const bool flag = p.seg_flags && (p.seg_flags[~s] & RQSID_SEG_PENALTY);
      w.n = flag ? -2 : -3;
    } else {
      w.seg = s;
      const uint32_t* mw = reinterpret_cast<const uint32_t*>(p.work + row);
      uint32_t m[8];
      int tot = 0;
      for (int q = 0; q < 8; ++q) {
        m[q] = q < ncw ? mw[q] : 0u;
        tot += __popc(m[q]);
      }
      if (tot >= 1 && tot <= kMaxList) {
        w.n = tot;
        int c = 0;
        for (int q = 0; q < 8; ++q) {
          uint32_t x = m[q];
          while (x) {
            w.cand[c++] = (uint16_t)(32 * q + __ffs(x) - 1);
            x &= x - 1;
          }
        }
      } else {
        w.n = -1;  // more than kMaxList pass (or none: a NaN distance): every candidate
      }
    }
    p.work[row] = w;
  }
}

}  // namespace

void launch_resident_expand(const AssignParams& p, const int32_t* seg_of_row, bool t3, int64_t n_rows, hipStream_t st) {
  hipLaunchKernelGGL(res_expand_kernel, dim3(grid_cap(cdiv(n_rows, 256), 2048)), dim3(256), 0, st, p, seg_of_row,
                     t3 ? ResLayout<true, 0>::NCW : ResLayout<false, 0>::NCW);
}

bool resident_supported(int dim, int cand_count_max, bool t3, int rl) {
  // one fp16 term only: the 3-term form (hi / lo centre waves) does not fit the LDS budget and
  // registers beside the one-exchange epilogue (the per-tile screen serves those levels)
  (void)rl;
  return dim == kRD && cand_count_max >= 1 && cand_count_max <= 256 && !t3;
}

int64_t resident_desc_bytes(int64_t n_rows) { return (n_rows > 0 ? n_rows : 0) * (int64_t)sizeof(int4); }

int launch_resident_screen(const AssignParams& p, bool t3, int rl, bool norm, int4* desc, int32_t* seg_tile32,
                           int32_t* seg_of_row, int64_t cap, hipStream_t st) {
  hipLaunchKernelGGL(res_tiles_kernel, dim3(1), dim3(1024), 0, st, p.seg_row_off, p.n_segments, seg_tile32);
  hipLaunchKernelGGL(res_desc_kernel, dim3(grid_cap(cdiv(cap, 256), 4096)), dim3(256), 0, st, p.seg_row_off, seg_tile32,
                     p.n_segments, cap, desc);
  int rc = check_launch("assign_resident tiles");
  if (rc) return rc;
#define RQ_R(RL, NORM, T3) return launch_res<RL, NORM, T3>(p, desc, seg_tile32, seg_of_row, st)
  if (t3) return fail(RQSID_E_ARG, "assign: the resident screen has no 3-term form");
  if (rl == 0) RQ_R(0, false, false);
  if (rl == 1) { if (norm) RQ_R(1, true, false); RQ_R(1, false, false); }
  if (norm) RQ_R(2, true, false);
  RQ_R(2, false, false);
#undef RQ_R
}

}  // namespace rqsid

#ifdef RQSID_STAMPS
extern "C" int rqsid_debug_stamps_res(unsigned long long* out16) {
  if (hipMemcpyFromSymbol(out16, HIP_SYMBOL(g_rstamps), 32 * sizeof(unsigned long long)) != hipSuccess) return -1;
  unsigned long long z[32] = {};
  return hipMemcpyToSymbol(HIP_SYMBOL(g_rstamps), z, sizeof(z)) == hipSuccess ? 0 : -1;
}
#endif
