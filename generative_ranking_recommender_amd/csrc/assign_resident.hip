// assign_resident.hip — the centre-resident, warp-specialised screen: rqsid_assign's path for 512-d rows
// whose segments hold <= 256 candidates, one fp16 term (RQSID_SCREEN_VARIANT=6).
//
// Same arithmetic as assign.hip's single-pass screen (fp16 MFMA X·Cᵀ with a rigorous per-candidate
// error bound, the exact fp64 re-score of ambiguous rows), different data movement.  The per-tile
// kernel re-streams a segment's candidate centres through LDS for every row tile; here they stay in
// registers, and the block is split by role so that HBM waits never stall the matrix pipe:
//  * One persistent 12-wave block per CU walks an XCD-contiguous run of 32-row tiles (a segment's
//    tiles are consecutive, so the block meets each segment once).
//  * Waves 0-7 (candidate waves) hold 32 candidates each as the MFMA A operand for the whole segment
//    (32 k-steps x f16x8 = 128 VGPRs per lane; 8 x 32 = 256 candidates), multiply tile j and run its
//    bound epilogue.  They issue no row loads.
//  * Waves 8-11 (producer waves) own 8 rows of every tile: they load the rows of tile j+2 (fp32, two
//    coalesced 1-KiB loads per row, non-temporal) while producing tile j+1 from registers: the
//    reference's residual chain in fp32, fp16 rounding, the MFMA B-operand image in LDS (double
//    buffered; padded groups: conflict-free writes and fragment reads), the bound's row statistics.
//    They also prepare segments ahead of use: the tile-info ring (segment, candidates, LDS slot), the
//    residual centre rows (two tiles ahead) and the candidates' |c|^2, |c|, ids and collapsed-bound
//    maxima (one tile ahead), from dependent global loads the candidate waves never wait on.
//  * One barrier per tile.  Epilogue: each candidate wave posts per row {least upper bound, lower
//    bound of the candidate attaining it, least lower bound of the others}; after the barrier the row
//    is definitive iff no other lower bound passes (the owning wave writes the ID); ambiguous rows
//    store one pass-mask word per wave in work[row] for res_expand_kernel and the fp64 re-score.
// Segment changes reload the candidate waves' centre registers right after their last MFMA of the old
// segment (one L2 round trip per change).
#include "assign_common.h"

#ifdef RQSID_STAMPS
// diagnostic build: per role (candidate wave 0, producer wave 8) cycles of
// {loop, -, produce / mfma, reload, epilogue 1, barrier, epilogue 2, tiles, -, ...}
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
constexpr int kRD = 512;                 // row width of this kernel
constexpr int kRT = 32;                  // rows per tile (the MFMA's N)
constexpr int kKS = kRD / 16;            // k-steps of v_mfma_f32_32x32x16_f16
constexpr int kGS = (kRT + 1) * 16;      // bytes per eight-dim group: 32 rows x 16 B + 16 B pad
constexpr int kImg = kRD / 8 * kGS;      // one fp16 image: 64 eight-dim groups (33 KiB)
constexpr int kCW = 8;                   // candidate waves
constexpr int kPW = 4;                   // producer waves
constexpr int kRPW = kRT / kPW;          // rows per producer wave per tile
constexpr int kThreads = (kCW + kPW) * 64;
constexpr int kNC = kCW * 32;            // candidate capacity
#ifndef RQ_PFT
#define RQ_PFT 1  // L2 prefetch of the rows one tile ahead of their register loads
#endif
#ifndef RQ_LA
#define RQ_LA 4  // k-steps of the centres kept in LDS (wave-private) instead of registers
#endif
constexpr int kLA = RQ_LA;
constexpr int kKR = kKS - kLA;           // k-steps held in registers

__device__ __forceinline__ int runi(int v) { return __builtin_amdgcn_readfirstlane(v); }

// image slot of eight-dim group kh (= dims 8kh .. 8kh+7) of tile row n.  The 16-B pad per group
// shifts consecutive groups by 4 banks, so a producer write (fixed n, kh = lane/2: 8 groups per
// 16-lane group) is conflict-free, a fragment read (fixed kh per half-wave, n = 0..31) is 512
// contiguous bytes, and a lane's reads over the k-steps are one base + immediate offsets
__device__ __forceinline__ int img_off(int kh, int n) { return kh * kGS + n * 16; }

template <int RL>
struct ResLayout {
  static constexpr int kStat = 2 * kImg;                 // [2 bufs][32 rows] float4 {m2, A2, row id, -}
  static constexpr int kCsq = kStat + 2 * kRT * 16;      // [2 slots][kNC] |c|^2 (inf: padding)
  static constexpr int kCy = kCsq + 2 * kNC * 4;         // [2 slots][kNC] |c|
  static constexpr int kCid = kCy + 2 * kNC * 4;         // [2 slots][kNC] global centre id of list position
  static constexpr int kClid = kCid + 2 * kNC * 4;       // [2 slots][kNC] local id reported for it
  static constexpr int kEX = kCW + 1;                    // exchange row stride in float4 (padded: conflict-free)
  static constexpr int kExch = kClid + 2 * kNC * 4;      // [2 bufs][32 rows][kEX] float4 per-wave row summaries
  static constexpr int kInfo = kExch + 2 * kRT * kEX * 16;  // [4 tiles][8] int tile-info ring
  static constexpr int kAL = kInfo + 4 * 8 * 4;          // [kCW waves][kLA k-steps][64 lanes] f16x8 centre fragments
  static constexpr int kRes = kAL + kCW * kLA * 64 * 16; // [2 slots][RL rows] residual centre rows
  static constexpr int kBytes = kRes + 2 * RL * kRD * 4;
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

// Loads completed inside their asm statement (s_waitcnt vmcnt(0) there).  The compiler's wait counting
// does not see them: the producers' rare segment preparation, written with these, leaves the loop
// without conditional vector loads, whose path-insensitive counting would otherwise put a full drain
// of the row stream in every iteration.  (The drain here happens on segment changes only.)
__device__ __forceinline__ void ld4_sync(int (&v)[4], const int32_t* a0, const int32_t* a1, const int32_t* a2,
                                         const int32_t* a3) {
  asm volatile(
      "global_load_dword %0, %4, off\n\tglobal_load_dword %1, %5, off\n\t"
      "global_load_dword %2, %6, off\n\tglobal_load_dword %3, %7, off\n\ts_waitcnt vmcnt(0)"
      : "=&v"(v[0]), "=&v"(v[1]), "=&v"(v[2]), "=&v"(v[3])
      : "v"(a0), "v"(a1), "v"(a2), "v"(a3)
      : "memory");
}
__device__ __forceinline__ void ldf4x4_sync(float4 (&v)[4], const float4* a0, const float4* a1, const float4* a2,
                                            const float4* a3) {
  typedef __attribute__((ext_vector_type(4))) float f4;
  f4 t0, t1, t2, t3;
  asm volatile(
      "global_load_dwordx4 %0, %4, off\n\tglobal_load_dwordx4 %1, %5, off\n\t"
      "global_load_dwordx4 %2, %6, off\n\tglobal_load_dwordx4 %3, %7, off\n\ts_waitcnt vmcnt(0)"
      : "=&v"(t0), "=&v"(t1), "=&v"(t2), "=&v"(t3)
      : "v"(a0), "v"(a1), "v"(a2), "v"(a3)
      : "memory");
  v[0] = make_float4(t0.x, t0.y, t0.z, t0.w);
  v[1] = make_float4(t1.x, t1.y, t1.z, t1.w);
  v[2] = make_float4(t2.x, t2.y, t2.z, t2.w);
  v[3] = make_float4(t3.x, t3.y, t3.z, t3.w);
}
__device__ __forceinline__ float4 ldf4_sync(const float4* a) {
  typedef __attribute__((ext_vector_type(4))) float f4;
  f4 t;
  asm volatile("global_load_dwordx4 %0, %1, off\n\ts_waitcnt vmcnt(0)" : "=v"(t) : "v"(a) : "memory");
  return make_float4(t.x, t.y, t.z, t.w);
}

// res_seg through ld4_sync (the producers' loop)
__device__ __forceinline__ ResSeg res_seg_sync(const AssignParams& p, int s) {
  int v[4], f;
  ld4_sync(v, p.cand_count + s, p.cand_base + s, p.seg_ca ? p.seg_ca + s : p.cand_count + s,
           p.seg_cb ? p.seg_cb + s : p.cand_count + s);
  const uint8_t* fb = p.seg_flags ? p.seg_flags + s : reinterpret_cast<const uint8_t*>(p.cand_count + s);
  asm volatile("global_load_ubyte %0, %1, off\n\ts_waitcnt vmcnt(0)" : "=v"(f) : "v"(fb) : "memory");
  ResSeg g;
  g.s = s;
  g.cnt = runi(v[0]);
  g.cbase = runi(v[1]);
  const bool flag = p.seg_flags && (runi(f) & RQSID_SEG_PENALTY);
  g.pen = flag ? 2 : (g.cnt <= 0 ? 3 : 0);
  g.ca = p.seg_ca ? runi(v[2]) : s;
  g.cb = p.seg_cb ? runi(v[3]) : s;
  return g;
}

__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// wave sums of eight rows' per-lane partials: lanes with bits (b5 b4 b3) = r end with row r's total
template <typename T>
__device__ __forceinline__ T red8(const T (&v)[8], int lane) {
  const bool b5 = lane & 32, b4 = lane & 16, b3 = lane & 8;
  T t[4], u[2];
#pragma unroll
  for (int i = 0; i < 4; ++i) t[i] = (b5 ? v[i + 4] : v[i]) + __shfl_xor(b5 ? v[i] : v[i + 4], 32);
#pragma unroll
  for (int i = 0; i < 2; ++i) u[i] = (b4 ? t[i + 2] : t[i]) + __shfl_xor(b4 ? t[i] : t[i + 2], 16);
  T w = (b3 ? u[1] : u[0]) + __shfl_xor(b3 ? u[0] : u[1], 8);
  w += __shfl_xor(w, 4);
  w += __shfl_xor(w, 2);
  w += __shfl_xor(w, 1);
  return w;
}
__device__ __forceinline__ int red8_row(int lane) { return ((lane >> 3) & 1) + 2 * ((lane >> 4) & 1) + 4 * ((lane >> 5) & 1); }

// tile-info ring entry {segment, candidates, list base, pen, LDS slot}
struct TileInfo {
  int s, cnt, cbase, pen, slot;
};

template <int RL, bool NORM>
__global__ __launch_bounds__(kThreads, 1) void assign_resident_kernel(AssignParams p, const int4* __restrict__ desc,
                                                                      const int32_t* __restrict__ seg_tile32,
                                                                      int32_t* __restrict__ seg_of_row) {
  using L = ResLayout<RL>;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  // FP16 (and FP64) denormals flushed: no subnormal operand reaches the MFMA (to_f16, assign.hip)
  asm volatile("s_setreg_imm32_b32 hwreg(HW_REG_MODE, 6, 2), 0");
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = runi(tid >> 6);
  const bool producer = wave >= kCW;
  const int T = runi(seg_tile32[p.n_segments]);
  const int G = gridDim.x;
  const int xb = (blockIdx.x & 7) * (G >> 3) + (blockIdx.x >> 3);  // XCD-contiguous tile runs
  const int tb = (int)((int64_t)T * xb / G), te = (int)((int64_t)T * (xb + 1) / G);
  if (tb >= te) return;

  float* const csq_base = reinterpret_cast<float*>(smem + L::kCsq);
  float* const cy_base = reinterpret_cast<float*>(smem + L::kCy);
  int32_t* const cid_base = reinterpret_cast<int32_t*>(smem + L::kCid);
  int32_t* const clid_base = reinterpret_cast<int32_t*>(smem + L::kClid);
  float4* const exch = reinterpret_cast<float4*>(smem + L::kExch);
  int32_t* const info = reinterpret_cast<int32_t*>(smem + L::kInfo);
  auto read_info = [&](int t) __attribute__((always_inline)) {
    const int4 a = reinterpret_cast<const int4*>(info + (t & 3) * 8)[0];
    const int b = info[(t & 3) * 8 + 4];
    TileInfo r;
    r.s = runi(a.x);
    r.cnt = runi(a.y);
    r.cbase = runi(a.z);
    r.pen = runi(a.w);
    r.slot = runi(b);
    return r;
  };
  auto desc_of = [&](int t) __attribute__((always_inline)) { return desc[t]; };
  auto U4 = [&](const int4& d) __attribute__((always_inline)) { return make_int4(runi(d.x), runi(d.y), runi(d.z), 0); };
  RS(uint32_t rs_acc[16] = {}; uint32_t rs_t = RS_NOW(); const uint32_t rs_0 = rs_t;)
#define RS_MARK(k) RS({ const uint32_t t_ = RS_NOW(); rs_acc[k] += t_ - rs_t; rs_t = t_; })

  if (producer) {
    // =========================== producer waves: rows, images, statistics, segments
    const int pw = wave - kCW, pt = tid - kCW * 64;  // producer wave / thread (0..255)
    const float tscale = __int_as_float(runi(__float_as_int(p.c_meta[4 * p.n_centers])));
    const float ar = p.acc_rel;
    typedef __attribute__((ext_vector_type(4))) float f4v;
    const float den_eps = (0.125f * (float)kRD + 3.0f) * 5.97e-8f;
    f4v R[kRPW][2];
    float dvr[kRPW];
    int rrow[kRPW], prow[kRPW];
#pragma unroll
    for (int r = 0; r < kRPW; ++r) {
      dvr[r] = 1.f;
      rrow[r] = prow[r] = 0;
    }
    // lanes: id of tile row kRPW pw + (lane & 7).  The load is unconditional (without a row index it
    // reads the position array's stand-in, the descriptors): a conditional load would break the counting
    const int32_t* const ri_base = p.row_index ? p.row_index : reinterpret_cast<const int32_t*>(desc);
    auto load_rids = [&](const int4& d) __attribute__((always_inline)) {
      const int pos = d.y + min(kRPW * pw + (lane & 7), d.z - 1);
      const int v = ri_base[p.row_index ? pos : 0];
      return p.row_index ? v : pos;
    };
    // Unconditional loads (padding rows re-load the tile's last row; past the block's last tile the
    // descriptors are clamped): the same loads in the same order every iteration keep hipcc's counted
    // waits exact.
    auto issue_row = [&](int rid, int r) __attribute__((always_inline)) {
      rrow[r] = __builtin_amdgcn_readlane(rid, r);
      const f4v* xr = reinterpret_cast<const f4v*>(p.x + (int64_t)rrow[r] * kRD);
#ifndef RQ_AB_NOLOAD  // (timing-only A/B builds: results wrong)
      R[r][0] = __builtin_nontemporal_load(xr + lane);
      R[r][1] = __builtin_nontemporal_load(xr + 64 + lane);
      if (RL >= 2 && NORM) dvr[r] = p.den_in[rrow[r]];
#else
      (void)xr;
      R[r][0] += 1.0f;
#endif
    };
    // residual centre rows of segment g -> LDS slot sl (producer threads 0..255)
    auto load_res_rows = [&](const ResSeg& g, int sl) __attribute__((always_inline)) {
      if (RL == 0) return;
      float4* dst = reinterpret_cast<float4*>(smem + L::kRes) + sl * RL * (kRD / 4);
      const float4* src = pt < kRD / 4 ? reinterpret_cast<const float4*>(p.ca + (int64_t)g.ca * kRD) + pt
                                       : reinterpret_cast<const float4*>(p.cb + (int64_t)g.cb * kRD) + (pt - kRD / 4);
      if (pt < RL * kRD / 4) dst[pt] = ldf4_sync(src);
    };
    // candidate |c|^2, |c| and ids of segment g -> LDS slot sl (this wave: list positions 64 pw ..),
    // the collapsed bound's segment maxima -> sgz, sgy (every producer wave: all positions)
    float sgz = 0.f, sgy = 0.f;
    auto write_cmeta = [&](const ResSeg& g, int sl) __attribute__((always_inline)) {
      float gz = 0.f, gy = 0.f;
      if (g.cnt > 0) {
        int kl[kPW], cg[kPW], lid[kPW];
        const int32_t* ia[kPW];
        const int32_t* la[kPW];
#pragma unroll
        for (int q = 0; q < kPW; ++q) {
          kl[q] = min(64 * q + lane, g.cnt - 1);
          ia[q] = p.cand_idx ? p.cand_idx + g.cbase + kl[q] : p.cand_count;  // (stand-in: any valid word)
          la[q] = p.cand_lid ? p.cand_lid + g.cbase + kl[q] : p.cand_count;
        }
        ld4_sync(cg, ia[0], ia[1], ia[2], ia[3]);
        ld4_sync(lid, la[0], la[1], la[2], la[3]);
        const float4* ma[kPW];
#pragma unroll
        for (int q = 0; q < kPW; ++q) {
          cg[q] = p.cand_idx ? cg[q] : g.cbase + kl[q];
          lid[q] = p.cand_lid ? lid[q] : kl[q];
          ma[q] = reinterpret_cast<const float4*>(p.c_meta) + cg[q];
        }
        float4 m[kPW];
        ldf4x4_sync(m, ma[0], ma[1], ma[2], ma[3]);
#pragma unroll
        for (int q = 0; q < kPW; ++q) {
          const int k = 64 * q + lane;
          if (q == pw) {
            csq_base[sl * kNC + k] = k < g.cnt ? m[q].x : INFINITY;
            cy_base[sl * kNC + k] = m[q].y;
            cid_base[sl * kNC + k] = cg[q];
            clid_base[sl * kNC + k] = lid[q];
          }
          gz = fmaxf(gz, ratio_up(m[q].w, m[q].y));
          gy = fmaxf(gy, m[q].y);
        }
      }
      sgz = wave_max(gz);
      sgy = wave_max(gy);
    };
    auto write_info = [&](int t, const ResSeg& g, int sl) __attribute__((always_inline)) {
      if (pt == 0) {
        reinterpret_cast<int4*>(info + (t & 3) * 8)[0] = make_int4(g.s, g.cnt, g.cbase, g.pen);
        info[(t & 3) * 8 + 4] = sl;
      }
    };
    // L2 prefetch of a tile's rows (this wave's 8 rows, ids in lanes 0..7 of rid): two dword loads, each
    // lane one 128-B line, into a register nothing reads.  Invisible to the compiler's wait counting (it
    // only makes some of its counted waits a little longer); the register stays reserved (loop-carried)
    // and the kernel ends with vmcnt(0).
    int pf_sink = 0;
    auto prefetch_rows = [&](int rid) __attribute__((always_inline)) {
#if RQ_PFT
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int row = __shfl(rid, (lane >> 4) + 4 * i);
        const char* a = reinterpret_cast<const char*>(p.x + (int64_t)row * kRD) + (lane & 15) * 128;
        asm volatile("global_load_dword %0, %1, off" : "+v"(pf_sink) : "v"(a));
      }
#else
      (void)rid;
#endif
    };
    float s_ex[kRPW], s_v[kRPW];
    double s_v64[kRPW];
    // produce row r of the next tile from R[r] into image buffer bf with residual rows of slot rs
    auto produce_row = [&](int r, int bf, int rs) __attribute__((always_inline)) {
      unsigned char* img = smem + bf * kImg;
      const int tr = kRPW * pw + r;  // tile row
      prow[r] = rrow[r];
      float inv1 = 1.0f;
      if (RL >= 2 && NORM) inv1 = 1.0f / dvr[r];
      float v[8] = {R[r][0].x, R[r][0].y, R[r][0].z, R[r][0].w, R[r][1].x, R[r][1].y, R[r][1].z, R[r][1].w};
      const float4* res = reinterpret_cast<const float4*>(smem + L::kRes) + rs * RL * (kRD / 4);
#ifdef RQ_AB_NORES
      if (false) {
#else
      if (RL >= 1) {
#endif
        const float4 caA = res[lane], caB = res[64 + lane];
        const float c[8] = {caA.x, caA.y, caA.z, caA.w, caB.x, caB.y, caB.z, caB.w};
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = v[e] - c[e];
      }
#ifdef RQ_AB_NORES
      if (false) {
#else
      if (RL >= 2) {
#endif
        const float4 cbA = res[kRD / 4 + lane], cbB = res[kRD / 4 + 64 + lane];
        const float c[8] = {cbA.x, cbA.y, cbA.z, cbA.w, cbB.x, cbB.y, cbB.z, cbB.w};
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = (NORM ? v[e] * inv1 : v[e]) - c[e];
      }
      h2 hh[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) hh[e] = __builtin_convertvector(f2{v[2 * e], v[2 * e + 1]}, h2);
      float se = 0.f, sv = 0.f;
      double sv64 = 0.0;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float ex = (e & 1) ? sub_f16<1>(v[e], hh[e >> 1]) : sub_f16<0>(v[e], hh[e >> 1]);
        se = fmaf(ex, ex, se);
        if (fp64_norm(RL, NORM)) sv64 = fma((double)v[e], (double)v[e], sv64);
        else sv = fmaf(v[e], v[e], sv);
      }
      // dims 4l..4l+3 -> group kh = l/2, byte (l&1)*8; dims 256+4l.. -> group 32 + l/2
      const int o0 = img_off(lane >> 1, tr) + (lane & 1) * 8, o1 = img_off(32 + (lane >> 1), tr) + (lane & 1) * 8;
      typedef __attribute__((ext_vector_type(4))) _Float16 h4;
      *reinterpret_cast<h4*>(img + o0) = __builtin_shufflevector(hh[0], hh[1], 0, 1, 2, 3);
      *reinterpret_cast<h4*>(img + o1) = __builtin_shufflevector(hh[2], hh[3], 0, 1, 2, 3);
      s_ex[r] = se;
      s_v[r] = sv;
      s_v64[r] = sv64;
    };
    // wave totals of the produced rows -> row statistics of tile d in buffer bf (+ den_out)
    auto finish_rows = [&](const int4& d, int bf, bool live) __attribute__((always_inline)) {
      const float e2 = red8(s_ex, lane);
      float nrm;
      if (fp64_norm(RL, NORM)) nrm = (float)sqrt(red8(s_v64, lane));
      else nrm = sqrtf(red8(s_v, lane));
      int row = 0;  // lane 8 r: row id of produced row r (red8's layout)
#pragma unroll
      for (int q = 0; q < kRPW; ++q) row = lane == 8 * q ? prow[q] : row;
      if ((lane & 7) == 0) {
        const int r = red8_row(lane);
        const int tr = kRPW * pw + r;
        const bool valid = live && tr < d.z;
        const float en = sqrtf(e2) * 1.001f + 1e-30f;
        float inv_den = 1.f, dr = 0.f;
        if (NORM && RL >= 1) {
          const float den = nrm + 1e-8f;
          inv_den = 1.0f / den;
          if (RL == 1 && valid && p.den_out) p.den_out[row] = den;
          dr = RL == 1 ? 2.0f * 5.97e-8f
                       : (4.0f * 2.39e-7f * (1.0f + nrm) * inv_den + 4.0f * 5.97e-8f + 1.01f * den_eps * nrm * inv_den);
        }
        const float vn = nrm * 1.0001f + 1e-30f;
        // the collapsed bound's row coefficients (assign.hip): distance estimate P = |c|^2 + m2 (c.vh),
        // error E = A2 |c|
        const float hn = vn + en;       // >= |vh|
        const float vr = vn * inv_den;  // |r| of the row being assigned
        const float k2 = 2.0f * inv_den * 1.000001f;
        const float A = k2 * (en + ar * hn) + 2.0f * dr + 4.8e-7f * vr;
        const float B = k2 * hn * (1.0f + ar);
        const float A2 = (A + B * sgz + 2.39e-7f * sgy) * 1.000001f;
        const float m2 = -2.0f * inv_den * tscale;
        reinterpret_cast<float4*>(smem + L::kStat)[bf * kRT + tr] =
            make_float4(m2, A2, __int_as_float(valid ? row : -1), 0.f);
      }
    };

    // ---- prologue: segments of tiles tb, tb+1; tile tb produced into buffer 0; rows of tb+1 in flight
    int4 d0 = U4(desc_of(tb));
    int4 d1 = U4(desc_of(min(tb + 1, te - 1)));
    int4 d2 = U4(desc_of(min(tb + 2, te - 1)));
    int4 d3 = U4(desc_of(min(tb + 3, te - 1)));
    ResSeg g0 = res_seg_sync(p, d0.x);
    int slot0 = 0;
    ResSeg g1 = g0;
    int slot1 = 0;
    if (d1.x != d0.x) {
      g1 = res_seg_sync(p, d1.x);
      slot1 = 1;
    }
    load_res_rows(g0, 0);
    if (slot1 != slot0) load_res_rows(g1, slot1);
    write_cmeta(g0, slot0);
    write_info(tb, g0, slot0);
    write_info(tb + 1, g1, slot1);
    lds_barrier();  // P1: residual rows, meta, info
    const int rid1 = load_rids(d1);
    int rid2 = load_rids(d2);
    int rid3 = load_rids(d3);
    {
      const int rid0 = load_rids(d0);
#pragma unroll
      for (int r = 0; r < kRPW; ++r) issue_row(rid0, r);
#pragma unroll
      for (int r = 0; r < kRPW; ++r) produce_row(r, 0, slot0);
      finish_rows(d0, 0, true);
    }
    prefetch_rows(rid2);
    int4 d4raw = desc_of(min(tb + 4, te - 1));
#pragma unroll
    for (int r = 0; r < kRPW; ++r) issue_row(rid1, r);
    lds_barrier();  // P2: tile tb's image and statistics
    // ---- steady state.  Vector loads per iteration, always the same and in this order (the counted
    // waits stay exact and never drain the row stream): the descriptor of tile j+4 and the row ids of
    // tile j+3 (waited for an iteration later, behind the rows), then per produced row of tile j+1 the
    // rows of tile j+2 (+ den_in).  Segment preparation loads through the *_sync helpers.
    for (int j = tb; j < te; ++j) {
      const int b = (j - tb) & 1;
      const bool has1 = j + 1 < te;
      const int4 d4 = U4(d4raw);  // issued an iteration ago, before the rows now in flight
      d4raw = desc_of(min(j + 5, te - 1));
      const int rid4 = load_rids(d4);
      prefetch_rows(rid3);  // tile j+3 into L2 (its register loads: next iteration)
      // segment of tile j+2: residual rows now (read by the production of j+2 in the next iteration),
      // tile info for the candidate waves
      ResSeg g2 = g1;
      int slot2 = slot1;
      if (d2.x != d1.x) {
        g2 = res_seg_sync(p, d2.x);
        slot2 = slot1 ^ 1;
        load_res_rows(g2, slot2);
      }
      write_info(j + 2, g2, slot2);
      // candidate meta (and the maxima) of tile j+1's segment, first needed by its production below
      if (has1 && d1.x != d0.x) write_cmeta(g1, slot1);
      RS_MARK(1);
      // tile j+1: produce from R, re-fill R with tile j+2
#pragma unroll
      for (int r = 0; r < kRPW; ++r) {
        produce_row(r, b ^ 1, slot1);
        issue_row(rid2, r);
      }
      finish_rows(d1, b ^ 1, has1);
      RS_MARK(2);
      lds_barrier();
      RS_MARK(5);
      d0 = d1;
      d1 = d2;
      d2 = d3;
      d3 = d4;
      rid2 = rid3;
      rid3 = rid4;
      g0 = g1;
      slot0 = slot1;
      g1 = g2;
      slot1 = slot2;
    }
    asm volatile("s_waitcnt vmcnt(0)" : "+v"(pf_sink));  // the prefetches land before the wave ends
  } else {
    // =========================== candidate waves: MFMA + bound epilogue
    const int h = lane >> 5, n = lane & 31;
    const int cw = wave;
    // this wave's 32 candidates (A operand) of the current segment: k-steps < kKR in registers, the
    // rest in the wave's LDS area (the registers are the budget: 3 waves per SIMD)
    f16x8 a[kKR];
    f16x8* const al = reinterpret_cast<f16x8*>(smem + L::kAL) + cw * kLA * 64 + lane;
    auto load_centres = [&](int cnt, int cbase) __attribute__((always_inline)) {
      const int m = min(32 * cw + n, cnt - 1);
      const int cg = cand_global(p, cbase, m);
      const _Float16* src = reinterpret_cast<const _Float16*>(p.c16) + (int64_t)cg * (2 * kRD) + 8 * h;
      f16x8 t[kLA];
#pragma unroll
      for (int ks = 0; ks < kKS; ++ks) {
        const f16x8 v = *reinterpret_cast<const f16x8*>(src + (ks >> 1) * 64 + (ks & 1) * 16);
        if (ks < kKR) a[ks] = v;
        else t[ks - kKR] = v;
      }
#pragma unroll
      for (int ks = 0; ks < kKR; ++ks) asm volatile("" : "+v"(a[ks]));  // complete here (see the loop)
#pragma unroll
      for (int i = 0; i < kLA; ++i) al[64 * i] = t[i];
    };
    {
      const ResSeg g0 = res_seg(p, runi(desc[tb].x));
      lds_barrier();  // P1
      if (g0.cnt > 0) load_centres(g0.cnt, g0.cbase);
      lds_barrier();  // P2
    }
    for (int j = tb; j < te; ++j) {
      const int b = (j - tb) & 1;
      const TileInfo ti = read_info(j);
      RS_MARK(1);
      f32x16 acc = {};
      {
        const unsigned char* ib = smem + b * kImg + img_off(h, n);  // + 2 kGS per k-step
        f16x8 fb[RQ_PF];
#pragma unroll
        for (int i = 0; i < RQ_PF; ++i) fb[i] = *reinterpret_cast<const f16x8*>(ib + 2 * kGS * i);
#pragma unroll
        for (int ks = 0; ks < kKS; ++ks) {
          const f16x8 bf = fb[ks % RQ_PF];
          if (ks + RQ_PF < kKS) fb[ks % RQ_PF] = *reinterpret_cast<const f16x8*>(ib + 2 * kGS * (ks + RQ_PF));
          const f16x8 af = ks < kKR ? a[ks < kKR ? ks : 0] : al[64 * (ks < kKR ? 0 : ks - kKR)];
          acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(af, bf, acc, 0, 0, 0);
        }
      }
      RS_MARK(2);
      // the next tile's segment: reload the centres (completed inside: hipcc's wait counting is
      // path-insensitive, a load left pending here would put a wait before every MFMA)
      if (j + 1 < te) {
        const TileInfo tn = read_info(j + 1);
        if (tn.s != ti.s && tn.cnt > 0) load_centres(tn.cnt, tn.cbase);
      }
      RS_MARK(3);
      // ---- epilogue 1: per-candidate bounds, this wave's row summary (the collapsed bound of assign.hip)
      int row_id, my_cid, my_clid;
#ifdef RQ_AB_E2REG
      float e1U = 0.f, e1lb = 0.f, e1Lo = 0.f;
#endif
      float lbv[16];  // lower bounds, kept for the pass masks of an ambiguous row
      {
        const float4 st = reinterpret_cast<const float4*>(smem + L::kStat)[b * kRT + n];
        const float m2 = st.x, A2 = st.y;
        row_id = __float_as_int(st.z);
        const float* csq = csq_base + ti.slot * kNC + 32 * cw + 4 * h;
        const float* cy = cy_base + ti.slot * kNC + 32 * cw + 4 * h;
        float U = INFINITY, lbk = INFINITY, Lo = INFINITY;
        int kv = 0;
#pragma unroll
        for (int g = 0; g < 8; ++g) {  // two candidates at a time (register pressure)
          __builtin_amdgcn_sched_barrier(0);
          const float2 cs = *reinterpret_cast<const float2*>(csq + 8 * (g >> 1) + 2 * (g & 1));
          const float2 yy = *reinterpret_cast<const float2*>(cy + 8 * (g >> 1) + 2 * (g & 1));
          const float csv[2] = {cs.x, cs.y}, yv[2] = {yy.x, yy.y};
#pragma unroll
          for (int e = 0; e < 2; ++e) {
            const int v = 2 * g + e;
            const float P = fmaf(m2, acc[v], csv[e]);
            const float E = fmaf(A2, yv[e], 1e-30f);
            const float ub = P + E, lb = P - E;
            const bool nm = ub < U;
            Lo = fminf(Lo, nm ? lbk : lb);
            lbk = nm ? lb : lbk;
            kv = nm ? v : kv;
            U = nm ? ub : U;
            lbv[v] = lb;
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
#ifdef RQ_AB_E2REG
        e1U = U;
        e1lb = lbk;
        e1Lo = Lo;
#endif
        // this wave's candidate ids, read before the barrier: after it a producer may rewrite the slot
        my_cid = cid_base[ti.slot * kNC + kpos];
        my_clid = clid_base[ti.slot * kNC + kpos];
      }
      RS_MARK(4);
      lds_barrier();
      RS_MARK(5);
      // ---- epilogue 2: the row decision (every candidate wave computes it; the winner's wave writes)
      {
        // (narrow reads in groups of two waves: the centres leave ~20 registers beside the bounds)
#ifdef RQ_AB_E2REG  // (timing-only: the exchange replaced by this wave's own summary)
        float exr[4 * kCW];
#pragma unroll
        for (int w = 0; w < 4 * kCW; ++w) exr[w] = (w & 3) == 0 ? e1U : (w & 3) == 1 ? e1lb : e1Lo;
        const float* ex = exr;
#else
        const float* ex = reinterpret_cast<const float*>(exch + (b * kRT + n) * L::kEX);
#endif
        float U = INFINITY;
#pragma unroll
        for (int w = 0; w < kCW; ++w) U = fminf(U, ex[4 * w]);
        // pass: lb < Up, Up above U by >= 2 ulp (a candidate admitted by rounding is only re-scored)
        const float Up = fmaf(fabsf(U), 0x1p-22f, U) + 1.2e-38f;
        RS_MARK(8);
        int cnt = 0, win = 0;
        bool many = false;
#pragma unroll
        for (int w = 0; w < kCW; ++w) {
          if ((w & 1) == 0) __builtin_amdgcn_sched_barrier(0);
          const float2 e = *reinterpret_cast<const float2*>(ex + 4 * w + 1);
          const bool pk = (__float_as_uint(e.x - Up) >> 31) != 0;
          cnt += pk ? 1 : 0;
          win = pk ? w : win;
          many = many || (__float_as_uint(e.y - Up) >> 31) != 0;
        }
        const bool valid = row_id >= 0;
        const bool definitive = !ti.pen && !many && cnt == 1;
        RS_MARK(9);
#ifdef RQ_AB_NOSTORE
        if (h == 0 && valid && definitive && win == cw && row_id == -7) {
#else
        if (h == 0 && valid && definitive && win == cw) {
#endif
          p.out_local[row_id] = my_clid;
          p.out_global[row_id] = my_cid;
        }
        // ambiguous rows (a few per cent): every candidate wave stores its pass mask in work[row]
        // (word cw); wave 0 marks the row (sentinel -2, segment in seg_of_row, ~segment for a row of
        // a penalty / empty segment).  Behind a wave-uniform branch: the common tile skips it.
        RS_MARK(10);
        const bool amb = valid && !definitive;
        if (__builtin_amdgcn_ballot_w64(amb)) {
          uint32_t mk = 0;
#pragma unroll
          for (int v = 0; v < 16; ++v) mk |= (__float_as_uint(lbv[v] - Up) >> 31) << ((v & 3) + 8 * (v >> 2) + 4 * h);
          mk |= __shfl_xor(mk, 32);
          if (h == 0 && amb) {
            reinterpret_cast<uint32_t*>(p.work + row_id)[cw] = mk;
            if (cw == 0) {
              p.out_global[row_id] = -2;
              seg_of_row[row_id] = ti.pen ? ~ti.s : ti.s;
            }
          }
        }
      }
      RS_MARK(6);
    }
  }
#ifdef RQSID_STAMPS
  RS(rs_acc[7] = (uint32_t)(te - tb);)
  if (lane == 0 && (wave == 0 || wave == kCW)) {
    rs_acc[0] = RS_NOW() - rs_0;
    for (int k = 0; k < 16; ++k) atomicAdd(&g_rstamps[(wave >= kCW ? 1 : 0) * 16 + k], (unsigned long long)rs_acc[k]);
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
  bool attr[3][2] = {};  // [RL][NORM]
};
DevState g_dev[64];

template <int RL, bool NORM>
int launch_res(const AssignParams& p, const int4* desc, const int32_t* seg_tile32, int32_t* seg_of_row, hipStream_t st) {
  using L = ResLayout<RL>;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return fail(RQSID_E_LAUNCH, "assign: hipGetDevice");
  DevState& ds = g_dev[dev];
  if (!ds.ncu) {
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, dev) != hipSuccess) return fail(RQSID_E_LAUNCH, "assign: device properties");
    ds.ncu = prop.multiProcessorCount;
  }
  const void* k = (const void*)assign_resident_kernel<RL, NORM>;
  if (!ds.attr[RL][NORM]) {
    if (hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, L::kBytes) != hipSuccess)
      return fail(RQSID_E_LAUNCH, "assign: cannot raise the dynamic LDS limit (resident screen)");
    ds.attr[RL][NORM] = true;
  }
  const unsigned g = (unsigned)(ds.ncu >= 8 ? ds.ncu / 8 * 8 : 8);  // one persistent block per CU
  hipLaunchKernelGGL((assign_resident_kernel<RL, NORM>), dim3(g), dim3(kThreads), L::kBytes, st, p, desc, seg_tile32,
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
                     t3 ? 0 : kCW);
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
#define RQ_R(RL, NORM, T3) return launch_res<RL, NORM>(p, desc, seg_tile32, seg_of_row, st)
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
