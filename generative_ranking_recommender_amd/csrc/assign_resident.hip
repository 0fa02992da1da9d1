// assign_resident.hip — the centre-resident, warp-specialised, barrier-free screen: rqsid_assign's path
// for 512-d rows whose segments hold <= 256 candidates, one fp16 term (RQSID_SCREEN_VARIANT=6;
// DESIGN.md §3.1b).
//
// Same arithmetic as assign.hip's single-pass screen (fp16 MFMA X·Cᵀ with a rigorous per-candidate
// error bound, the exact fp64 re-score of ambiguous rows), different data movement.  The per-tile
// kernel re-streams a segment's candidate centres through LDS for every row tile; here they stay in
// registers, and the block is split by role:
//  * One persistent 12-wave block per CU walks an XCD-contiguous run of 32-row tiles (a segment's
//    tiles are consecutive, so the block meets each segment once).
//  * Waves 0-7 (candidate waves) hold 32 candidates each as the MFMA A operand for the whole segment
//    (28 k-steps in registers, 4 in a wave-private LDS area; 8 x 32 = 256 candidates), multiply tile j
//    and run its bound epilogue.  They issue no row loads.
//  * Waves 8-11 (producer waves) own 8 rows of every tile: they load the rows of tile j+2 while
//    producing tile j+1 from registers (the reference's residual chain in fp32 from the segment's
//    residual centre rows, held in registers; fp16 rounding; the MFMA B-operand image in LDS; the
//    bound's per-row coefficients), and prepare segments ahead of use (tile-info ring, the candidates'
//    |c|^2, |c|, ids and collapsed-bound maxima).
//  * No per-tile barrier.  Three monotonic LDS counters order the roles: `ready` (producers: tile
//    written), `consumed` (candidates: MFMAs of a tile done, its image buffer free) and `posted`
//    (candidates: row summaries of a tile in the exchange).  Waves drift within the bounds the
//    buffers allow (images x2, statistics x4, exchange x4, segment metadata x3), so one wave's
//    epilogue overlaps another's MFMAs on the same SIMD instead of all of them alternating in
//    lockstep.  Spins are bounded: a logic error ends in wrong results (caught by the parity tests),
//    never in a hung GPU.
//  * Epilogue: each candidate wave posts per row {least upper bound, lower bound of the candidate
//    attaining it, least lower bound of the others}; once all eight have posted, the row is definitive
//    iff no other lower bound passes (the owning wave writes the ID); ambiguous rows store one pass-mask
//    word per wave in work[row] for res_expand_kernel and the fp64 re-score.
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
#ifndef RQ_E1R
#define RQ_E1R 8  // rounds of LDS metadata reads in epilogue 1
#endif
#ifndef RQ_DEFER
#define RQ_DEFER 1  // epilogue 2 of tile j-1 after tile j's MFMAs
#endif
#ifndef RQ_LBF16
#define RQ_LBF16 1  // deferred lower bounds as bf16 pairs rounded down
#endif
#ifndef RQ_NT
#define RQ_NT 1  // non-temporal row loads (read once)
#endif
#ifndef RQ_E1V2
#define RQ_E1V2 0  // epilogue 1 as independent bounds + min trees (summary: least lb, second least lb, least ub)
#endif
#if RQ_E1V2 && !RQ_LBF16
#error "RQ_E1V2 keeps the deferred lower bounds as bf16 pairs"
#endif
#ifndef RQ_LA
#define RQ_LA 6  // k-steps of the centres kept in LDS (wave-private) instead of registers
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
  static constexpr int kNS = 4;                          // statistics buffers (drift bound 3)
  static constexpr int kNM = 3;                          // segment-metadata slots (drift bound 3)
  static constexpr int kNE = 3;                          // exchange buffers (drift bound 3)
  static constexpr int kStat = 2 * kImg;                 // [kNS][32 rows] float4 {m2, A2, row id, -}
  static constexpr int kCsq = kStat + kNS * kRT * 16;    // [kNM][kNC] |c|^2 (inf: padding)
  static constexpr int kCy = kCsq + kNM * kNC * 4;       // [kNM][kNC] |c|
  static constexpr int kCid = kCy + kNM * kNC * 4;       // [kNM][kNC] global centre id of list position
  static constexpr int kClid = kCid + kNM * kNC * 4;     // [kNM][kNC] local id reported for it
  static constexpr int kEX = kCW + 1;                    // exchange row stride in float4 (padded: conflict-free)
  static constexpr int kExch = kClid + kNM * kNC * 4;    // [kNE][32 rows][kEX] float4 per-wave row summaries
  static constexpr int kIds = kExch + kNE * kRT * kEX * 16;  // [kNE][32 rows][kEX] int2 {global, local} id of each wave's best
  static constexpr int kMask = kIds + kNE * kRT * kEX * 8;   // [2][32 rows][kCW] u32 pass masks of ambiguous rows
  static constexpr int kInfo = kMask + 2 * kRT * kCW * 4;   // [4 tiles][8] int tile-info ring
  static constexpr int kCtr = kInfo + 4 * 8 * 4;         // per-wave counters: ready [4], -, consumed [8], posted [8]
  static constexpr int kAL = kCtr + 24 * 4 + 32;         // [kCW waves][kLA k-steps][64 lanes] f16x8 centre fragments
  static constexpr int kBytes = kAL + kCW * kLA * 64 * 16;
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

// res_seg through ld4_sync (the producers' loop)
__device__ __forceinline__ ResSeg res_seg_sync(const AssignParams& p, int s) {
  const int32_t* a0 = p.cand_count + s;
  const int32_t* a1 = p.cand_base + s;
  const int32_t* a2 = p.seg_ca ? p.seg_ca + s : a0;
  const int32_t* a3 = p.seg_cb ? p.seg_cb + s : a0;
  const uint8_t* fb = p.seg_flags ? p.seg_flags + s : reinterpret_cast<const uint8_t*>(a0);
  int v0, v1, v2, v3, f;
  asm volatile(
      "global_load_dword %0, %5, off\n\tglobal_load_dword %1, %6, off\n\tglobal_load_dword %2, %7, off\n\t"
      "global_load_dword %3, %8, off\n\tglobal_load_ubyte %4, %9, off\n\ts_waitcnt vmcnt(0)"
      : "=&v"(v0), "=&v"(v1), "=&v"(v2), "=&v"(v3), "=&v"(f)
      : "v"(a0), "v"(a1), "v"(a2), "v"(a3), "v"(fb)
      : "memory");
  ResSeg g;
  g.s = s;
  g.cnt = runi(v0);
  g.cbase = runi(v1);
  const bool flag = p.seg_flags && (runi(f) & RQSID_SEG_PENALTY);
  g.pen = flag ? 2 : (g.cnt <= 0 ? 3 : 0);
  g.ca = p.seg_ca ? runi(v2) : s;
  g.cb = p.seg_cb ? runi(v3) : s;
  return g;
}

// a segment's candidate list words (4 cand_idx + 4 cand_lid per lane) and residual centre rows (4
// float4 per lane) in one round trip
__device__ __forceinline__ void ld_seg_sync(int (&ci)[4], int (&cl)[4], float4 (&rr)[4], const int32_t* const (&ia)[4],
                                            const int32_t* const (&la)[4], const float4* const (&ra)[4]) {
  typedef __attribute__((ext_vector_type(4))) float f4;
  f4 r0, r1, r2, r3;
  asm volatile(
      "global_load_dword %0, %12, off\n\tglobal_load_dword %1, %13, off\n\t"
      "global_load_dword %2, %14, off\n\tglobal_load_dword %3, %15, off\n\t"
      "global_load_dword %4, %16, off\n\tglobal_load_dword %5, %17, off\n\t"
      "global_load_dword %6, %18, off\n\tglobal_load_dword %7, %19, off\n\t"
      "global_load_dwordx4 %8, %20, off\n\tglobal_load_dwordx4 %9, %21, off\n\t"
      "global_load_dwordx4 %10, %22, off\n\tglobal_load_dwordx4 %11, %23, off\n\ts_waitcnt vmcnt(0)"
      : "=&v"(ci[0]), "=&v"(ci[1]), "=&v"(ci[2]), "=&v"(ci[3]), "=&v"(cl[0]), "=&v"(cl[1]), "=&v"(cl[2]), "=&v"(cl[3]),
        "=&v"(r0), "=&v"(r1), "=&v"(r2), "=&v"(r3)
      : "v"(ia[0]), "v"(ia[1]), "v"(ia[2]), "v"(ia[3]), "v"(la[0]), "v"(la[1]), "v"(la[2]), "v"(la[3]), "v"(ra[0]),
        "v"(ra[1]), "v"(ra[2]), "v"(ra[3])
      : "memory");
  rr[0] = make_float4(r0.x, r0.y, r0.z, r0.w);
  rr[1] = make_float4(r1.x, r1.y, r1.z, r1.w);
  rr[2] = make_float4(r2.x, r2.y, r2.z, r2.w);
  rr[3] = make_float4(r3.x, r3.y, r3.z, r3.w);
}

__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// Role signalling through per-wave monotonic LDS counters: each wave publishes how many tiles it has
// finished a phase for (ready: producers; consumed, posted: candidates) in its own word, and a waiter
// takes the minimum over the waves it depends on.  (A sum over waves would be wrong: waves of a role
// drift, so a fast wave's extra tile can complete a sum while a slow wave is still mid-tile.)
// Publish: this wave's LDS writes complete (lgkmcnt(0); the LDS performs a wave's operations in order),
// then the new count.  Wait: spin (s_sleep between reads) until every counter reaches the target; the
// asm memory clobbers keep the compiler from moving LDS accesses across either.  Vector-memory counts
// are untouched (no fence): the roles exchange LDS data only.
constexpr int kSpinCap = 1 << 20;  // ~0.1 s: far beyond any legitimate wait
// ``dead`` (wave-uniform): set by a wait that reached the cap; later waits of the wave return at once,
// so even a broken protocol ends the kernel in about one capped wait per wave.  Its results would be
// wrong: every wave that went dead sets bit 0 of the device error word p.err at its exit, and
// rqsid_assign reads the word back and returns RQSID_E_LAUNCH (never wrong IDs silently).
__device__ __forceinline__ void lds_publish(uint32_t* own, uint32_t count) {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  *reinterpret_cast<volatile uint32_t*>(own) = count;
  asm volatile("" ::: "memory");
}
template <int N>  // N = 4 or 8 counters, 16-B aligned
__device__ __forceinline__ void lds_wait_all(const uint32_t* ctr, uint32_t target, int& dead, int cap = kSpinCap) {
  int spin = dead ? cap : 0;
  for (; spin < cap; ++spin) {
    asm volatile("" ::: "memory");
    const volatile uint32_t* c = ctr;
    uint32_t m = c[0];
#pragma unroll
    for (int i = 1; i < N; ++i) m = min(m, (uint32_t)c[i]);
    if ((uint32_t)runi((int)m) >= target) break;
    __builtin_amdgcn_s_sleep(1);
  }
  dead = spin >= cap ? 1 : dead;
  asm volatile("" ::: "memory");
}

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
  uint32_t* const ctr_ready = reinterpret_cast<uint32_t*>(smem + L::kCtr);  // [kPW]
  uint32_t* const ctr_consumed = ctr_ready + 8;                              // [kCW]
  uint32_t* const ctr_posted = ctr_ready + 16;                               // [kCW]
  if (tid < 24) ctr_ready[tid] = 0;
  lds_barrier();  // the only barrier: counters zeroed
  int dead = 0;

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
    // =========================== producer waves: rows, images, row coefficients, segments
    const int pw = wave - kCW, pt = tid - kCW * 64;  // producer wave / thread (0..255)
    const float tscale = __int_as_float(runi(__float_as_int(p.c_meta[4 * p.n_centers])));
    const float ar = p.acc_rel;
    typedef __attribute__((ext_vector_type(4))) float f4v;
    const float den_eps = (0.125f * (float)kRD + 3.0f) * 5.97e-8f;
    f4v R[kRPW][2];
    int rrow[kRPW], prow[kRPW];
#pragma unroll
    for (int r = 0; r < kRPW; ++r) rrow[r] = prow[r] = 0;
    // lanes: id of tile row kRPW pw + (lane & 7).  The load is unconditional (without a row index it
    // reads a stand-in word): a conditional load would break hipcc's counted waits
    const int32_t* const ri_base = p.row_index ? p.row_index : reinterpret_cast<const int32_t*>(desc);
    auto load_rids = [&](const int4& d) __attribute__((always_inline)) {
      const int pos = d.y + min(kRPW * pw + (lane & 7), d.z - 1);
      const int v = ri_base[p.row_index ? pos : 0];
      return p.row_index ? v : pos;
    };
    // Unconditional loads (padding rows re-load the tile's last row; past the block's last tile the
    // descriptors are clamped): the same loads in the same order every iteration keep the waits exact.
    auto issue_row = [&](int rid, int r) __attribute__((always_inline)) {
      rrow[r] = __builtin_amdgcn_readlane(rid, r);
      const f4v* xr = reinterpret_cast<const f4v*>(p.x + (int64_t)rrow[r] * kRD);
#ifndef RQ_AB_NOLOAD
#if RQ_NT
      R[r][0] = __builtin_nontemporal_load(xr + lane);
      R[r][1] = __builtin_nontemporal_load(xr + 64 + lane);
#else
      R[r][0] = xr[lane];
      R[r][1] = xr[64 + lane];
#endif
#else
      (void)xr;
      R[r][0] += 1.0f;
#endif
    };
    // RL 2 NORM: the previous level's denominators of a tile's rows, one gather (lane r: row r), issued
    // with the row ids so that waiting for it never waits for rows
    auto load_dens = [&](int rid) __attribute__((always_inline)) {
      return (RL >= 2 && NORM) ? p.den_in[rid] : 1.0f;
    };
    // the segment's residual centre rows in registers (lane: dims 4l..4l+3 and 256+4l..): ca, cb
    float4 cres[2][2] = {};
    // Segment preparation in two round trips: (1) the candidate list words and the residual centre
    // rows, (2) the candidates' c_meta.  Then: |c|^2, |c| and ids -> metadata slot sl (this wave: list
    // positions 64 pw ..), the collapsed bound's segment maxima -> sgz, sgy (every producer wave: all
    // positions), the residual rows -> cres.
    float sgz = 0.f, sgy = 0.f;
    auto prep_segment = [&](const ResSeg& g, int sl) __attribute__((always_inline)) {
      const bool any = g.cnt > 0;
      int kl[kPW], cg[kPW], lid[kPW];
      const int32_t* ia[kPW];
      const int32_t* la[kPW];
#pragma unroll
      for (int q = 0; q < kPW; ++q) {
        kl[q] = any ? min(64 * q + lane, g.cnt - 1) : 0;
        ia[q] = p.cand_idx && any ? p.cand_idx + g.cbase + kl[q] : p.cand_count;  // (stand-in: any valid word)
        la[q] = p.cand_lid && any ? p.cand_lid + g.cbase + kl[q] : p.cand_count;
      }
      const float4* stand = reinterpret_cast<const float4*>(p.c_meta);
      const float4* ca = RL >= 1 ? reinterpret_cast<const float4*>(p.ca + (int64_t)g.ca * kRD) : stand;
      const float4* cb = RL >= 2 ? reinterpret_cast<const float4*>(p.cb + (int64_t)g.cb * kRD) : stand;
      const float4* ra[4] = {RL >= 1 ? ca + lane : stand, RL >= 1 ? ca + 64 + lane : stand,
                             RL >= 2 ? cb + lane : stand, RL >= 2 ? cb + 64 + lane : stand};
      float4 rr[4];
      ld_seg_sync(cg, lid, rr, ia, la, ra);
      cres[0][0] = rr[0];
      cres[0][1] = rr[1];
      cres[1][0] = rr[2];
      cres[1][1] = rr[3];
      float gz = 0.f, gy = 0.f;
      if (any) {
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
    float s_ex[kRPW], s_v[kRPW];
    double s_v64[kRPW];
    // produce row r of the next tile from R[r] into image buffer bf
    auto produce_row = [&](int r, int bf, float dvs) __attribute__((always_inline)) {
      unsigned char* img = smem + bf * kImg;
      const int tr = kRPW * pw + r;  // tile row
      prow[r] = rrow[r];
      float inv1 = 1.0f;
      if (RL >= 2 && NORM) inv1 = 1.0f / __int_as_float(__builtin_amdgcn_readlane(__float_as_int(dvs), r));
      float v[8] = {R[r][0].x, R[r][0].y, R[r][0].z, R[r][0].w, R[r][1].x, R[r][1].y, R[r][1].z, R[r][1].w};
      if (RL >= 1) {
        const float c[8] = {cres[0][0].x, cres[0][0].y, cres[0][0].z, cres[0][0].w,
                            cres[0][1].x, cres[0][1].y, cres[0][1].z, cres[0][1].w};
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = v[e] - c[e];
      }
      if (RL >= 2) {
        const float c[8] = {cres[1][0].x, cres[1][0].y, cres[1][0].z, cres[1][0].w,
                            cres[1][1].x, cres[1][1].y, cres[1][1].z, cres[1][1].w};
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
    // wave totals of the produced rows -> the bound's row coefficients of tile d in statistics buffer
    // sb (+ den_out)
    auto finish_rows = [&](const int4& d, int sb, bool live) __attribute__((always_inline)) {
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
        reinterpret_cast<float4*>(smem + L::kStat)[sb * kRT + tr] =
            make_float4(m2, A2, __int_as_float(valid ? row : -1), 0.f);
      }
    };

    // ---- prologue: segments of tiles tb, tb+1; tile tb produced into image 0 / statistics 0; rows of
    // tb+1 in flight
    int4 d0 = U4(desc_of(tb));
    int4 d1 = U4(desc_of(min(tb + 1, te - 1)));
    int4 d2 = U4(desc_of(min(tb + 2, te - 1)));
    ResSeg g0 = res_seg_sync(p, d0.x);
    int slot0 = 0;
    ResSeg g1 = g0;
    int slot1 = 0;
    if (d1.x != d0.x) {
      g1 = res_seg_sync(p, d1.x);
      slot1 = 1;
    }
    prep_segment(g0, slot0);
    write_info(tb, g0, slot0);
    write_info(tb + 1, g1, slot1);
    const int rid1 = load_rids(d1);
    int rid2 = load_rids(d2);
    float dv1 = load_dens(rid1);
    {
      const int rid0 = load_rids(d0);
      const float dv0 = load_dens(rid0);
#pragma unroll
      for (int r = 0; r < kRPW; ++r) issue_row(rid0, r);
#pragma unroll
      for (int r = 0; r < kRPW; ++r) produce_row(r, 0, dv0);
      finish_rows(d0, 0, true);
    }
    int4 d3raw = desc_of(min(tb + 3, te - 1));
#pragma unroll
    for (int r = 0; r < kRPW; ++r) issue_row(rid1, r);
    lds_publish(ctr_ready + pw, 1);  // tile tb (and info tb, tb+1, the metadata of its segment)
    // ---- steady state: iteration j produces tile j+1.  Vector loads per iteration, always the same
    // and in this order (counted waits stay exact and never drain the row stream): the descriptor of
    // tile j+3 and the row ids of tile j+2... issued before the rows; segment preparation loads through
    // the *_sync helpers.
    for (int j = tb; j < te; ++j) {
      const int it = j - tb;
      const bool has1 = j + 1 < te;
      const int4 d3 = U4(d3raw);  // issued an iteration ago, before the rows now in flight
      d3raw = desc_of(min(j + 4, te - 1));
      const int rid3 = load_rids(d3);
      const float dv2 = load_dens(rid2);
      // every candidate wave is done with tile j-1's MFMAs (so with its image buffer, which tile j+1
      // reuses) and, before them, with tile j-2's epilogue: the metadata slot, statistics buffer and
      // info entry written below are free
      lds_wait_all<kCW>(ctr_consumed, (uint32_t)it, dead);
      RS_MARK(1);
      // segment of tile j+2 (tile info for the candidate waves); tile j+1's: metadata, maxima and
      // residual rows, first needed by its production below
      ResSeg g2 = g1;
      int slot2 = slot1;
      if (d2.x != d1.x) {
        g2 = res_seg_sync(p, d2.x);
        slot2 = slot1 == L::kNM - 1 ? 0 : slot1 + 1;
      }
      write_info(j + 2, g2, slot2);
      if (has1 && d1.x != d0.x) prep_segment(g1, slot1);
      RS_MARK(2);
      // tile j+1: produce from R, re-fill R with tile j+2
#pragma unroll
      for (int r = 0; r < kRPW; ++r) {
        produce_row(r, (it + 1) & 1, dv1);
        issue_row(rid2, r);
      }
      finish_rows(d1, (it + 1) & (L::kNS - 1), has1);
      lds_publish(ctr_ready + pw, (uint32_t)(it + 2));  // tiles tb .. j+1
      RS_MARK(3);
      d0 = d1;
      d1 = d2;
      d2 = d3;
      rid2 = rid3;
      dv1 = dv2;
      g0 = g1;
      slot0 = slot1;
      g1 = g2;
      slot1 = slot2;
    }
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
      if (g0.cnt > 0) load_centres(g0.cnt, g0.cbase);
    }
    // the previous tile's row and ambiguity (its pass masks are stored one tile later)
    int prev_row = -1;
    bool prev_amb = false;
    auto store_masks = [&](int row, bool am, int mb) __attribute__((always_inline)) {
      if (h == 0 && am) {
        const uint4* src = reinterpret_cast<const uint4*>(smem + L::kMask) + (mb * kRT + n) * 2;
        uint4* dst = reinterpret_cast<uint4*>(p.work + row);
        dst[0] = src[0];
        dst[1] = src[1];
      }
    };
    // Epilogue 2 of tile j-1 runs after tile j's MFMAs (its inputs: the exchange of tile j-1, the row
    // ids and lower bounds below, the tile's segment): the eight waves then meet only loosely (every
    // wave has long posted j-1 when any wave gets there), so the waves of a SIMD drift apart and one
    // wave's epilogues overlap the other's MFMAs.
    int e2_row = -1, e2_it = -1, e2_s = 0, e2_pen = 0;
    // lower bounds of the tile awaiting epilogue 2 (pass masks of an ambiguous row), as bf16 pairs
    // rounded toward -inf: a rounded-down lower bound can only add candidates to an ambiguous row's
    // re-score list, never drop one, and the pair packing keeps the deferral within the registers
#if RQ_LBF16
    uint32_t lbp[8];
#pragma unroll
    for (int v = 0; v < 8; ++v) lbp[v] = 0u;
#else
    float lbf[16];
#pragma unroll
    for (int v = 0; v < 16; ++v) lbf[v] = 0.f;
#endif
    auto bf16_down = [](float x) __attribute__((always_inline)) {  // bf16 bits <= x (x finite or inf)
      const uint32_t u = __float_as_uint(x);
      return (int32_t)u >= 0 ? (u >> 16) : ((u + 0xFFFFu) >> 16);
    };
    auto epilogue2 = [&]() __attribute__((always_inline)) {
      const int t = e2_it;
      lds_wait_all<kCW>(ctr_posted, (uint32_t)(t + 1), dead);  // every wave's summary of that tile
      RS_MARK(5);
      const float* ex = reinterpret_cast<const float*>(exch + ((t % L::kNE) * kRT + n) * L::kEX);
      const int2* id_row = reinterpret_cast<const int2*>(smem + L::kIds) + ((t % L::kNE) * kRT + n) * L::kEX;
      float U = INFINITY;
#pragma unroll
      for (int w = 0; w < kCW; ++w) U = fminf(U, ex[4 * w + 2]);
      // pass: lb < Up, Up above U by >= 2 ulp (a candidate admitted by rounding is only re-scored)
      const float Up = fmaf(fabsf(U), 0x1p-22f, U) + 1.2e-38f;
      int cnt = 0, win = 0;
      bool many = false;
#pragma unroll
      for (int w = 0; w < kCW; ++w) {
        if ((w & 1) == 0) __builtin_amdgcn_sched_barrier(0);
        const float2 e = *reinterpret_cast<const float2*>(ex + 4 * w);  // {lb of the wave's best, least other lb}
        const bool pk = (__float_as_uint(e.x - Up) >> 31) != 0;
        cnt += pk ? 1 : 0;
        win = pk ? w : win;
        many = many || (__float_as_uint(e.y - Up) >> 31) != 0;
      }
      const int row_id = e2_row;
      const bool valid = row_id >= 0;
      const bool definitive = !e2_pen && !many && cnt == 1;
      // ambiguous rows (a few per cent): every wave's pass-mask word of the row into the LDS mask
      // buffer (behind a wave-uniform branch: the common tile skips it)
      const bool amb = valid && !definitive;
      uint32_t* const mrow = reinterpret_cast<uint32_t*>(smem + L::kMask) + ((t & 1) * kRT + n) * kCW;
      if (__builtin_amdgcn_ballot_w64(amb)) {
        uint32_t mk = 0;
#pragma unroll
        for (int v = 0; v < 16; ++v) {
#if RQ_LBF16
          const float lb = __uint_as_float((v & 1) ? (lbp[v >> 1] & 0xFFFF0000u) : (lbp[v >> 1] << 16));
#else
          const float lb = lbf[v];
#endif
          mk |= (__float_as_uint(lb - Up) >> 31) << ((v & 3) + 8 * (v >> 2) + 4 * h);
        }
        mk |= __shfl_xor(mk, 32);
        if (h == 0) mrow[cw] = mk;
      }
      // All of the tile's global stores come from one wave (rotating), each a single instruction over
      // the tile's rows: the IDs of definitive rows (the winner's ids from the exchange), the sentinel
      // -2 and segment of ambiguous rows, and the previous tile's ambiguous rows' pass masks as whole
      // 32-B work records (complete: every wave has posted this tile, so finished the last epilogue 2).
      if (cw == (t & (kCW - 1))) {
        store_masks(prev_row, prev_amb, (t + 1) & 1);
        if (h == 0 && valid) {
          if (definitive) {
            const int2 id = id_row[win];
            p.out_local[row_id] = id.y;
            p.out_global[row_id] = id.x;
          } else {
            p.out_global[row_id] = -2;
            seg_of_row[row_id] = e2_pen ? ~e2_s : e2_s;
          }
        }
      }
      prev_row = row_id;
      prev_amb = amb;
      RS_MARK(6);
    };
    for (int j = tb; j < te; ++j) {
      const int it = j - tb;
      const int b = it & 1;
      lds_wait_all<kPW>(ctr_ready, (uint32_t)(it + 1), dead);  // tile j's image, statistics, info, metadata
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
      lds_publish(ctr_consumed + cw, (uint32_t)(it + 1));  // (fragment reads complete: the MFMAs consumed them)
      RS_MARK(2);
      // the next tile's segment: reload the centres (completed inside: hipcc's wait counting is
      // path-insensitive, a load left pending here would put a wait before every MFMA)
      if (j + 1 < te) {
        const TileInfo tn = read_info(j + 1);
        if (tn.s != ti.s && tn.cnt > 0) load_centres(tn.cnt, tn.cbase);
      }
      RS_MARK(3);
      if (RQ_DEFER && it > 0) epilogue2();  // tile j-1
      // ---- epilogue 1: per-candidate bounds, this wave's row summary (the collapsed bound of assign.hip)
      {
        float4* const ex_row = exch + ((it % L::kNE) * kRT + n) * L::kEX;
        int2* const id_row = reinterpret_cast<int2*>(smem + L::kIds) + ((it % L::kNE) * kRT + n) * L::kEX;
        const float4 st = reinterpret_cast<const float4*>(smem + L::kStat)[(it & (L::kNS - 1)) * kRT + n];
        const float m2 = st.x, A2 = st.y;
        e2_row = __float_as_int(st.z);
        e2_it = it;
        e2_s = ti.s;
        e2_pen = ti.pen;
        const float* csq = csq_base + ti.slot * kNC + 32 * cw + 4 * h;
        const float* cy = cy_base + ti.slot * kNC + 32 * cw + 4 * h;
#if RQ_E1V2
        // Summary {least lb, second least lb, least ub} with the candidate of the least lb: a row is
        // definitive iff exactly one candidate of all waves has lb <= U' (epilogue 2), and that one is
        // then the argmin of ub too (its own lb <= its ub = U), so this posts what epilogue 2 needs with
        // independent bounds (no serial select chain) and three-level min trees.
        float ubv[16], lbv[16];
#pragma unroll
        for (int g = 0; g < 8; ++g) {
          if (g % (8 / RQ_E1R) == 0) __builtin_amdgcn_sched_barrier(0);
          const float2 cs = *reinterpret_cast<const float2*>(csq + 8 * (g >> 1) + 2 * (g & 1));
          const float2 yy = *reinterpret_cast<const float2*>(cy + 8 * (g >> 1) + 2 * (g & 1));
          const float csv[2] = {cs.x, cs.y}, yv[2] = {yy.x, yy.y};
#pragma unroll
          for (int e = 0; e < 2; ++e) {
            const int v = 2 * g + e;
            const float P = fmaf(m2, acc[v], csv[e]);
            const float E = fmaf(A2, yv[e], 1e-30f);
            ubv[v] = P + E;
            lbv[v] = P - E;
          }
          lbp[g] = bf16_down(lbv[2 * g]) | (bf16_down(lbv[2 * g + 1]) << 16);
        }
        float U = fminf(fminf(fminf(fminf(ubv[0], ubv[1]), ubv[2]), fminf(fminf(ubv[3], ubv[4]), ubv[5])),
                        fminf(fminf(fminf(ubv[6], ubv[7]), ubv[8]), fminf(fminf(ubv[9], ubv[10]), ubv[11])));
        U = fminf(U, fminf(fminf(ubv[12], ubv[13]), fminf(ubv[14], ubv[15])));
        float l1[8], l2[8];
        int ix[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const float a0 = lbv[2 * i], a1 = lbv[2 * i + 1];
          const bool lo = a0 <= a1;
          l1[i] = fminf(a0, a1);
          l2[i] = fmaxf(a0, a1);
          ix[i] = lo ? 2 * i : 2 * i + 1;
        }
#pragma unroll
        for (int w = 4; w >= 1; w >>= 1) {
#pragma unroll
          for (int i = 0; i < w; ++i) {
            const bool lo = l1[i] <= l1[i + w];
            l2[i] = fminf(fminf(fmaxf(l1[i], l1[i + w]), l2[i]), l2[i + w]);
            l1[i] = fminf(l1[i], l1[i + w]);
            ix[i] = lo ? ix[i] : ix[i + w];
          }
        }
        float lbk = l1[0], Lo = l2[0];
        int kpos = 32 * cw + (ix[0] & 3) + 8 * (ix[0] >> 2) + 4 * h;
        const float oU = __shfl_xor(U, 32), ol1 = __shfl_xor(lbk, 32), ol2 = __shfl_xor(Lo, 32);
        const int ok = __shfl_xor(kpos, 32);
        const bool take = ol1 < lbk || (ol1 == lbk && ok < kpos);
        Lo = fminf(fminf(fmaxf(lbk, ol1), Lo), ol2);
        lbk = fminf(lbk, ol1);
        kpos = take ? ok : kpos;
        U = fminf(U, oU);
        if (h == 0) ex_row[cw] = make_float4(lbk, Lo, U, 0.f);
        if (h == 0) id_row[cw] = make_int2(cid_base[ti.slot * kNC + kpos], clid_base[ti.slot * kNC + kpos]);
#else
        float U = INFINITY, lbk = INFINITY, Lo = INFINITY;
        int kv = 0;
#pragma unroll
        for (int g = 0; g < 8; ++g) {  // metadata read in RQ_E1R rounds (latency vs register pressure)
          if (g % (8 / RQ_E1R) == 0) __builtin_amdgcn_sched_barrier(0);
          const float2 cs = *reinterpret_cast<const float2*>(csq + 8 * (g >> 1) + 2 * (g & 1));
          const float2 yy = *reinterpret_cast<const float2*>(cy + 8 * (g >> 1) + 2 * (g & 1));
          const float csv[2] = {cs.x, cs.y}, yv[2] = {yy.x, yy.y};
          uint32_t lbh[2];
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
            lbh[e] = bf16_down(lb);
#if !RQ_LBF16
            lbf[v] = lb;
#endif
          }
#if RQ_LBF16
          lbp[g] = lbh[0] | (lbh[1] << 16);
#endif
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
        if (h == 0) ex_row[cw] = make_float4(lbk, Lo, U, 0.f);  // (lbk, Lo): an 8-B aligned pair
        // this wave's candidate ids, posted beside the summary for the tile's store wave
        if (h == 0) id_row[cw] = make_int2(cid_base[ti.slot * kNC + kpos], clid_base[ti.slot * kNC + kpos]);
#endif
      }
      lds_publish(ctr_posted + cw, (uint32_t)(it + 1));
      RS_MARK(4);
      if (!RQ_DEFER) epilogue2();
    }
    if (RQ_DEFER) epilogue2();  // the last tile
    // the last tile's ambiguous rows: its mask words are complete once every wave has left its last
    // epilogue
    const int nt = te - tb;
    lds_publish(ctr_posted + cw, (uint32_t)(nt + 1));
    if (cw == (nt & (kCW - 1))) {
      lds_wait_all<kCW>(ctr_posted, (uint32_t)(nt + 1), dead, p.force_cap ? 0 : kSpinCap);
      store_masks(prev_row, prev_amb, (nt - 1) & 1);
    }
  }
  if (dead && lane == 0) atomicOr(p.err, 1);
#ifdef RQSID_STAMPS
  RS(rs_acc[7] = (uint32_t)(te - tb);)
  if (lane == 0 && (wave == 0 || wave == kCW)) {
    rs_acc[0] = RS_NOW() - rs_0;
    for (int k = 0; k < 16; ++k) atomicAdd(&g_rstamps[(wave >= kCW ? 1 : 0) * 16 + k], (unsigned long long)rs_acc[k]);
  }
#endif
#undef RS_MARK
}

// 32-row tiling of the segments: seg_tile32[s] = sum_{s' < s} ceil(rows(s') / 32) (one block); the total is
// clamped to the descriptor area's max_tiles entries, raising kErrTiles (as stream_tiles_kernel)
__global__ __launch_bounds__(1024) void res_tiles_kernel(const int32_t* __restrict__ seg_row_off, int nseg,
                                                         int64_t max_tiles, int32_t* __restrict__ err,
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
  if (tid == 1023) {
    int total = part[1023];
    if ((int64_t)total > max_tiles) {
      if (err) atomicOr(err, kErrTiles);
      total = (int)max_tiles;
    }
    seg_tile32[nseg] = total;
  }
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
  hipLaunchKernelGGL(res_tiles_kernel, dim3(1), dim3(1024), 0, st, p.seg_row_off, p.n_segments, cap,
                     p.work_count ? p.work_count + kErrSlot : (int32_t*)nullptr, seg_tile32);
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
