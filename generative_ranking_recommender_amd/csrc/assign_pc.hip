// assign_pc.hip — producer/consumer screen: rqsid_assign's default for the gathered 1-term residual level of
// 512-d rows (PROD level 2: <= 256 candidates per segment).  The 3-term form (<= 128 candidates, PROD level
// 1) is built and parity-tested but slower there than the per-tile kernel: RQSID_PC=2 or
// RQSID_SCREEN_VARIANT=9 select it.
//
// Same arithmetic as the ping-pong form (assign_stream.hip) and the per-tile kernel (assign.hip,
// ONE = true): fp16 MFMA screen, the collapsed per-candidate bound, pass-bit masks, fp64 re-score of the
// rows the bound leaves ambiguous; the returned IDs are the exact argmin, bit-identical to every other form.
// What differs is who does what:
//  * One persistent 512-thread block per CU, 128-row tiles of one segment, XCD-contiguous tile runs.
//  * Waves 0-3 are CONSUMERS (one per SIMD): each owns 32 rows of the tile and runs only LDS fragment
//    reads, MFMAs (32 rows x all candidates, 128 accumulator registers) and the tile's bound epilogue and
//    output stores.  They issue no global load, so no wave that computes ever stalls on DMA issue.
//  * Waves 4-7 are PRODUCERS (one per SIMD, beside a consumer): they issue every global_load_lds of the
//    block (row chunks from HBM four chunks ahead, the candidates' fp16 centre chunks two ahead, the next
//    tile's header in two dependent levels), run the fused residual chain on the landed fp32 rows and
//    write the MFMA B operand (fp16 rows, and their rounding residuals for the 3-term screen) into a
//    double-buffered LDS image, and reduce the rows' bound coefficients {m2, A2} once per tile.  So the
//    residual chain's VALU of one wave runs beside the MFMAs of the other wave on the same SIMD.
//  * One barrier per 32-dim chunk; every producer wait is a counted vmcnt whose count depends only on the
//    chunk's position in the tile (a fixed number of DMA ops per phase, dummy sources when a tile has no
//    successor), and the block waits vmcnt(0) before it exits.
// Ring schedule, phase g (chunk g of the block's tile sequence, 16 per tile):
//   consumer: MFMAs of chunk g from B(g) and C(g); after chunk 15 of a tile, that tile's epilogue
//   producer: DMA C(g+2), DMA R(g+4), [header steps], build B(g+1) from R(g+1); wait C(g+1); barrier
// LDS: R 4 x 16 KiB, C 3 x 16 KiB, B 2 x 8 (1-term) / 16 KiB (3-term), 2 header parities, coefficients.
// hipcc keeps nothing in M0 in this translation unit (tests/test_abi.py checks the built code object: every
// M0 write in assign_pc_kernel sets the LDS-DMA base right before its global_load_lds), so the DMA asm does
// not save and restore it (two scalar instructions fewer per DMA)
#define RQ_M0_KEEP 0
#include "assign_common.h"

#ifdef RQSID_STAMPS
// diagnostic build only (tools/pc_stamps.py): per role (0 consumer, 1 row producer, 2 loader) lane 0 of every
// wave adds {total, barrier, vmcnt wait, epilogue / finish, waves, compute / build, DMA issue, -} cycles
__device__ unsigned long long g_pc_stamps[24];
#define PST(...) __VA_ARGS__
#define PNOW() __builtin_amdgcn_s_memtime()
#else
#define PST(...)
#endif

namespace rqsid {
namespace {

constexpr int kQDim = 512, kQC = 32, kQNch = kQDim / kQC;  // 512-d rows, 32-dim chunks, 16 per tile
constexpr int kQRows = 128;                                  // rows per tile
constexpr int kQSentinel = -2;

// per-tile descriptor, built by pc_desc_kernel (32 B: one s_load_dwordx8)
struct PcDesc {
  int32_t s, t0, nrows, cnt, cbase, flags, ca_row, cb_row;  // flags: bit 0 no screen (penalty / no candidates), bit 1 penalty
};
static_assert(sizeof(PcDesc) == 32, "descriptor layout");

template <int NT, int RL, bool T3>
struct PcLayout {
  static constexpr int Sr = 4, Sc = 3;                              // row / centre ring stages
  static constexpr int kTerms = T3 ? 2 : 1;
  static constexpr int kXS = kQRows * kQC * 4;                      // one row chunk: 128 rows x 128 B
  static constexpr int kCT = NT * 32 * kQC * 2;                     // one fp16 table image: NT*32 x 64 B
  static constexpr int kCS = kCT * kTerms;                          // centre stage (hi [+ lo])
  static constexpr int kBW = 2 * kTerms * 1024;                     // one consumer's B operand per chunk
  static constexpr int kBS = 4 * kBW;                               // B stage
  static constexpr int kX = 0;
  static constexpr int kC = kX + Sr * kXS;
  static constexpr int kB = kC + Sc * kCS;
  static constexpr int kH = kB + 2 * kBS;                           // [2 parities] header
  static constexpr int kHRow = 0;                                   //   128 i32 row ids
  static constexpr int kHCidx = kHRow + kQRows * 4;                 //   NT*32 i32 candidate ids
  static constexpr int kHCsq = kHCidx + NT * 128;                   //   NT*32 f32 |c|^2
  static constexpr int kHY = kHCsq + NT * 128;                      //   NT*32 f32 |c|
  static constexpr int kHDen = kHY + NT * 128;                      //   128 f32 den_in (RL 2)
  static constexpr int kHRes = kHDen + kQRows * 4;                  //   RL x 512 f32 residual centre rows
  static constexpr int kHBytes = kHRes + RL * kQDim * 4;
  static constexpr int kCoef = kH + 2 * kHBytes;                    // 128 x {m2, A2, den, -}
  static constexpr int kBytes = kCoef + kQRows * 16;
  static constexpr int kCI = NT / 2;                                // centre DMA ops per loader per table
  static constexpr int H = 3;                                       // ops of each header level
  static_assert(kCI * kTerms == 4, "four centre DMA ops per loader and phase");
  static_assert(kBytes <= 160 * 1024, "LDS budget");
};

__device__ __forceinline__ int uni(int v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ uint64_t uni64(const void* ptr) {
  const uint64_t a = reinterpret_cast<uint64_t>(ptr);
  return ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(a >> 32)) << 32) |
         (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)a);
}
// the descriptor of tile T: one scalar load that completes inside the asm (an SMEM op: lgkmcnt, never vmcnt)
__device__ __forceinline__ PcDesc load_desc(const PcDesc* d) {
  typedef __attribute__((ext_vector_type(8))) int i32x8;
  i32x8 v;
  asm volatile("s_load_dwordx8 %0, %1, 0x0\n\ts_waitcnt lgkmcnt(0)" : "=s"(v) : "s"(uni64(d)) : "memory");
  PcDesc o;
  o.s = v[0]; o.t0 = v[1]; o.nrows = v[2]; o.cnt = v[3]; o.cbase = v[4]; o.flags = v[5]; o.ca_row = v[6]; o.cb_row = v[7];
  return o;
}
// one global_load_lds_dword: every lane moves 4 B from its own address to lds_base + lane*4
__device__ __forceinline__ void dma4(const void* gsrc, uint32_t lds_base) {
  uint32_t keep;
  asm volatile(
      RQ_M0_SAVE
      "s_mov_b32 m0, %2\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dword %1, off"
      RQ_M0_RESTORE
      : "=&s"(keep)
      : "v"(gsrc), "s"(lds_base)
      : "memory");
}
template <int N>
__device__ __forceinline__ void vm_lgkm_barrier() {
  asm volatile("s_waitcnt vmcnt(%0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::"i"(N) : "memory");
}
__device__ __forceinline__ void lgkm_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

template <int NT, int RL, bool NORM, bool T3>
__global__ __launch_bounds__(768, 3) void assign_pc_kernel(AssignParams p, const int32_t* seg_tiles,
                                                           const PcDesc* desc) {
  using L = PcLayout<NT, RL, T3>;
  constexpr int kCI = L::kCI, H = L::H;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  asm volatile("s_setreg_imm32_b32 hwreg(HW_REG_MODE, 6, 2), 0");  // fp16/fp64 denormals flushed (to_f16)
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = uni(tid >> 6);
  const int h = lane >> 5, r = lane & 31;
  const uint32_t lds0 = lds_addr(smem);

  // XCD-contiguous tile runs (block b on XCD b % 8 walks tiles xlo + slot, + G8, ...)
  const int ntiles = uni(seg_tiles[p.n_segments]);  // (<= max_tiles: stream_tiles_kernel clamps it)
  const int G8 = (int)(gridDim.x >> 3), xcd = (int)(blockIdx.x & 7), slot = (int)(blockIdx.x >> 3);
  const int xlo = (int)((int64_t)xcd * ntiles / 8), xhi = (int)((int64_t)(xcd + 1) * ntiles / 8);
  const int T0 = xlo + slot;
  if (T0 >= xhi) return;  // block-uniform: every wave of the block leaves together

  if (wave < 4) {
    // ================================ consumer (wave c = rows 32c .. 32c+31) ================================
    const int c = wave;
    const int csw = (r >> 2) & 3;  // centre image swizzle of this lane's candidate rows
    f32x16 acc[NT];
    f32x16 accl[T3 ? NT : 1];
    // MFMAs of chunk g from B(g) (stage g & 1) and C(g) (stage g % 3); FIRST: the tile's first chunk
    // (zero accumulators in, a compile-time choice: the call sites pass a literal)
    auto compute = [&](int g, bool first) __attribute__((always_inline)) {
      const f32x16 zero16 = {};
      const unsigned char* bimg = smem + L::kB + (g & 1) * L::kBS + c * L::kBW + lane * 16;
      const unsigned char* cimg0 = smem + L::kC + (g % L::Sc) * L::kCS + r * 64;
      f16x8 bf[2], bl[2];
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        bf[ks] = *reinterpret_cast<const f16x8*>(bimg + (ks * L::kTerms) * 1024);
        if (T3) bl[ks] = *reinterpret_cast<const f16x8*>(bimg + (ks * L::kTerms + 1) * 1024);
      }
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const unsigned char* cimg = cimg0 + (((2 * ks + h) ^ csw) << 4);
#pragma unroll
        for (int t = 0; t < NT; ++t) {
          const f16x8 af = *reinterpret_cast<const f16x8*>(cimg + t * 32 * 64);
          acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(af, bf[ks], (first && ks == 0) ? zero16 : acc[t], 0, 0, 0);
          if (T3) {
            const f16x8 al = *reinterpret_cast<const f16x8*>(cimg + L::kCT + t * 32 * 64);
            accl[T3 ? t : 0] = __builtin_amdgcn_mfma_f32_32x32x16_f16(af, bl[ks], (first && ks == 0) ? zero16 : accl[T3 ? t : 0],
                                                                      0, 0, 0);
            accl[T3 ? t : 0] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, bf[ks], accl[T3 ? t : 0], 0, 0, 0);
          }
        }
      }
    };
    // epilogue of tile T (its {m2, A2} were written by the producers in the phase before)
    PST(uint64_t s_eM = 0, s_eU = 0, s_eB = 0, s_eD = 0;)
    auto epilogue = [&](const PcDesc& D, int par) __attribute__((always_inline)) {
#ifdef RQSID_STAMPS
      uint64_t e0 = PNOW();
      {
        float dmy;  // the last MFMA's result: the matrix pipe drained
        asm volatile("v_mov_b32 %0, %1" : "=v"(dmy) : "v"(acc[NT - 1][15]));
        asm volatile("s_waitcnt lgkmcnt(0)" ::"v"(dmy));
      }
      s_eM += PNOW() - e0;
      e0 = PNOW();
#endif
      const unsigned char* hb = smem + L::kH + par * L::kHBytes;
      const int lr = 32 * c + r;
      const bool row_valid = lr < D.nrows;
      const int my_row = p.row_index ? reinterpret_cast<const int*>(hb + L::kHRow)[min(lr, D.nrows - 1)]
                                     : D.t0 + min(lr, D.nrows - 1);
      auto cand_of = [&](int k) -> int {
        if (D.flags & 1) return 0;
        if (!p.cand_idx) return D.cbase + min(k, D.cnt - 1);
        return reinterpret_cast<const int*>(hb + L::kHCidx)[min(k, NT * 32 - 1)];
      };
      int out_l = kQSentinel, out_g = kQSentinel;
      bool need = false;
      WorkItem w{};
      w.row = my_row;
      w.seg = D.s;
      if (D.flags & 1) {
        need = true;
        w.n = (D.flags & 2) ? -2 : -3;
      } else {
        const float4 rc = *reinterpret_cast<const float4*>(smem + L::kCoef + lr * 16);
        // per candidate P = m2 d + |c|^2, E = A2 |c| (+ 1e-30); ub = P + E, lb = P - E, U = min ub, and a
        // candidate passes iff lb <= U' (the pp / per-tile epilogue).  Here ub and lb are one FMA each on P
        // and the two 1e-30 terms move into U' (lb - 1e-30 <= U + 1e-30 <=> lb <= U + 2e-30): the same test
        const f2 m2v = {rc.x, rc.x}, a2v = {rc.y, rc.y}, na2v = {-rc.y, -rc.y};
        const float* m_csq = reinterpret_cast<const float*>(hb + L::kHCsq);
        const float* m_y = reinterpret_cast<const float*>(hb + L::kHY);
        float U = INFINITY;
#pragma unroll
        for (int t = 0; t < NT; ++t) {
#pragma unroll
          for (int gq = 0; gq < 4; ++gq) {
            const float4 csq = *reinterpret_cast<const float4*>(m_csq + t * 32 + 8 * gq + 4 * h);
            const float4 yy = *reinterpret_cast<const float4*>(m_y + t * 32 + 8 * gq + 4 * h);
#pragma unroll
            for (int e = 0; e < 2; ++e) {
              const int v = 4 * gq + 2 * e;
              f2 d = {acc[t][v], acc[t][v + 1]};
              if (T3) d = f2{accl[T3 ? t : 0][v], accl[T3 ? t : 0][v + 1]} * 0x1p-12f + d;
              const f2 P2 = m2v * d + (e ? f2{csq.z, csq.w} : f2{csq.x, csq.y});
              const f2 y2 = e ? f2{yy.z, yy.w} : f2{yy.x, yy.y};
              const f2 ub = a2v * y2 + P2, lb = na2v * y2 + P2;
              U = fminf(U, fminf(ub.x, ub.y));
              acc[t][v] = lb.x;
              acc[t][v + 1] = lb.y;
            }
          }
        }
        U = fminf(U, xor32(U));
        const float Up = fmaf(fabsf(U), 0x1p-22f, U) + (1.2e-38f + 2e-30f);
        PST(asm volatile("" ::"v"(Up)); s_eU += PNOW() - e0; e0 = PNOW();)
        const f2 upv = {Up, Up};
        uint32_t pbt[NT];
#pragma unroll
        for (int t = 0; t < NT; ++t) pbt[t] = 0u;
#pragma unroll
        for (int v = 0; v < 16; v += 2)
#pragma unroll
          for (int t = 0; t < NT; ++t) {
            const f2 d = f2{acc[t][v], acc[t][v + 1]} - upv;
            pbt[t] = __builtin_amdgcn_alignbit(pbt[t], __float_as_uint(d.x), 31);
            pbt[t] = __builtin_amdgcn_alignbit(pbt[t], __float_as_uint(d.y), 31);
          }
        uint32_t pbits[NT / 2];
#pragma unroll
        for (int wd = 0; wd < NT / 2; ++wd) pbits[wd] = (pbt[2 * wd] << 16) | pbt[2 * wd + 1];
        if (D.cnt < NT * 32) {  // candidates beyond cnt (duplicates of the last one) never pass
#pragma unroll
          for (int wd = 0; wd < NT / 2; ++wd) {
            uint32_t m = 0;
#pragma unroll
            for (int qq = 0; qq < 2; ++qq) {
              const int rem = D.cnt - 32 * (2 * wd + qq) - 4 * h;  // valid iff (v&3) + 8(v>>2) < rem
              int nv = 0;
#pragma unroll
              for (int gq = 0; gq < 4; ++gq) nv += min(4, max(0, rem - 8 * gq));
              const uint32_t pre = (uint32_t)((0xFFFFull << (16 - nv)) & 0xFFFFull);
              m |= qq == 0 ? pre << 16 : pre;
            }
            pbits[wd] &= m;
          }
        }
        PST(asm volatile("" ::"v"(pbits[0]), "v"(pbits[NT / 2 - 1])); s_eB += PNOW() - e0; e0 = PNOW();)
        int k = -1;
        if (pass_decide(pbits, h, k, w)) {
          out_l = p.cand_lid ? cand_local(p, D.cbase, k) : k;  // (a deduplicated list reports the original local id)
          out_g = cand_of(k);
        } else {
          need = true;
        }
      }
      if (h == 0 && row_valid) {  // a consumer issues no load: its stores need no fixed count
        p.out_local[my_row] = out_l;
        p.out_global[my_row] = out_g;
        if (need) p.work[my_row] = w;
        if (RL == 1 && NORM) p.den_out[my_row] = reinterpret_cast<const float*>(smem + L::kCoef + lr * 16)[2];
      }
      PST(s_eD += PNOW() - e0;)
    };
    lgkm_barrier();  // prologue barriers a, b, c (loaders: header, centres; producers: rows, B(0))
    lgkm_barrier();
    lgkm_barrier();
    PST(uint64_t s_bar = 0, s_cmp = 0, s_epi = 0; const uint64_t s_t0 = PNOW(); uint64_t s_a;)
    int g = 0;
    for (int T = T0; T < xhi; T += G8) {
      const int par = (g >> 4) & 1;
      PST(s_a = PNOW();)
      compute(g, true);
      const PcDesc D = load_desc(desc + T);  // (phase 0 has slack; the epilogue's chain does not)
      PST(s_cmp += PNOW() - s_a; s_a = PNOW();)
      lgkm_barrier();  // end of phase g: B(g) / C(g) reads retired
      PST(s_bar += PNOW() - s_a;)
      ++g;
#pragma unroll 1
      for (int j = 1; j < kQNch - 1; ++j, ++g) {
        PST(s_a = PNOW();)
        compute(g, false);
        PST(s_cmp += PNOW() - s_a; s_a = PNOW();)
        lgkm_barrier();
        PST(s_bar += PNOW() - s_a;)
      }
      PST(s_a = PNOW();)
      compute(g, false);
      PST(s_cmp += PNOW() - s_a; s_a = PNOW();)
      epilogue(D, par);
      PST(s_epi += PNOW() - s_a; s_a = PNOW();)
      lgkm_barrier();
      PST(s_bar += PNOW() - s_a;)
      ++g;
    }
#ifdef RQSID_STAMPS
    if (lane == 0) {
      atomicAdd(&g_pc_stamps[0], (unsigned long long)(PNOW() - s_t0));
      atomicAdd(&g_pc_stamps[1], (unsigned long long)s_bar);
      atomicAdd(&g_pc_stamps[3], (unsigned long long)s_epi);
      atomicAdd(&g_pc_stamps[4], 1ull);
      atomicAdd(&g_pc_stamps[5], (unsigned long long)s_cmp);
      atomicAdd(&g_pc_stamps[2], (unsigned long long)s_eM);
      atomicAdd(&g_pc_stamps[6], (unsigned long long)s_eU);
      atomicAdd(&g_pc_stamps[7], (unsigned long long)s_eB);
      atomicAdd(&g_pc_stamps[23], (unsigned long long)s_eD);
    }
#endif
    return;
  }

  const float* trow = p.c_meta + 4 * (int64_t)p.n_centers;
  auto hdr_base = [&](int par) { return lds0 + L::kH + par * L::kHBytes; };
  auto row_of = [&](const PcDesc& D, int par, int lr) -> int {  // lr: row of the tile (clamped to the last one)
    const int l = min(lr, D.nrows - 1);
    return p.row_index ? reinterpret_cast<const int*>(smem + L::kH + par * L::kHBytes + L::kHRow)[l] : D.t0 + l;
  };

  if (wave < 8) {
    // ============================= row producer (wave 4+q: rows 32q .. 32q+31) =============================
    // Its vector-memory ops are its own row chunks only, so its one counted wait (R(g+1) landed, R(g+2..g+4)
    // younger) gives every row chunk three phases to arrive.
    const int q = wave - 4;
    const float tscale = __uint_as_float(uni(__float_as_uint(trow[0])));
    const float tgz = __uint_as_float(uni(__float_as_uint(trow[1])));
    const float tgw = __uint_as_float(uni(__float_as_uint(trow[2])));
    const float tgy = __uint_as_float(uni(__float_as_uint(trow[3])));
    const int xsw = (r >> 1) & 7;  // x image swizzle of this lane's row
    const char* const xbase = reinterpret_cast<const char*>(p.x);
    struct XSrc {
      uint64_t xo[4];  // row instruction i: byte offset of its lane's row piece (row*2048 + slot*16)
    };
    auto x_src = [&](const PcDesc& D, int par, XSrc& s) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {  // instruction i: rows 8i + lane/8 of this producer's 32, slot lane % 8
        const int lr = 8 * i + (lane >> 3);
        const int sl = (lane & 7) ^ ((lr >> 1) & 7);
        s.xo[i] = (uint64_t)(uint32_t)row_of(D, par, 32 * q + lr) * 2048u + (uint64_t)(sl * 16);
      }
    };
    auto issue_r = [&](const XSrc& s, int cj, int st) {
      const uint32_t sx = lds0 + L::kX + st * L::kXS + q * 4096;
      const char* xb = xbase + cj * (kQC * 4);
#pragma unroll
      for (int i = 0; i < 4; ++i) dma16_nt(xb + s.xo[i], uni(sx + i * 1024));
    };
    RowSums rs;
    float inv1 = 1.0f;
    // B of chunk cj of tile D (parity par) from row stage rst into B stage bst
    auto build = [&](const PcDesc& D, int par, int cj, int rst, int bst) {
      const unsigned char* hb = smem + L::kH + par * L::kHBytes;
      if (cj == 0) {
        rs = RowSums{};
        if (RL == 2 && NORM) inv1 = 1.0f / reinterpret_cast<const float*>(hb + L::kHDen)[32 * q + r];
      }
      const float* lds_ca = reinterpret_cast<const float*>(hb + L::kHRes);
      const float* lds_cb = reinterpret_cast<const float*>(hb + L::kHRes + (RL == 2 ? kQDim * 4 : 0));
      const unsigned char* xrow = smem + L::kX + rst * L::kXS + q * 4096 + r * 128;
      unsigned char* bimg = smem + L::kB + bst * L::kBS + q * L::kBW + lane * 16;
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const int q0 = 4 * ks + 2 * h;
        const float4 xa = *reinterpret_cast<const float4*>(xrow + ((q0 ^ xsw) << 4));
        const float4 xc = *reinterpret_cast<const float4*>(xrow + (((q0 + 1) ^ xsw) << 4));
        f16x8 bf, bl = {};
        row_frag<RL, NORM, T3, true>(xa, xc, lds_ca, lds_cb, cj * kQC + 16 * ks + 8 * h, inv1, bf, bl, rs);
        *reinterpret_cast<f16x8*>(bimg + (ks * L::kTerms) * 1024) = bf;
        if (T3) *reinterpret_cast<f16x8*>(bimg + (ks * L::kTerms + 1) * 1024) = bl;
      }
    };
    // after chunk 15 of a tile: the rows' {m2, A2, den} (the consumers write den_out for RL 1 NORM)
    auto finish = [&]() {
      const int lr = 32 * q + r;
      float inv_den = 1.f, dr = 0.f, vn, en, en2 = 0.f, den = 0.f;
      const float se2 = rs.se2v.x + rs.se2v.y, sf2 = rs.sf2v.x + rs.sf2v.y;
      en = sqrtf(se2 + xor32(se2)) * 1.001f + 1e-30f;
      if (T3) {
        const float l2 = rs.se2l.x + rs.se2l.y;
        en2 = sqrtf(l2 + xor32(l2)) * (1.001f / 4096.0f) + 1e-30f;
      }
      float nrm;
      if (NORM && RL >= 1) {
        if (RL == 1) {  // exact: the next level's divisor
          const double t2 = rs.sv2 + rs.sv2b;
          nrm = (float)sqrt(t2 + xor32(t2));
        } else {  // fp32 sums: |nrm - |v|| <= den_eps |v| (chains of dim/4 + 2 terms, sqrt's half ulp)
          nrm = sqrtf(sf2 + xor32(sf2));
        }
        den = nrm + 1e-8f;
        inv_den = 1.0f / den;
        const float den_eps = (0.125f * (float)(kQDim) + 3.0f) * 5.97e-8f;
        dr = RL == 1 ? 2.0f * 5.97e-8f
                     : (4.0f * 2.39e-7f * (1.0f + nrm) * inv_den + 4.0f * 5.97e-8f + 1.01f * den_eps * nrm * inv_den);
      } else {
        nrm = sqrtf(sf2 + xor32(sf2));
      }
      vn = nrm * 1.0001f + 1e-30f;
      const float hn = vn + en;
      const float vr = vn * inv_den;
      const float ar = p.acc_rel, ar2 = 2.0f * p.acc_rel, k2 = 2.0f * inv_den * 1.000001f;
      const float A = T3 ? k2 * (en2 + ar * hn + ar2 * (en + en2)) + 2.0f * dr + 7.2e-7f * vr
                         : k2 * (en + ar * hn) + 2.0f * dr + 4.8e-7f * vr;
      const float B = T3 ? k2 * (hn * (1.0f + ar2) + 2.0f * (en + en2)) : k2 * hn * (1.0f + ar);
      const float C = T3 ? k2 * ((en + en2) + ar * hn + ar2 * (hn + en + en2)) : 0.0f;
      const float m2 = -2.0f * inv_den * tscale;
      const float A2 = (A + B * (T3 ? tgz : tgw) + C * tgw + 2.39e-7f * tgy) * 1.000001f;
      if (h == 0) *reinterpret_cast<float4*>(smem + L::kCoef + lr * 16) = make_float4(m2, A2, den, 0.f);
    };

    PcDesc Dc = load_desc(desc + T0);
    lgkm_barrier();                               // a: the loaders' level 1 of tile T0 (row ids) landed
    XSrc cur, nxt;
    x_src(Dc, 0, cur);
#pragma unroll
    for (int i = 0; i < 4; ++i) issue_r(cur, i, i);
    vm_lgkm_barrier<0>();                         // b: R(0..3) landed; the loaders' level 2 too
    build(Dc, 0, 0, 0, 0);
    lgkm_barrier();                               // c = the barrier of phase 0
    PcDesc Dn = Dc;
    PST(uint64_t s_bar = 0, s_vm = 0, s_fin = 0, s_bld = 0, s_iss = 0; const uint64_t s_t0 = PNOW(); uint64_t s_a;)
    int g = 0;
    for (int T = T0; T < xhi; T += G8) {
      const int Tn = T + G8;
      const bool more = Tn < xhi;
      const int par = (g >> 4) & 1;
#pragma unroll 1
      for (int j = 0; j < kQNch; ++j, ++g) {
        // ---- phase g: DMA R(g+4); wait R(g+1); build B(g+1); barrier ----
        PST(s_a = PNOW();)
        {
          const int cj = j + 4;
          issue_r(cj < kQNch ? cur : nxt, cj & (kQNch - 1), (g + 4) & 3);
        }
        PST(s_iss += PNOW() - s_a;)
        if (j == 0) Dn = load_desc(desc + (more ? Tn : T));  // no successor: the current tile's valid sources
        if (j == 4) x_src(Dn, par ^ 1, nxt);  // the loaders' level 1 (phase 1) retired by their wait of phase 3
        PST(s_a = PNOW();)
        asm volatile("s_waitcnt vmcnt(12)" ::: "memory");  // R(g+1) landed: younger are R(g+2), R(g+3), R(g+4)
        PST(s_vm += PNOW() - s_a; s_a = PNOW();)
        if (j < kQNch - 1) build(Dc, par, j + 1, (g + 1) & 3, (g + 1) & 1);
        else build(Dn, par ^ 1, 0, (g + 1) & 3, (g + 1) & 1);
        PST(s_bld += PNOW() - s_a; s_a = PNOW();)
        if (j == kQNch - 2) finish();
        PST(s_fin += PNOW() - s_a; s_a = PNOW();)
        lgkm_barrier();
        PST(s_bar += PNOW() - s_a;)
      }
      Dc = Dn;
      cur = nxt;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no LDS-DMA may outlive the block
#ifdef RQSID_STAMPS
    if (lane == 0) {
      atomicAdd(&g_pc_stamps[8], (unsigned long long)(PNOW() - s_t0));
      atomicAdd(&g_pc_stamps[9], (unsigned long long)s_bar);
      atomicAdd(&g_pc_stamps[10], (unsigned long long)s_vm);
      atomicAdd(&g_pc_stamps[11], (unsigned long long)s_fin);
      atomicAdd(&g_pc_stamps[12], 1ull);
      atomicAdd(&g_pc_stamps[13], (unsigned long long)s_bld);
      atomicAdd(&g_pc_stamps[14], (unsigned long long)s_iss);
    }
#endif
    return;
  }

  // ============================ loader (wave 8+q): centre chunks and tile headers ============================
  const int q = wave - 8;
  const bool hi_tab = !T3 && p.c16h;
  const char* const cbase16 = reinterpret_cast<const char*>(hi_tab ? p.c16h : p.c16);
  const uint32_t cunits = hi_tab ? 64u : 128u;   // 16-B units per centre row of the gathered table
  const int cchunk = hi_tab ? kQC * 2 : kQC * 4;  // bytes per chunk of a centre row
  struct CSrc {
    uint32_t ci[kCI];  // centre instruction j: 16-B unit of its lane's candidate piece
  };
  // level 1 of tile D's header (3 ops): row ids, candidate ids, the residual centre rows
  auto hdr_level1 = [&](const PcDesc& D, int par) {
    const int lr = min(32 * q + r, D.nrows - 1);
    if (lane < 32)  // (exec-masked: still one vector-memory op of this wave, lanes 0..31 are never all off)
      dma4(p.row_index ? (const void*)(p.row_index + D.t0 + lr) : (const void*)p.seg_row_off,
           uni(hdr_base(par) + L::kHRow + q * 128));
    const int k = q * (NT * 8) + (lane & (NT * 8 - 1));  // this loader's NT*8 candidates
    const int kc = D.cnt > 0 ? min(k, D.cnt - 1) : 0;
    if (NT == 8 || lane < 32)
      dma4(p.cand_idx && D.cnt > 0 ? (const void*)(p.cand_idx + D.cbase + kc) : (const void*)p.seg_row_off,
           uni(hdr_base(par) + L::kHCidx + q * (NT * 32)));
    // RL 2: loaders 0,1 load the halves of ca, 2,3 of cb; RL 1: ca halves twice (identical bytes)
    const bool second = RL == 2 && q >= 2;
    const int half = q & 1;
    const float* src = second ? p.cb + (int64_t)D.cb_row * kQDim : p.ca + (int64_t)D.ca_row * kQDim;
    dma16(src + half * 256 + lane * 4, uni(hdr_base(par) + L::kHRes + (second ? kQDim * 4 : 0) + half * 1024));
  };
  auto cand_of = [&](const PcDesc& D, int par, int k) -> int {
    if (D.flags & 1) return 0;
    if (!p.cand_idx) return D.cbase + min(k, D.cnt - 1);
    return reinterpret_cast<const int*>(smem + L::kH + par * L::kHBytes + L::kHCidx)[min(k, NT * 32 - 1)];
  };
  auto c_src = [&](const PcDesc& D, int par, CSrc& s) {
#pragma unroll
    for (int j = 0; j < kCI; ++j) {  // instruction j: candidates (q*kCI + j)*16 + lane/4, slot lane % 4
      const int k = (q * kCI + j) * 16 + (lane >> 2);
      const int sl = (lane & 3) ^ ((k >> 2) & 3);
      s.ci[j] = (uint32_t)cand_of(D, par, k) * cunits + (uint32_t)sl;
    }
  };
  // level 2 (3 ops): the candidates' |c|^2 and |c|, the rows' den_in (RL 2 NORM)
  auto hdr_level2 = [&](const PcDesc& D, int par) {
    const int k = q * (NT * 8) + (lane & (NT * 8 - 1));
    const float* m = p.c_meta + 4 * (int64_t)cand_of(D, par, k);
    if (NT == 8 || lane < 32) {
      dma4(m, uni(hdr_base(par) + L::kHCsq + q * (NT * 32)));
      dma4(m + 1, uni(hdr_base(par) + L::kHY + q * (NT * 32)));
    }
    if (lane < 32)
      dma4(RL == 2 && NORM ? (const void*)(p.den_in + row_of(D, par, 32 * q + r)) : (const void*)p.seg_row_off,
           uni(hdr_base(par) + L::kHDen + q * 128));
  };
  auto issue_c = [&](const CSrc& s, int cj, int st) {
    const uint32_t sc = lds0 + L::kC + st * L::kCS;
    const char* cb = cbase16 + cj * cchunk;
#pragma unroll
    for (int j = 0; j < kCI; ++j) dma16(cb + (uint64_t)s.ci[j] * 16u, uni(sc + (q * kCI + j) * 1024));
    if (T3) {
#pragma unroll
      for (int j = 0; j < kCI; ++j) dma16(cb + kQC * 2 + (uint64_t)s.ci[j] * 16u, uni(sc + L::kCT + (q * kCI + j) * 1024));
    }
  };

  PcDesc Dc = load_desc(desc + T0);
  hdr_level1(Dc, 0);
  vm_lgkm_barrier<0>();                           // a
  CSrc cur, nxt;
  c_src(Dc, 0, cur);
  hdr_level2(Dc, 0);
  issue_c(cur, 0, 0);
  issue_c(cur, 1, 1);
  vm_lgkm_barrier<0>();                           // b
  lgkm_barrier();                                 // c = the barrier of phase 0
  PcDesc Dn = Dc;
  PST(uint64_t s_bar = 0, s_vm = 0, s_iss = 0; const uint64_t s_t0 = PNOW(); uint64_t s_a;)
  int g = 0;
  for (int T = T0; T < xhi; T += G8) {
    const int Tn = T + G8;
    const bool more = Tn < xhi;
    const int par = (g >> 4) & 1;
#pragma unroll 1
    for (int j = 0; j < kQNch; ++j, ++g) {
      // ---- phase g: DMA C(g+2); header steps; wait C(g+1); barrier ----
      PST(s_a = PNOW();)
      {
        const int cj = j + 2;
        issue_c(cj < kQNch ? cur : nxt, cj & (kQNch - 1), (g + 2) % L::Sc);
      }
      PST(s_iss += PNOW() - s_a;)
      if (j == 0) Dn = load_desc(desc + (more ? Tn : T));
      if (j == 1) hdr_level1(Dn, par ^ 1);
      if (j == 4) {  // level 1 (issued in phase 1) retired by the wait of phase 3
        c_src(Dn, par ^ 1, nxt);
        hdr_level2(Dn, par ^ 1);
      }
      // C(g+1) (issued first in phase g-1) landed: the younger ops are phase g-1's header ops and phase g's
      PST(s_a = PNOW();)
#ifdef RQSID_STAMPS
      if (j == 1 || j == 2 || j == 4 || j == 5) asm volatile("s_waitcnt vmcnt(%0)" ::"i"(kCI * L::kTerms + H) : "memory");
      else asm volatile("s_waitcnt vmcnt(%0)" ::"i"(kCI * L::kTerms) : "memory");
      s_vm += PNOW() - s_a;
      s_a = PNOW();
#endif
      if (j == 1 || j == 2 || j == 4 || j == 5) vm_lgkm_barrier<kCI * L::kTerms + H>();
      else vm_lgkm_barrier<kCI * L::kTerms>();
      PST(s_bar += PNOW() - s_a;)
    }
    Dc = Dn;
    cur = nxt;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no LDS-DMA may outlive the block
#ifdef RQSID_STAMPS
  if (lane == 0) {
    atomicAdd(&g_pc_stamps[16], (unsigned long long)(PNOW() - s_t0));
    atomicAdd(&g_pc_stamps[17], (unsigned long long)s_bar);
    atomicAdd(&g_pc_stamps[18], (unsigned long long)s_vm);
    atomicAdd(&g_pc_stamps[20], 1ull);
    atomicAdd(&g_pc_stamps[22], (unsigned long long)s_iss);
  }
#endif
}

// per-tile descriptors (one thread per tile): segment by binary search over the R-row tile offsets
__global__ __launch_bounds__(256) void pc_desc_kernel(AssignParams p, const int32_t* __restrict__ seg_tiles, int64_t cap,
                                                      int R, PcDesc* __restrict__ desc) {
  const int nseg = p.n_segments;
  const int ntiles = seg_tiles[nseg];
  for (int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x; t < ntiles && t < cap; t += (int64_t)gridDim.x * 256) {
    int lo = 0, hi = nseg;
    while (hi - lo > 1) {
      const int mid = (lo + hi) >> 1;
      if (seg_tiles[mid] <= t) lo = mid; else hi = mid;
    }
    const int s = lo;
    PcDesc d;
    const int r0 = p.seg_row_off[s], r1 = p.seg_row_off[s + 1];
    d.s = s;
    d.t0 = r0 + (int)(t - seg_tiles[s]) * R;
    d.nrows = min(R, r1 - d.t0);
    d.cnt = p.cand_count[s];
    d.cbase = p.cand_base[s];
    const bool flag = p.seg_flags && (p.seg_flags[s] & RQSID_SEG_PENALTY);
    d.flags = (flag || d.cnt <= 0 ? 1 : 0) | (flag ? 2 : 0);
    d.ca_row = p.seg_ca ? p.seg_ca[s] : s;
    d.cb_row = p.seg_cb ? p.seg_cb[s] : s;
    desc[t] = d;
  }
}


// ================================================================================================
// Wide form (assign_pcw_kernel, RQSID_PCW=1, an A/B kept for the record): 256-row tiles, 16-dim phases.
// Parity-green but slower at level 2 (10M rows: 17.5 ms vs 7.3 ms; with 64-B row pieces 10.7 ms): the stamps
// (profiles/r6_pc_stamps_wide.txt) show the feeders blocked 72% of a phase issuing their LDS-DMAs -- with one
// issuing wave per SIMD the CU moves ~3.4 B/clk, the 128-row form's two issuing waves per SIMD ~13 B/clk.
// In the 128-row form every 16-KiB row chunk is paired with a 16-KiB centre chunk, and the LDS-DMA bytes per
// phase set its pace (tools/pc_stamps.py: ~2.46k cycles per phase whatever the split of work between waves).
// Here a 32-dim centre chunk serves 256 rows over two 16-dim phases: 3 KiB of LDS-DMA per row instead of 4.
//  * Waves 0-7 are consumers: wave w owns rows 32w .. 32w+31 (one MFMA row tile) and all 256 candidates
//    (eight 32-candidate tiles): 8 accumulators, and the epilogue of assign_pc_kernel, in-wave.
//  * Waves 8-11 are feeders: feeder f issues row group f's 32-dim row pieces (128 B per row: whole lines; a
//    16-dim piece fetches every line twice and ran 1.5x slower) in even phases, two stages, and builds both
//    k-steps of a piece into a 3-slot B ring in odd phases; a quarter of every centre chunk (half of it in
//    each phase, two phases ahead); a quarter of the next tile's header; and row group f's bound sums.
// One counted wait per feeder and phase: every op issued two phases earlier has landed (the rows of the next
// build, the centre chunk of the next phase): 10 + 2 ops per phase pair + 3 header ops in phases 2 and 6.
constexpr int kWRows = 256, kWPh = 32;  // rows per tile, 16-dim phases per tile

// a feeder's bound sums of one row (both lane halves): sum (v - fp16(v))^2 and the norm's sum (the fp32 sum,
// widened; se2l unused by the 1-term form)
struct PcPart {
  float se2, se2l;
  double nv;
};
static_assert(sizeof(PcPart) == 16, "partial sums layout");

template <int RL>
struct PcwLayout {
  static constexpr int Sr = 2, Sc = 3;
  static constexpr int kXS = kWRows * 128;                          // one 32-dim row piece of every row (full lines)
  static constexpr int kCS = 256 * kQC * 2;                         // one 32-dim fp16 centre chunk, 256 candidates
  static constexpr int kBS = kWRows * 16 * 2;                       // B operand of one phase: [group][tile][lane]
  static constexpr int kX = 0;
  static constexpr int kC = kX + Sr * kXS;
  static constexpr int kB = kC + Sc * kCS;
  static constexpr int kH = kB + 3 * kBS;                           // B ring: phase g in slot g % 3
  static constexpr int kHRow = 0;                                   //   256 i32 row ids
  static constexpr int kHCidx = kHRow + kWRows * 4;                 //   256 i32 candidate ids
  static constexpr int kHCsq = kHCidx + 1024;                       //   256 f32 |c|^2
  static constexpr int kHY = kHCsq + 1024;                          //   256 f32 |c|
  static constexpr int kHDen = kHY + 1024;                          //   256 f32 den_in (RL 2)
  static constexpr int kHRes = kHDen + kWRows * 4;                  //   RL x 512 f32 residual centre rows
  static constexpr int kHBytes = kHRes + RL * kQDim * 4;
  static constexpr int kPart = kH + 2 * kHBytes;                    // [256 rows] partial sums (PcPart)
  static constexpr int kBytes = kPart + kWRows * 16;
  static_assert(kBytes <= 160 * 1024, "LDS budget");
};

template <int RL, bool NORM>
__global__ __launch_bounds__(768, 3) void assign_pcw_kernel(AssignParams p, const int32_t* seg_tiles,
                                                            const PcDesc* desc) {
  using L = PcwLayout<RL>;
  constexpr int H = 3;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  asm volatile("s_setreg_imm32_b32 hwreg(HW_REG_MODE, 6, 2), 0");  // fp16/fp64 denormals flushed (to_f16)
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = uni(tid >> 6);
  const int h = lane >> 5, r = lane & 31;
  const uint32_t lds0 = lds_addr(smem);

  const int ntiles = uni(seg_tiles[p.n_segments]);  // (<= max_tiles: stream_tiles_kernel clamps it)
  const int G8 = (int)(gridDim.x >> 3), xcd = (int)(blockIdx.x & 7), slot = (int)(blockIdx.x >> 3);
  const int xlo = (int)((int64_t)xcd * ntiles / 8), xhi = (int)((int64_t)(xcd + 1) * ntiles / 8);
  const int T0 = xlo + slot;
  if (T0 >= xhi) return;  // block-uniform
  const float* trow = p.c_meta + 4 * (int64_t)p.n_centers;

  if (wave < 8) {
    // ============ consumer w: rows 32w + r (row group w / 2, its row tile w % 2), all 256 candidates ============
    const int q = wave >> 1, rt = wave & 1, lr = 32 * wave + r;
    const int csw = (r >> 2) & 3;
    const float tscale = __uint_as_float(uni(__float_as_uint(trow[0])));
    const float tgw = __uint_as_float(uni(__float_as_uint(trow[2])));
    const float tgy = __uint_as_float(uni(__float_as_uint(trow[3])));
    f32x16 acc[8];
    auto compute = [&](int g, bool first) __attribute__((always_inline)) {
      const f32x16 zero16 = {};
      const f16x8 bf = *reinterpret_cast<const f16x8*>(smem + L::kB + (g % 3) * L::kBS + q * 2048 + rt * 1024 + lane * 16);
      // chunk g / 2 (stage (g / 2) % 3), k-step g & 1 of it: 16-B slot 2 (g & 1) + h of each candidate's 64 B
      const unsigned char* cimg = smem + L::kC + ((g >> 1) % L::Sc) * L::kCS + r * 64 + (((2 * (g & 1) + h) ^ csw) << 4);
#pragma unroll
      for (int t = 0; t < 8; ++t) {
        const f16x8 af = *reinterpret_cast<const f16x8*>(cimg + t * 32 * 64);
        acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(af, bf, first ? zero16 : acc[t], 0, 0, 0);
      }
    };
    struct Coef {
      float m2, A2, den;
    };
    auto coefficients = [&]() -> Coef {  // row lr, from its feeder's partial sums
      const PcPart s0 = reinterpret_cast<const PcPart*>(smem + L::kPart)[lr];
      float inv_den = 1.f, dr = 0.f, den = 0.f, nrm;
      const float en = sqrtf(s0.se2) * 1.001f + 1e-30f;
      if (NORM) {
        nrm = sqrtf((float)s0.nv);  // fp32 sums: |nrm - |v|| <= den_eps |v| (chains of <= dim/4 + 2 terms)
        den = nrm + 1e-8f;
        inv_den = 1.0f / den;
        const float den_eps = (0.125f * (float)(kQDim) + 3.0f) * 5.97e-8f;
        dr = RL == 1 ? 2.0f * 5.97e-8f
                     : (4.0f * 2.39e-7f * (1.0f + nrm) * inv_den + 4.0f * 5.97e-8f + 1.01f * den_eps * nrm * inv_den);
      } else {
        nrm = sqrtf((float)s0.nv);
      }
      const float vn = nrm * 1.0001f + 1e-30f;
      const float hn = vn + en;
      const float vr = vn * inv_den;
      const float ar = p.acc_rel, k2 = 2.0f * inv_den * 1.000001f;
      const float A = k2 * (en + ar * hn) + 2.0f * dr + 4.8e-7f * vr;
      const float B = k2 * hn * (1.0f + ar);
      Coef k;
      k.m2 = -2.0f * inv_den * tscale;
      k.A2 = (A + B * tgw + 2.39e-7f * tgy) * 1.000001f;
      k.den = den;
      return k;
    };
    // epilogue of tile D (parity par): the 256-candidate single-pass epilogue of assign_pc_kernel
    auto epilogue = [&](const PcDesc& D, int par, const Coef& cf) __attribute__((always_inline)) {
      const unsigned char* hb = smem + L::kH + par * L::kHBytes;
      const bool row_valid = lr < D.nrows;
      const int my_row = p.row_index ? reinterpret_cast<const int*>(hb + L::kHRow)[min(lr, D.nrows - 1)]
                                     : D.t0 + min(lr, D.nrows - 1);
      int out_l = kQSentinel, out_g = kQSentinel;
      bool need = false;
      WorkItem w{};
      w.row = my_row;
      w.seg = D.s;
      if (D.flags & 1) {
        need = true;
        w.n = (D.flags & 2) ? -2 : -3;
      } else {
        const f2 m2v = {cf.m2, cf.m2}, a2v = {cf.A2, cf.A2}, na2v = {-cf.A2, -cf.A2};
        const float* m_csq = reinterpret_cast<const float*>(hb + L::kHCsq);
        const float* m_y = reinterpret_cast<const float*>(hb + L::kHY);
        float U = INFINITY;
#pragma unroll
        for (int t = 0; t < 8; ++t) {
#pragma unroll
          for (int gq = 0; gq < 4; ++gq) {
            const float4 csq = *reinterpret_cast<const float4*>(m_csq + t * 32 + 8 * gq + 4 * h);
            const float4 yy = *reinterpret_cast<const float4*>(m_y + t * 32 + 8 * gq + 4 * h);
#pragma unroll
            for (int e = 0; e < 2; ++e) {
              const int v = 4 * gq + 2 * e;
              const f2 d = {acc[t][v], acc[t][v + 1]};
              const f2 P2 = m2v * d + (e ? f2{csq.z, csq.w} : f2{csq.x, csq.y});
              const f2 y2 = e ? f2{yy.z, yy.w} : f2{yy.x, yy.y};
              const f2 ub = a2v * y2 + P2, lb = na2v * y2 + P2;
              U = fminf(U, fminf(ub.x, ub.y));
              acc[t][v] = lb.x;
              acc[t][v + 1] = lb.y;
            }
          }
        }
        U = fminf(U, xor32(U));
        const float Up = fmaf(fabsf(U), 0x1p-22f, U) + (1.2e-38f + 2e-30f);
        const f2 upv = {Up, Up};
        uint32_t pbt[8];
#pragma unroll
        for (int t = 0; t < 8; ++t) pbt[t] = 0u;
#pragma unroll
        for (int v = 0; v < 16; v += 2)
#pragma unroll
          for (int t = 0; t < 8; ++t) {
            const f2 d = f2{acc[t][v], acc[t][v + 1]} - upv;
            pbt[t] = __builtin_amdgcn_alignbit(pbt[t], __float_as_uint(d.x), 31);
            pbt[t] = __builtin_amdgcn_alignbit(pbt[t], __float_as_uint(d.y), 31);
          }
        uint32_t pbits[4];
#pragma unroll
        for (int wd = 0; wd < 4; ++wd) pbits[wd] = (pbt[2 * wd] << 16) | pbt[2 * wd + 1];
        if (D.cnt < 256) {  // candidates beyond cnt (duplicates of the last one) never pass
#pragma unroll
          for (int wd = 0; wd < 4; ++wd) {
            uint32_t m = 0;
#pragma unroll
            for (int qq = 0; qq < 2; ++qq) {
              const int rem = D.cnt - 32 * (2 * wd + qq) - 4 * h;  // valid iff (v&3) + 8(v>>2) < rem
              int nv = 0;
#pragma unroll
              for (int gq = 0; gq < 4; ++gq) nv += min(4, max(0, rem - 8 * gq));
              const uint32_t pre = (uint32_t)((0xFFFFull << (16 - nv)) & 0xFFFFull);
              m |= qq == 0 ? pre << 16 : pre;
            }
            pbits[wd] &= m;
          }
        }
        int k = -1;
        if (pass_decide(pbits, h, k, w)) {
          out_l = p.cand_lid ? cand_local(p, D.cbase, k) : k;  // (a deduplicated list reports the original local id)
          out_g = !p.cand_idx ? D.cbase + min(k, D.cnt - 1) : reinterpret_cast<const int*>(hb + L::kHCidx)[min(k, 255)];
        } else {
          need = true;
        }
      }
      if (h == 0 && row_valid) {
        p.out_local[my_row] = out_l;
        p.out_global[my_row] = out_g;
        if (need) p.work[my_row] = w;
        if (RL == 1 && NORM)  // the coefficients' den, recomputed (its partial sums stay until phase 30 of the next tile)
          p.den_out[my_row] = sqrtf((float)reinterpret_cast<const PcPart*>(smem + L::kPart)[lr].nv) + 1e-8f;
      }
    };
    lgkm_barrier();  // prologue barriers a, b, c
    lgkm_barrier();
    lgkm_barrier();
    PST(uint64_t s_bar = 0, s_cmp = 0, s_epi = 0; const uint64_t s_t0 = PNOW(); uint64_t s_a;)
    int g = 0;
    for (int T = T0; T < xhi; T += G8) {
      const int par = (g >> 5) & 1;
      PST(s_a = PNOW();)
      compute(g, true);
      const PcDesc D = load_desc(desc + T);
      PST(s_cmp += PNOW() - s_a; s_a = PNOW();)
      lgkm_barrier();
      PST(s_bar += PNOW() - s_a;)
      ++g;
#pragma unroll 1
      for (int j = 1; j < kWPh - 1; ++j, ++g) {
        PST(s_a = PNOW();)
        compute(g, false);
        PST(s_cmp += PNOW() - s_a; s_a = PNOW();)
        lgkm_barrier();
        PST(s_bar += PNOW() - s_a;)
      }
      PST(s_a = PNOW();)
      const Coef cf = coefficients();
      compute(g, false);
      PST(s_cmp += PNOW() - s_a; s_a = PNOW();)
      epilogue(D, par, cf);
      PST(s_epi += PNOW() - s_a; s_a = PNOW();)
      lgkm_barrier();
      PST(s_bar += PNOW() - s_a;)
      ++g;
    }
#ifdef RQSID_STAMPS
    if (lane == 0) {
      atomicAdd(&g_pc_stamps[0], (unsigned long long)(PNOW() - s_t0));
      atomicAdd(&g_pc_stamps[1], (unsigned long long)s_bar);
      atomicAdd(&g_pc_stamps[3], (unsigned long long)s_epi);
      atomicAdd(&g_pc_stamps[4], 1ull);
      atomicAdd(&g_pc_stamps[5], (unsigned long long)s_cmp);
    }
#endif
    return;
  }

  // ===================== feeder f = wave - 8: row group f (rows 64f .. 64f+63) =====================
  const int f = wave - 8;
  auto hdr_base = [&](int par) { return lds0 + L::kH + par * L::kHBytes; };
  auto row_of = [&](const PcDesc& D, int par, int lr) -> int {
    const int l = min(lr, D.nrows - 1);
    return p.row_index ? reinterpret_cast<const int*>(smem + L::kH + par * L::kHBytes + L::kHRow)[l] : D.t0 + l;
  };
  auto cand_of = [&](const PcDesc& D, int par, int k) -> int {
    if (D.flags & 1) return 0;
    if (!p.cand_idx) return D.cbase + min(k, D.cnt - 1);
    return reinterpret_cast<const int*>(smem + L::kH + par * L::kHBytes + L::kHCidx)[min(k, 255)];
  };
  const char* const xbase = reinterpret_cast<const char*>(p.x);
  const bool hi_tab = p.c16h != nullptr;
  const char* const cbase16 = reinterpret_cast<const char*>(hi_tab ? p.c16h : p.c16);
  const uint32_t cunits = hi_tab ? 64u : 128u;
  const int cchunk = hi_tab ? kQC * 2 : kQC * 4;
  struct Src {
    uint32_t xr[8];  // row instruction i: the row of its lane's piece (rows 8i + lane/8 of group f)
    uint32_t ci[4];  // centre instruction 4f + i: candidates (4f + i)*16 + lane/4
  };
  // logical 16-B slot of this lane's row piece: (lane & 7) ^ ((row of the group >> 1) & 7), row 8i + lane/8:
  // one value for even i, one for odd i
  const uint32_t xslot0 = (uint32_t)(((lane & 7) ^ ((lane >> 4) & 7)) * 16);
  const uint32_t xslot1 = (uint32_t)(((lane & 7) ^ ((4 + (lane >> 4)) & 7)) * 16);
  auto srcs = [&](const PcDesc& D, int par, Src& s) {
#pragma unroll
    for (int i = 0; i < 8; ++i) s.xr[i] = (uint32_t)row_of(D, par, 64 * f + 8 * i + (lane >> 3));
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int k = (4 * f + i) * 16 + (lane >> 2);
      const int sl = (lane & 3) ^ ((k >> 2) & 3);
      s.ci[i] = (uint32_t)cand_of(D, par, k) * cunits + (uint32_t)sl;
    }
  };
  // header levels of tile D (3 ops each; every feeder covers its quarter, no lane masks)
  auto hdr_level1 = [&](const PcDesc& D, int par) {
    const int lr = min(64 * f + lane, D.nrows - 1);
    dma4(p.row_index ? (const void*)(p.row_index + D.t0 + lr) : (const void*)p.seg_row_off,
         uni(hdr_base(par) + L::kHRow + f * 256));
    const int k = 64 * f + lane;
    const int kc = D.cnt > 0 ? min(k, D.cnt - 1) : 0;
    dma4(p.cand_idx && D.cnt > 0 ? (const void*)(p.cand_idx + D.cbase + kc) : (const void*)p.seg_row_off,
         uni(hdr_base(par) + L::kHCidx + f * 256));
    const bool second = RL == 2 && f >= 2;
    const int half = f & 1;
    const float* src = second ? p.cb + (int64_t)D.cb_row * kQDim : p.ca + (int64_t)D.ca_row * kQDim;
    dma16(src + half * 256 + lane * 4, uni(hdr_base(par) + L::kHRes + (second ? kQDim * 4 : 0) + half * 1024));
  };
  auto hdr_level2 = [&](const PcDesc& D, int par) {
    const float* m = p.c_meta + 4 * (int64_t)cand_of(D, par, 64 * f + lane);
    dma4(m, uni(hdr_base(par) + L::kHCsq + f * 256));
    dma4(m + 1, uni(hdr_base(par) + L::kHY + f * 256));
    dma4(RL == 2 && NORM ? (const void*)(p.den_in + row_of(D, par, 64 * f + lane)) : (const void*)p.seg_row_off,
         uni(hdr_base(par) + L::kHDen + f * 256));
  };
  // half hf (0/1) of this feeder's quarter of centre chunk cj into stage st
  auto issue_c = [&](const Src& s, int cj, int st, int hf) {
    const uint32_t sc = lds0 + L::kC + st * L::kCS;
    const char* cb = cbase16 + cj * cchunk;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int J = 2 * hf + i;
      dma16(cb + (uint64_t)s.ci[J] * 16u, uni(sc + (4 * f + J) * 1024));
    }
  };
  auto issue_r = [&](const Src& s, int pj, int st) {  // 32-dim piece pj of the tile's rows (8 ops)
    const uint32_t sx = lds0 + L::kX + st * L::kXS + f * 8192;
    const char* xb0 = xbase + pj * 128 + xslot0;
    const char* xb1 = xbase + pj * 128 + xslot1;
#pragma unroll
    for (int i = 0; i < 8; ++i) dma16_nt((i & 1 ? xb1 : xb0) + (uint64_t)s.xr[i] * 2048u, uni(sx + i * 1024));
  };
  RowSums rs[2];
  float inv1[2] = {1.f, 1.f};
  // B of 32-dim piece pj of tile D (two phases: k-step ks into ring slot bs[ks]): rows 64f + 32rt + r,
  // dims 32pj + 16ks + 8h .. +7
  auto build = [&](const PcDesc& D, int par, int pj, int rst, int bs0, int bs1) {
    const unsigned char* hb = smem + L::kH + par * L::kHBytes;
    if (pj == 0) {
#pragma unroll
      for (int rt = 0; rt < 2; ++rt) {
        rs[rt] = RowSums{};
        if (RL == 2 && NORM) inv1[rt] = 1.0f / reinterpret_cast<const float*>(hb + L::kHDen)[64 * f + 32 * rt + r];
      }
    }
    const float* lds_ca = reinterpret_cast<const float*>(hb + L::kHRes);
    const float* lds_cb = reinterpret_cast<const float*>(hb + L::kHRes + (RL == 2 ? kQDim * 4 : 0));
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int rt = 0; rt < 2; ++rt) {
        __builtin_amdgcn_sched_barrier(0);  // one row tile's chain at a time (register pressure)
        const int lr = 32 * rt + r;  // row of the group
        const unsigned char* xrow = smem + L::kX + rst * L::kXS + f * 8192 + lr * 128;
        const int sw = (lr >> 1) & 7;
        const float4 xa = *reinterpret_cast<const float4*>(xrow + (((4 * ks + 2 * h) ^ sw) << 4));
        const float4 xc = *reinterpret_cast<const float4*>(xrow + (((4 * ks + 2 * h + 1) ^ sw) << 4));
        f16x8 bf, bl;
        row_frag<RL, NORM, false, true>(xa, xc, lds_ca, lds_cb, pj * 32 + 16 * ks + 8 * h, inv1[rt], bf, bl, rs[rt]);
        *reinterpret_cast<f16x8*>(smem + L::kB + (ks ? bs1 : bs0) * L::kBS + f * 2048 + rt * 1024 + lane * 16) = bf;
      }
  };
  auto leave_sums = [&]() {
#pragma unroll
    for (int rt = 0; rt < 2; ++rt) {
      float se2 = rs[rt].se2v.x + rs[rt].se2v.y;
      float sf2 = rs[rt].sf2v.x + rs[rt].sf2v.y;
      se2 += xor32(se2);
      sf2 += xor32(sf2);
      if (h == 0) {
        PcPart part;
        part.se2 = se2;
        part.se2l = 0.f;
        part.nv = (double)sf2;
        reinterpret_cast<PcPart*>(smem + L::kPart)[64 * f + 32 * rt + r] = part;
      }
    }
  };

  // ---- prologue: tile T0's header, centre chunks 0 and 1, row pieces 0..3, B(0) ----
  PcDesc Dc = load_desc(desc + T0);
  hdr_level1(Dc, 0);
  vm_lgkm_barrier<0>();                                   // a
  Src cur, nxt;
  srcs(Dc, 0, cur);
  hdr_level2(Dc, 0);
  issue_c(cur, 0, 0, 0);
  issue_c(cur, 0, 0, 1);
  issue_c(cur, 1, 1, 0);
  issue_c(cur, 1, 1, 1);
  issue_r(cur, 0, 0);
  issue_r(cur, 1, 1);
  vm_lgkm_barrier<0>();                                   // b
  build(Dc, 0, 0, 0, 0, 1);
  lgkm_barrier();                                         // c = the barrier of phase 0
  PcDesc Dn = Dc;
  PST(uint64_t s_bar = 0, s_iss = 0, s_bld = 0, s_vm = 0; const uint64_t s_t0 = PNOW(); uint64_t s_a;)
  int g = 0;
  for (int T = T0; T < xhi; T += G8) {
    const int Tn = T + G8;
    const bool more = Tn < xhi;
    const int par = (g >> 5) & 1;
#pragma unroll 1
    for (int j = 0; j < kWPh; ++j, ++g) {
      // ---- phase g: half (g & 1) of centre chunk g/2 + 2, row piece / build, header steps ----
      PST(s_a = PNOW();)
      {
        const int cj = (j >> 1) + 2;  // chunk of this tile (>= 16: the next tile's)
        issue_c(cj < 16 ? cur : nxt, cj & 15, ((g >> 1) + 2) % L::Sc, j & 1);
      }
      if (!(j & 1)) {  // even phases: row piece j/2 + 2 (>= 16: the next tile's) into stage (g/2) & 1
        const int pj = (j >> 1) + 2;
        issue_r(pj < 16 ? cur : nxt, pj & 15, (g >> 1) & 1);
      }
      if (j == 0) Dn = load_desc(desc + (more ? Tn : T));
      if (j == 2) hdr_level1(Dn, par ^ 1);
      if (j == 6) {  // level 1 (phase 2) retired by the wait of phase 4
        srcs(Dn, par ^ 1, nxt);
        hdr_level2(Dn, par ^ 1);
      }
      PST(s_iss += PNOW() - s_a; s_a = PNOW();)
      if (j & 1) {  // odd phases: B(g+1), B(g+2) from row piece (j+1)/2 (j = 31: the next tile's piece 0)
        if (j < kWPh - 1) build(Dc, par, (j + 1) >> 1, ((g + 1) >> 1) & 1, (g + 1) % 3, (g + 2) % 3);
        else build(Dn, par ^ 1, 0, ((g + 1) >> 1) & 1, (g + 1) % 3, (g + 2) % 3);
      }
      if (j == kWPh - 3) leave_sums();  // after piece 15 (built in phase 29); read in phase 31
      PST(s_bld += PNOW() - s_a; s_a = PNOW();)
      // every op issued up to phase g-2 has landed: younger are phases g-1 and g (12 ops + header ops)
#ifdef RQSID_STAMPS
      if (j == 2 || j == 3 || j == 6 || j == 7) asm volatile("s_waitcnt vmcnt(%0)" ::"i"(12 + H) : "memory");
      else asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
      s_vm += PNOW() - s_a;
      s_a = PNOW();
#endif
      if (j == 2 || j == 3 || j == 6 || j == 7) vm_lgkm_barrier<12 + H>();
      else vm_lgkm_barrier<12>();
      PST(s_bar += PNOW() - s_a;)
    }
    Dc = Dn;
    cur = nxt;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no LDS-DMA may outlive the block
#ifdef RQSID_STAMPS
  if (lane == 0) {
    atomicAdd(&g_pc_stamps[8], (unsigned long long)(PNOW() - s_t0));
    atomicAdd(&g_pc_stamps[9], (unsigned long long)s_bar);
    atomicAdd(&g_pc_stamps[10], (unsigned long long)s_vm);
    atomicAdd(&g_pc_stamps[12], 1ull);
    atomicAdd(&g_pc_stamps[13], (unsigned long long)s_bld);
    atomicAdd(&g_pc_stamps[14], (unsigned long long)s_iss);
  }
#endif
}

template <int RL, bool NORM>
bool launch_pcw(const AssignParams& p, const int32_t* seg_tiles, const PcDesc* desc, int64_t max_tiles, hipStream_t st) {
  using L = PcwLayout<RL>;
  static bool attr[kMaxDevices] = {};
  const int dev = current_device(), ncu = device_cu_count();
  if (dev < 0 || !ncu) return false;
  if (!attr[dev]) {
    if (hipFuncSetAttribute((const void*)assign_pcw_kernel<RL, NORM>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            L::kBytes) != hipSuccess)
      return false;
    attr[dev] = true;
  }
  int64_t g = ncu;  // one persistent block per CU
  if (g > max_tiles) g = max_tiles;
  g = g / 8 * 8;
  if (g < 8) g = 8;
  hipLaunchKernelGGL((assign_pcw_kernel<RL, NORM>), dim3((unsigned)g), dim3(768), L::kBytes, st, p, seg_tiles, desc);
  return true;
}

template <int NT, int RL, bool NORM, bool T3>
bool launch_pc(const AssignParams& p, const int32_t* seg_tiles, const PcDesc* desc, int64_t max_tiles, hipStream_t st) {
  using L = PcLayout<NT, RL, T3>;
  static bool attr[kMaxDevices] = {};
  const int dev = current_device(), ncu = device_cu_count();
  if (dev < 0 || !ncu) return false;
  if (!attr[dev]) {
    if (hipFuncSetAttribute((const void*)assign_pc_kernel<NT, RL, NORM, T3>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            L::kBytes) != hipSuccess)
      return false;
    attr[dev] = true;
  }
  int64_t g = ncu;  // one persistent block per CU
  if (g > max_tiles) g = max_tiles;
  g = g / 8 * 8;
  if (g < 8) g = 8;
  hipLaunchKernelGGL((assign_pc_kernel<NT, RL, NORM, T3>), dim3((unsigned)g), dim3(768), L::kBytes, st, p, seg_tiles, desc);
  return true;
}

}  // namespace

bool pc_supported(int dim, int cand_count_max, bool t3, int rl) {
  if (dim != kQDim || rl < 1 || rl > 2) return false;
  return t3 ? cand_count_max <= 128 : cand_count_max <= 256;
}

int64_t pc_desc_bytes(int64_t n_rows, int32_t n_segments) {
  return ((n_rows > 0 ? n_rows : 0) / kQRows + (int64_t)n_segments + 1) * (int64_t)sizeof(PcDesc);
}

int launch_pc_screen(const AssignParams& p, bool t3, int rl, bool norm, int32_t* tile_seg, int32_t* seg_tiles,
                     void* desc_mem, int64_t cap, hipStream_t st) {
  PcDesc* desc = reinterpret_cast<PcDesc*>(desc_mem);
  // RQSID_PCW=1: the wide form (256-row tiles) on 1-term levels, an A/B only -- measured slower
  const char* we = getenv("RQSID_PCW");
  const bool wide = !t3 && we && atoi(we) == 1;
  const int R = wide ? kWRows : kQRows;
  launch_tiling(p, R, tile_seg, seg_tiles, cap, st);
  const int64_t max_tiles = cap / R + p.n_segments;
  hipLaunchKernelGGL(pc_desc_kernel, dim3(grid_cap(cdiv(max_tiles, 256), 4096)), dim3(256), 0, st, p, seg_tiles,
                     max_tiles, R, desc);
  bool ok = false;
  if (wide) {
    if (rl == 1) ok = norm ? launch_pcw<1, true>(p, seg_tiles, desc, max_tiles, st) : launch_pcw<1, false>(p, seg_tiles, desc, max_tiles, st);
    else ok = norm ? launch_pcw<2, true>(p, seg_tiles, desc, max_tiles, st) : launch_pcw<2, false>(p, seg_tiles, desc, max_tiles, st);
  } else if (t3) {
    if (rl == 1) ok = norm ? launch_pc<4, 1, true, true>(p, seg_tiles, desc, max_tiles, st)
                           : launch_pc<4, 1, false, true>(p, seg_tiles, desc, max_tiles, st);
    else ok = norm ? launch_pc<4, 2, true, true>(p, seg_tiles, desc, max_tiles, st)
                   : launch_pc<4, 2, false, true>(p, seg_tiles, desc, max_tiles, st);
  } else {
    if (rl == 1) ok = norm ? launch_pc<8, 1, true, false>(p, seg_tiles, desc, max_tiles, st)
                           : launch_pc<8, 1, false, false>(p, seg_tiles, desc, max_tiles, st);
    else ok = norm ? launch_pc<8, 2, true, false>(p, seg_tiles, desc, max_tiles, st)
                   : launch_pc<8, 2, false, false>(p, seg_tiles, desc, max_tiles, st);
  }
  return ok ? RQSID_OK : fail(RQSID_E_LAUNCH, "assign: producer/consumer screen launch failed (device query / LDS attribute)");
}

}  // namespace rqsid

#ifdef RQSID_STAMPS
extern "C" int rqsid_debug_pc_stamps(unsigned long long* out24) {
  if (hipMemcpyFromSymbol(out24, HIP_SYMBOL(g_pc_stamps), 24 * sizeof(unsigned long long)) != hipSuccess) return -1;
  unsigned long long z[24] = {};
  return hipMemcpyToSymbol(HIP_SYMBOL(g_pc_stamps), z, sizeof(z)) == hipSuccess ? 0 : -1;
}
#endif
