// assign_rows.hip — the row-resident screen (round 4): rqsid_assign's screen for 1-term residual levels of
// 512-d rows with up to 512 candidates per segment (PROD level 2: 256, the XL preset's level 2: 512).
//
// Same arithmetic and bound as assign_screen_kernel (fp16 MFMA v_mfma_f32_32x32x16_f16, the collapsed
// per-candidate bound with the table-wide constants of the streamed forms, exact fp64 re-score of the
// ambiguous rows), different data movement:
//  * A wave's 32 rows are loaded ONCE per tile with plain global_load_dwordx4 (8 lanes per 128-B row
//    line, as the LDS-DMA row stream reads them), turned into the level's residual and into the MFMA B
//    operand, and kept in VGPRs for the whole tile: 32 k-steps x 8 fp16 = 128 VGPRs per lane.  Rows never
//    pass through LDS except a 4-KiB per-wave transpose into the fragment layout, so the LDS-DMA path
//    carries only the L2-resident centre stream, and a W-wave block (W*32 rows) shares one centre stream:
//    W = 8 halves the centre bytes per row of the 128-row tiles.
//  * Candidates stream in blocks of 128 (4 MFMA tiles) through an S-stage ring of 32-dim chunks; after
//    each block's 16 chunks the epilogue folds the block into a running least upper bound U and a list
//    of the candidates whose lower bound is <= U (<= 4 per lane half, compacted as U shrinks).  A row
//    whose list overflows goes to the fp32 re-screen / fp64 re-score with every candidate, as in the
//    multi-pass per-tile screen.
//  * Persistent blocks walk XCD-contiguous runs of W*32-row tiles (a segment's tiles share an L2).
// The returned IDs are the exact argmin (the screen only decides which rows need the re-score).
#include "assign_common.h"

namespace rqsid {
namespace {

constexpr int kRDim = 512;        // row width of this screen
constexpr int kRNch = kRDim / 32; // 32-dim chunks
constexpr int kRMaxCand = 512;    // candidates per segment
#ifndef RQSID_ROWS_NTB
#define RQSID_ROWS_NTB 2
#endif
constexpr int kNTB = RQSID_ROWS_NTB;  // MFMA tiles (32 candidates) per candidate block
template <int W, int S, int SR, int NTB>
struct RowsLayout {
  static constexpr int kCB = NTB * 32;                // candidates per block (NTB MFMA tiles of 32)
  static constexpr int kCStage = kCB * 64;            // kCB candidates x 32 fp16 dims (hi terms)
  static constexpr int kScr = S * kCStage;            // per-wave row rings: SR stages x 32 rows x 128 B (fp32)
  static constexpr int kScrWave = SR * 32 * 128;
  static constexpr int kMeta = kScr + W * kScrWave;   // |c|^2 [512], |c| [512]
  static constexpr int kGidx = kMeta + 2 * kRMaxCand * 4;  // global centre of each local candidate [512]
  static constexpr int kRes = kGidx + kRMaxCand * 4;  // residual centre rows ca, cb (fp32 512 each)
  static constexpr int kBytes = kRes + 2 * kRDim * 4;
  static constexpr int kBlocks = W == 4 ? 2 : 1;      // blocks per CU (2 waves per SIMD either way)
  static constexpr int kOps = kCB / 16;               // centre DMA ops per chunk (1 KiB each)
  static constexpr int P = kOps >= W ? kOps / W : 1;  // per issuing wave (waves >= kOps / P issue none)
  static_assert(kOps % W == 0 || W % kOps == 0, "centre DMA split");
  static_assert(kRNch % S == 0, "ring stages must divide the chunks of a block (static stage index)");
  static_assert(SR >= 2 && SR <= 4, "row ring depth");
  static_assert((S - 2) * P <= 63, "vmcnt field");
  static_assert(kBytes * kBlocks <= 160 * 1024, "LDS budget");
};

// wait until at most 4*younger vector-memory ops of this wave are outstanding, then drain its LDS ops
__device__ __forceinline__ void wait_rows(int younger) {
  if (younger >= 2) asm volatile("s_waitcnt vmcnt(8)\n\ts_waitcnt lgkmcnt(0)" ::: "memory");
  else if (younger == 1) asm volatile("s_waitcnt vmcnt(4)\n\ts_waitcnt lgkmcnt(0)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(0)\n\ts_waitcnt lgkmcnt(0)" ::: "memory");
}

template <int W, int S, int SR, int NTB, int RL, bool NORM>
__global__ __launch_bounds__(W * 64, 2) void assign_rows_kernel(AssignParams p, const int32_t* __restrict__ tile_seg,
                                                                const int32_t* __restrict__ seg_tiles) {
  static_assert(!(RL == 1 && NORM), "the first-residual normalising level writes den_out: per-tile kernel");
  using L = RowsLayout<W, S, SR, NTB>;
  constexpr int P = L::P, R = W * 32, kCB = L::kCB;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  asm volatile("s_setreg_imm32_b32 hwreg(HW_REG_MODE, 6, 2), 0");  // fp16/fp64 denormals flushed (to_f16)
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int h = lane >> 5, r = lane & 31;
  const uint32_t lds0 = lds_addr(smem);

  const int ntiles = __builtin_amdgcn_readfirstlane(seg_tiles[p.n_segments]);
  const int G8 = (int)(gridDim.x >> 3), xcd = (int)(blockIdx.x & 7), slot = (int)(blockIdx.x >> 3);
  const int xlo = (int)((int64_t)xcd * ntiles / 8), xhi = (int)((int64_t)(xcd + 1) * ntiles / 8);

  // table-wide bound constants (meta row k, rqsid_prepare_centers)
  const float* trow = p.c_meta + 4 * (int64_t)p.n_centers;
  const float tscale = __uint_as_float(__builtin_amdgcn_readfirstlane(__float_as_uint(trow[0])));
  const float tgw = __uint_as_float(__builtin_amdgcn_readfirstlane(__float_as_uint(trow[2])));
  const float tgy = __uint_as_float(__builtin_amdgcn_readfirstlane(__float_as_uint(trow[3])));
  float* const m_csq = reinterpret_cast<float*>(smem + L::kMeta);
  float* const m_y = m_csq + kRMaxCand;
  int* const gidx = reinterpret_cast<int*>(smem + L::kGidx);
  float* const lds_ca = reinterpret_cast<float*>(smem + L::kRes);
  float* const lds_cb = lds_ca + kRDim;
  const unsigned char* const xring = smem + L::kScr + wave * L::kScrWave;
  const int xsw = (r >> 1) & 7;  // swizzle of this lane's row in the x image
  const int csw = (r >> 2) & 3;  // swizzle of this lane's candidate row in the centre image
  const f32x16 zero16 = {};

  for (int T = xlo + slot; T < xhi; T += G8) {
    const int s = __builtin_amdgcn_readfirstlane(tile_seg[T]);
    const int r0 = __builtin_amdgcn_readfirstlane(p.seg_row_off[s]);
    const int r1 = __builtin_amdgcn_readfirstlane(p.seg_row_off[s + 1]);
    const int tb = __builtin_amdgcn_readfirstlane(seg_tiles[s]);
    const int t0 = r0 + (T - tb) * R;
    const int nrows = min(R, r1 - t0);
    const int cnt = __builtin_amdgcn_readfirstlane(p.cand_count[s]);
    const int cbase = __builtin_amdgcn_readfirstlane(p.cand_base[s]);
    const bool flag = p.seg_flags && (__builtin_amdgcn_readfirstlane(p.seg_flags[s]) & RQSID_SEG_PENALTY);
    const int my_local = wave * 32 + r;
    const bool row_valid = my_local < nrows;
    const bool wave_live = wave * 32 < nrows;
    const int pos = t0 + (row_valid ? my_local : 0);
    const int my_row = p.row_index ? p.row_index[pos] : pos;
    // the row's level-1 divisor, consumed here: a plain load still in flight when the row DMAs start would
    // make hipcc drain them with vmcnt(0) at its first use
    float inv1 = 1.0f;
    if (RL >= 2 && NORM) inv1 = 1.0f / p.den_in[my_row];
    asm volatile("" : "+v"(inv1));
    __syncthreads();  // the previous tile's LDS (ring, meta, candidate ids, residual rows) is consumed
    if (flag || cnt <= 0) {  // block-uniform
      WorkItem w{};
      w.row = my_row;
      w.seg = s;
      w.n = flag ? -2 : -3;
      push_work(p, h == 0 && row_valid, lane, w);
      continue;
    }
    const int nblk = (min(cnt, kRMaxCand) + kCB - 1) / kCB;
    const int NQ = nblk * kRNch;  // ring steps: (candidate block, chunk)
    for (int k = tid; k < nblk * kCB; k += W * 64) {
      const bool live = k < cnt;
      const int g = cand_global(p, cbase, live ? k : cnt - 1);
      const float2 m = *reinterpret_cast<const float2*>(p.c_meta + 4 * (int64_t)g);  // |c|^2, |c|
      m_csq[k] = live ? m.x : INFINITY;
      m_y[k] = m.y;
      gidx[k] = g;
    }
    if (RL >= 1) {
      const float4* a = reinterpret_cast<const float4*>(p.ca + (int64_t)seg_row(p.seg_ca, s) * kRDim);
      for (int i = tid; i < kRDim / 4; i += W * 64) reinterpret_cast<float4*>(lds_ca)[i] = a[i];
    }
    if (RL >= 2) {
      const float4* a = reinterpret_cast<const float4*>(p.cb + (int64_t)seg_row(p.seg_cb, s) * kRDim);
      for (int i = tid; i < kRDim / 4; i += W * 64) reinterpret_cast<float4*>(lds_cb)[i] = a[i];
    }
    __syncthreads();

    // centre DMA of ring step q (candidate block q/16, chunk q%16) into stage q%S: instruction j of wave w
    // moves the hi halves of candidates (w*P + j)*16 + lane/4 (64 B each; image row k*64, 16-B slot q
    // stored at q ^ ((k>>2)&3): conflict-free fragment reads)
    auto issue = [&](int q) {
      const int blk = q / kRNch, c = q % kRNch;
      if (wave * P >= L::kOps) return;
#pragma unroll
      for (int j = 0; j < P; ++j) {
        const int il = (wave * P + j) * 16 + (lane >> 2);
        const int g = gidx[blk * kCB + il];
        const int sl = (lane & 3) ^ ((il >> 2) & 3);
        const _Float16* src = p.c16h ? reinterpret_cast<const _Float16*>(p.c16h) + (int64_t)g * kRDim + c * 32 + sl * 8
                                     : reinterpret_cast<const _Float16*>(p.c16) + (int64_t)g * 2 * kRDim + c * 64 + sl * 8;
        dma16(src, __builtin_amdgcn_readfirstlane(lds0 + (uint32_t)((q % S) * L::kCStage + (wave * P + j) * 1024)));
      }
    };
#pragma unroll
    for (int q = 0; q < S - 1; ++q)
      if (q < NQ) issue(q);

    // ---- rows -> residual -> fp16 B operand, resident for the tile ----------------------------------
    // the wave's 32 rows stream chunk by chunk through its own SR-stage LDS-DMA ring (fp32 image: row rr at
    // rr*128 B, 16-B slot q stored at q ^ ((rr>>1)&7); instruction i moves rows 8i + lane/8, 8 lanes per
    // 128-B row line, the non-temporal hint) and row_frag turns each chunk into the B operand and the
    // bound's sums, exactly as in the per-tile screen.  The ring is private to the wave: vmcnt alone orders it.
    const float* xsrc[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int rr = 8 * i + (lane >> 3);
      const int grow = __shfl(my_row, rr);
      xsrc[i] = p.x + (int64_t)grow * kRDim + ((lane & 7) ^ ((rr >> 1) & 7)) * 4;
    }
    const uint32_t rbase = lds0 + (uint32_t)(L::kScr + wave * L::kScrWave);
    auto issue_rows = [&](int c) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
        dma16_nt(xsrc[i] + c * 32, __builtin_amdgcn_readfirstlane(rbase + (uint32_t)((c % SR) * 4096 + i * 1024)));
    };
    RowSums rs;
    f16x8 bf[2 * kRNch];
    // this lane's half of the residual centre rows, as opaque bases: the per-chunk offsets then fold into the
    // ds_read immediates (hipcc otherwise turns base + 8h + d into ORs of disjoint bits, materialises every
    // chunk's address and spills them)
    typedef __attribute__((address_space(3))) const float lds_f32;
    lds_f32* ca3 = (lds_f32*)(lds_ca + 8 * h);  // pinned as LDS pointers (a pinned generic pointer
    lds_f32* cb3 = (lds_f32*)(lds_cb + 8 * h);  // would turn the reads into flat loads, which count on vmcnt)
    asm volatile("" : "+v"(ca3), "+v"(cb3));
    const float* ca_h = (const float*)ca3;
    const float* cb_h = (const float*)cb3;
#pragma unroll
    for (int c = 0; c < SR - 1; ++c) issue_rows(c);
#pragma unroll
    for (int c = 0; c < kRNch; ++c) {
      __builtin_amdgcn_sched_barrier(0);  // one chunk at a time (hoisting every chunk's reads spills)
      wait_rows(min(SR - 2, kRNch - 1 - c));  // chunk c landed; the stage chunk c-1 used is read
      if (c + SR - 1 < kRNch) issue_rows(c + SR - 1);
      const unsigned char* xb = xring + (c % SR) * 4096 + r * 128;
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const int q0 = 4 * ks + 2 * h;
        const float4 xa = *reinterpret_cast<const float4*>(xb + ((q0 ^ xsw) << 4));
        const float4 xc = *reinterpret_cast<const float4*>(xb + (((q0 + 1) ^ xsw) << 4));
        f16x8 bl;
        row_frag<RL, NORM, false, true>(xa, xc, ca_h, cb_h, c * 32 + 16 * ks, inv1, bf[2 * c + ks], bl, rs);
      }
    }
    // bound constants of the row (assign_screen_kernel's pass-0 block, 1 term)
    const float se2 = rs.se2v.x + rs.se2v.y, sf2 = rs.sf2v.x + rs.sf2v.y;
    const float en = sqrtf(se2 + __shfl_xor(se2, 32)) * 1.001f + 1e-30f;
    float inv_den = 1.f, dr = 0.f;
    const float nrm = sqrtf(sf2 + __shfl_xor(sf2, 32));
    if (NORM && RL >= 1) {  // RL 2: fp32 sums, |nrm - |v|| <= den_eps |v| (chains of dim/4 + 2 terms)
      const float den = nrm + 1e-8f;
      inv_den = 1.0f / den;
      const float den_eps = (0.125f * (float)kRDim + 3.0f) * 5.97e-8f;
      dr = 4.0f * 2.39e-7f * (1.0f + nrm) * inv_den + 4.0f * 5.97e-8f + 1.01f * den_eps * nrm * inv_den;
    }
    const float vn = nrm * 1.0001f + 1e-30f;
    const float hn = vn + en;
    const float vr = vn * inv_den;
    const float ar = p.acc_rel, k2 = 2.0f * inv_den * 1.000001f;
    const float A = k2 * (en + ar * hn) + 2.0f * dr + 4.8e-7f * vr;
    const float B = k2 * hn * (1.0f + ar);
    const float m2 = -2.0f * inv_den * tscale;
    const float A2 = (A + B * tgw + 2.39e-7f * tgy) * 1.000001f;
    const f2 m2v = {m2, m2}, a2v = {A2, A2}, epsv = {1e-30f, 1e-30f};

    float U = INFINITY;
    int nlist = 0;
    bool ovf = false;
    int lk[kListPerHalf];
    float llb[kListPerHalf];
#pragma unroll
    for (int j = 0; j < kListPerHalf; ++j) {
      lk[j] = -1;
      llb[j] = INFINITY;
    }
    for (int blk = 0; blk < nblk; ++blk) {
      f32x16 acc[NTB];
#pragma unroll
      for (int t = 0; t < NTB; ++t) acc[t] = zero16;
      if (!wave_live) {  // a wave past the tile's rows keeps the ring's waits and DMAs, computes nothing
#pragma unroll
        for (int c = 0; c < kRNch; ++c) {
          const int q = blk * kRNch + c;
          wait_chunks<S, P>(min(S - 2, NQ - 1 - q));
          if (q + S - 1 < NQ) issue(q + S - 1);
        }
        continue;
      }
#pragma unroll
      for (int c = 0; c < kRNch; ++c) {
        const int q = blk * kRNch + c;
        wait_chunks<S, P>(min(S - 2, NQ - 1 - q));  // step q landed (every wave), step q-1 fully read
        if (q + S - 1 < NQ) issue(q + S - 1);       // into the stage step q-1 used
        const unsigned char* cbp = smem + (c % S) * L::kCStage + r * 64;
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
          const int qa = (2 * ks + h) ^ csw;
#pragma unroll
          for (int t = 0; t < NTB; ++t) {
            const f16x8 af = *reinterpret_cast<const f16x8*>(cbp + t * 32 * 64 + (qa << 4));
            acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(af, bf[2 * c + ks], acc[t], 0, 0, 0);
          }
        }
      }
      // sweep 1: ub / lb of the block's candidates (lb kept in the accumulator), U = least ub so far
      const int kb = blk * kCB;
#pragma unroll
      for (int t = 0; t < NTB; ++t) {
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const float4 cs = *reinterpret_cast<const float4*>(m_csq + kb + t * 32 + 8 * g + 4 * h);
          const float4 yy = *reinterpret_cast<const float4*>(m_y + kb + t * 32 + 8 * g + 4 * h);
#pragma unroll
          for (int e = 0; e < 2; ++e) {
            const int v = 4 * g + 2 * e;
            const f2 d = {acc[t][v], acc[t][v + 1]};
            const f2 P2 = m2v * d + (e ? f2{cs.z, cs.w} : f2{cs.x, cs.y});
            const f2 E2 = a2v * (e ? f2{yy.z, yy.w} : f2{yy.x, yy.y}) + epsv;
            const f2 ub = P2 + E2, lb = P2 - E2;
            U = fminf(U, fminf(ub.x, ub.y));
            acc[t][v] = lb.x;
            acc[t][v + 1] = lb.y;
          }
        }
      }
      U = fminf(U, __shfl_xor(U, 32));
      const float Up = fmaf(fabsf(U), 0x1p-22f, U) + 1.2e-38f;
      // listed candidates whose lower bound no longer reaches the shrunken U leave the list (stable)
      {
        int nk = 0;
        int lk2[kListPerHalf];
        float llb2[kListPerHalf];
#pragma unroll
        for (int i = 0; i < kListPerHalf; ++i) {
          lk2[i] = -1;
          llb2[i] = INFINITY;
        }
#pragma unroll
        for (int j = 0; j < kListPerHalf; ++j) {
          const bool keep = j < nlist && llb[j] <= Up;
#pragma unroll
          for (int i = 0; i < kListPerHalf; ++i) {
            const bool put = keep && nk == i;
            lk2[i] = put ? lk[j] : lk2[i];
            llb2[i] = put ? llb[j] : llb2[i];
          }
          nk += keep ? 1 : 0;
        }
#pragma unroll
        for (int i = 0; i < kListPerHalf; ++i) {
          lk[i] = lk2[i];
          llb[i] = llb2[i];
        }
        nlist = nk;
      }
      // sweep 2: list (ascending) the block's candidates whose lower bound is <= U
#pragma unroll
      for (int t = 0; t < NTB; ++t) {
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int v = 0; v < 16; ++v) {
          const int kl = kb + t * 32 + (v & 3) + 8 * (v >> 2) + 4 * h;
          const float lb = acc[t][v];
          const bool q = lb <= Up && kl < cnt;
          if (__builtin_amdgcn_ballot_w64(q)) {  // wave-uniform skip: most candidates qualify for no row
            ovf = ovf || (q && nlist >= kListPerHalf);
#pragma unroll
            for (int j = 0; j < kListPerHalf; ++j) {
              const bool take = q && nlist == j;
              lk[j] = take ? kl : lk[j];
              llb[j] = take ? lb : llb[j];
            }
            nlist += (q && nlist < kListPerHalf) ? 1 : 0;
          }
        }
      }
    }
    if (!wave_live) continue;
    // row decision (assign_screen_kernel's multi-pass form): the listed candidates still within the final
    // U; an overflowing half, a non-finite bound or no candidate -> re-score every candidate
    const float Uf = fmaf(fabsf(U), 0x1p-22f, U) + 1.2e-38f;
    ovf = ovf || !(U < INFINITY);
    int nh = 0;
    int kk[kListPerHalf];
#pragma unroll
    for (int j = 0; j < kListPerHalf; ++j) {
      const bool keep = j < nlist && llb[j] <= Uf;
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
      p.out_global[my_row] = gidx[k];
    }
    WorkItem w{};
    w.row = my_row;
    w.seg = s;
    if (overflow) {
      w.n = -1;
    } else {
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
      w.n = ncand;
    }
    push_work(p, h == 0 && row_valid && !definitive, lane, w);
  }
}

template <int W, int S, int SR, int NTB, int RL, bool NORM>
bool launch_rows_one(const AssignParams& p, const int32_t* tile_seg, const int32_t* seg_tiles, hipStream_t st) {
  using L = RowsLayout<W, S, SR, NTB>;
  static bool attr[kMaxDevices] = {};
  const int dev = current_device(), ncu = device_cu_count();
  if (dev < 0 || !ncu) return false;
  if (!attr[dev]) {
    if (hipFuncSetAttribute((const void*)assign_rows_kernel<W, S, SR, NTB, RL, NORM>,
                            hipFuncAttributeMaxDynamicSharedMemorySize, L::kBytes) != hipSuccess)
      return false;
    attr[dev] = true;
  }
  const int64_t g = (int64_t)ncu * L::kBlocks / 8 * 8;  // persistent: every block resident at once
  hipLaunchKernelGGL((assign_rows_kernel<W, S, SR, NTB, RL, NORM>), dim3((unsigned)(g < 8 ? 8 : g)), dim3(W * 64),
                     L::kBytes, st, p, tile_seg, seg_tiles);
  return true;
}

// block shape RQSID_ROWS_SHAPE = 100 W + 10 S + SR (waves, centre ring stages, per-wave row ring stages):
// 443 (the default) and 482: 4 waves, two blocks per CU (one block's row stream overlaps the other's
// MFMAs); 883: 8 waves, one block per CU (half the centre bytes per row, the row stream exposed)
int rows_shape() {
  const char* e = getenv("RQSID_ROWS_SHAPE");
  const int v = e ? atoi(e) : 443;
  return v == 482 || v == 883 ? v : 443;
}

template <int W, int S, int SR>
bool launch_rows_w(const AssignParams& p, int rl, bool norm, const int32_t* tile_seg, const int32_t* seg_tiles,
                   hipStream_t st) {
  if (rl == 0) return launch_rows_one<W, S, SR, kNTB, 0, false>(p, tile_seg, seg_tiles, st);
  if (rl == 1) return !norm && launch_rows_one<W, S, SR, kNTB, 1, false>(p, tile_seg, seg_tiles, st);
  if (norm) return launch_rows_one<W, S, SR, kNTB, 2, true>(p, tile_seg, seg_tiles, st);
  return launch_rows_one<W, S, SR, kNTB, 2, false>(p, tile_seg, seg_tiles, st);
}

}  // namespace

bool rows_supported(int dim, int cand_count_max, bool t3, int rl, bool norm) {
  return dim == kRDim && !t3 && cand_count_max > 0 && cand_count_max <= kRMaxCand && rl >= 0 && rl <= 2 &&
         !(rl == 1 && norm);
}

int launch_rows_screen(const AssignParams& p, int rl, bool norm, int32_t* tile_seg, int32_t* seg_tiles, int64_t cap,
                       hipStream_t st) {
  const int shape = rows_shape();
  const int R = shape == 883 ? 256 : 128;
  launch_tiling(p, R, tile_seg, seg_tiles, cap, st);
  const bool ok = shape == 883   ? launch_rows_w<8, 8, 3>(p, rl, norm, tile_seg, seg_tiles, st)
                  : shape == 482 ? launch_rows_w<4, 8, 2>(p, rl, norm, tile_seg, seg_tiles, st)
                                 : launch_rows_w<4, 4, 3>(p, rl, norm, tile_seg, seg_tiles, st);
  return ok ? RQSID_OK : fail(RQSID_E_LAUNCH, "assign: row-resident screen launch failed (device query / LDS attribute)");
}

}  // namespace rqsid
