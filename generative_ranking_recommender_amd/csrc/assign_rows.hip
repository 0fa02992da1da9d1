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
#ifndef RQSID_ROWS_BCH
#define RQSID_ROWS_BCH 1
#endif
constexpr int kBCH = RQSID_ROWS_BCH;  // row chunks per load batch (two batches in flight)

template <int W, int S, int BCH, int NTB>
struct RowsLayout {
  static constexpr int kCB = NTB * 32;                // candidates per block (NTB MFMA tiles of 32)
  static constexpr int kCStage = kCB * 64;            // kCB candidates x 32 fp16 dims (hi terms)
  static constexpr int kScr = S * kCStage;            // per-wave transpose scratch: BCH chunks x 32 rows x 64 B
  static constexpr int kScrWave = BCH * 32 * 64;
  static constexpr int kMeta = kScr + W * kScrWave;   // |c|^2 [512], |c| [512]
  static constexpr int kGidx = kMeta + 2 * kRMaxCand * 4;  // global centre of each local candidate [512]
  static constexpr int kRes = kGidx + kRMaxCand * 4;  // residual centre rows ca, cb (fp32 512 each)
  static constexpr int kBytes = kRes + 2 * kRDim * 4;
  static constexpr int kBlocks = W == 4 ? 2 : 1;      // blocks per CU (2 waves per SIMD either way)
  static constexpr int kOps = kCB / 16;               // centre DMA ops per chunk (1 KiB each)
  static constexpr int P = kOps >= W ? kOps / W : 1;  // per issuing wave (waves >= kOps / P issue none)
  static_assert(kOps % W == 0 || W % kOps == 0, "centre DMA split");
  static_assert(kRNch % S == 0, "ring stages must divide the chunks of a block (static stage index)");
  static_assert(kRNch % (2 * BCH) == 0, "row batches (two in flight)");
  static_assert((S - 2) * P <= 63, "vmcnt field");
  static_assert(kBytes * kBlocks <= 160 * 1024, "LDS budget");
};

template <int W, int S, int BCH, int NTB, int RL, bool NORM>
__global__ __launch_bounds__(W * 64, 2) void assign_rows_kernel(AssignParams p, const int32_t* __restrict__ tile_seg,
                                                                const int32_t* __restrict__ seg_tiles) {
  static_assert(!(RL == 1 && NORM), "the first-residual normalising level writes den_out: per-tile kernel");
  using L = RowsLayout<W, S, BCH, NTB>;
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
  unsigned char* const scr = smem + L::kScr + wave * L::kScrWave;
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
        const _Float16* src = reinterpret_cast<const _Float16*>(p.c16) + (int64_t)g * 2 * kRDim + c * 64 + sl * 8;
        dma16(src, __builtin_amdgcn_readfirstlane(lds0 + (uint32_t)((q % S) * L::kCStage + (wave * P + j) * 1024)));
      }
    };
#pragma unroll
    for (int q = 0; q < S - 1; ++q)
      if (q < NQ) issue(q);

    // ---- rows -> residual -> fp16 B operand, resident for the tile ----------------------------------
    // load layout: instruction i moves rows 8i + lane/8 (of this wave's 32), 16 B at dims 4*(lane%8) of a
    // chunk; fragment layout: lane (r, h) holds dims 16 ks + 8 h .. +7 of row r for every k-step ks
    int grow[4];
    float inv1[4];
    float se2[4], sf2[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int lr = 8 * i + (lane >> 3);
      grow[i] = __shfl(my_row, lr);
      inv1[i] = (RL >= 2 && NORM) ? 1.0f / p.den_in[grow[i]] : 1.0f;
      se2[i] = 0.f;
      sf2[i] = 0.f;
    }
    const int q8 = lane & 7;
    f16x8 bf[2 * kRNch];
    typedef __attribute__((ext_vector_type(4))) float v4;
    // two batches of BCH chunks in flight: batch b+1's loads are issued before batch b is converted
    auto load = [&](v4 (&xv)[BCH][4], int c0) {
#pragma unroll
      for (int bc = 0; bc < BCH; ++bc)
#pragma unroll
        for (int i = 0; i < 4; ++i)
          xv[bc][i] = __builtin_nontemporal_load(
              reinterpret_cast<const v4*>(p.x + (int64_t)grow[i] * kRDim + (c0 + bc) * 32 + 4 * q8));
    };
    auto convert = [&](const v4 (&xv)[BCH][4], int c0) {
#pragma unroll
      for (int bc = 0; bc < BCH; ++bc) {
        const int d0 = (c0 + bc) * 32 + 4 * q8;
        float4 a4 = make_float4(0.f, 0.f, 0.f, 0.f), b4 = a4;
        if (RL >= 1) a4 = *reinterpret_cast<const float4*>(lds_ca + d0);
        if (RL >= 2) b4 = *reinterpret_cast<const float4*>(lds_cb + d0);
        const float av[4] = {a4.x, a4.y, a4.z, a4.w}, bv[4] = {b4.x, b4.y, b4.z, b4.w};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          float v[4] = {xv[bc][i].x, xv[bc][i].y, xv[bc][i].z, xv[bc][i].w};
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            if (RL >= 1) v[e] = v[e] - av[e];  // the reference's fp32 operation sequence (row_frag)
            if (RL >= 2) v[e] = (NORM ? v[e] * inv1[i] : v[e]) - bv[e];
          }
          const h2 lo = __builtin_convertvector(f2{v[0], v[1]}, h2);
          const h2 hi = __builtin_convertvector(f2{v[2], v[3]}, h2);
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float ex = v[e] - (float)(e < 2 ? lo[e] : hi[e - 2]);  // exact: the fp16 rounding residual
            se2[i] = fmaf(ex, ex, se2[i]);
            sf2[i] = fmaf(v[e], v[e], sf2[i]);
          }
          // scratch row lr at lr*64 B (32 fp16 dims), 16-B slot q stored at q ^ ((lr>>2)&3)
          const int lr = 8 * i + (lane >> 3);
          typedef __attribute__((ext_vector_type(4))) _Float16 h4;
          const h4 hv = __builtin_shufflevector(lo, hi, 0, 1, 2, 3);
          *reinterpret_cast<h4*>(scr + bc * 2048 + lr * 64 + (((q8 >> 1) ^ ((lr >> 2) & 3)) << 4) + (q8 & 1) * 8) = hv;
        }
      }
      __builtin_amdgcn_wave_barrier();
      asm volatile("" ::: "memory");
#pragma unroll
      for (int bc = 0; bc < BCH; ++bc)
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
          bf[2 * (c0 + bc) + ks] =
              *reinterpret_cast<const f16x8*>(scr + bc * 2048 + r * 64 + (((2 * ks + h) ^ ((r >> 2) & 3)) << 4));
      __builtin_amdgcn_wave_barrier();
      asm volatile("" ::: "memory");
    };
    {
      v4 xa[BCH][4], xb[BCH][4];
      load(xa, 0);
#pragma unroll
      for (int c0 = 0; c0 < kRNch; c0 += 2 * BCH) {
        load(xb, c0 + BCH);
        convert(xa, c0);
        if (c0 + 2 * BCH < kRNch) load(xa, c0 + 2 * BCH);
        convert(xb, c0 + BCH);
      }
    }
    // row sums: the 8 lanes of a row line -> every lane; then lane (r, h) takes row r's
    float e2r = 0.f, f2r = 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      float a = se2[i], b = sf2[i];
#pragma unroll
      for (int o = 1; o < 8; o <<= 1) {
        a += __shfl_xor(a, o);
        b += __shfl_xor(b, o);
      }
      const float ar = __shfl(a, (r & 7) * 8), br = __shfl(b, (r & 7) * 8);
      e2r = (r >> 3) == i ? ar : e2r;
      f2r = (r >> 3) == i ? br : f2r;
    }
    // bound constants of the row (assign_screen_kernel's pass-0 block, 1 term)
    const float en = sqrtf(e2r) * 1.001f + 1e-30f;
    float inv_den = 1.f, dr = 0.f;
    const float nrm = sqrtf(f2r);
    if (NORM && RL >= 1) {  // RL 2: fp32 sums, |nrm - |v|| <= den_eps |v| (chains of <= dim/8 + 3 terms)
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

template <int W, int S, int BCH, int NTB, int RL, bool NORM>
bool launch_rows_one(const AssignParams& p, const int32_t* tile_seg, const int32_t* seg_tiles, hipStream_t st) {
  using L = RowsLayout<W, S, BCH, NTB>;
  static bool attr[kMaxDevices] = {};
  const int dev = current_device(), ncu = device_cu_count();
  if (dev < 0 || !ncu) return false;
  if (!attr[dev]) {
    if (hipFuncSetAttribute((const void*)assign_rows_kernel<W, S, BCH, NTB, RL, NORM>,
                            hipFuncAttributeMaxDynamicSharedMemorySize, L::kBytes) != hipSuccess)
      return false;
    attr[dev] = true;
  }
  const int64_t g = (int64_t)ncu * L::kBlocks / 8 * 8;  // persistent: every block resident at once
  hipLaunchKernelGGL((assign_rows_kernel<W, S, BCH, NTB, RL, NORM>), dim3((unsigned)(g < 8 ? 8 : g)), dim3(W * 64),
                     L::kBytes, st, p, tile_seg, seg_tiles);
  return true;
}

// block shape RQSID_ROWS_SHAPE = 10 W + S: 48 (4 waves, 8 ring stages, two blocks per CU: one block's row
// loads overlap the other's MFMAs; the default), 44 (4 stages) or 88 (8 waves, one block per CU: half the
// centre bytes per row, row loads exposed)
int rows_shape() {
  const char* e = getenv("RQSID_ROWS_SHAPE");
  const int v = e ? atoi(e) : 48;
  return v == 44 || v == 88 ? v : 48;
}

template <int W, int S>
bool launch_rows_w(const AssignParams& p, int rl, bool norm, const int32_t* tile_seg, const int32_t* seg_tiles,
                   hipStream_t st) {
  if (rl == 0) return launch_rows_one<W, S, kBCH, kNTB, 0, false>(p, tile_seg, seg_tiles, st);
  if (rl == 1) return !norm && launch_rows_one<W, S, kBCH, kNTB, 1, false>(p, tile_seg, seg_tiles, st);
  if (norm) return launch_rows_one<W, S, kBCH, kNTB, 2, true>(p, tile_seg, seg_tiles, st);
  return launch_rows_one<W, S, kBCH, kNTB, 2, false>(p, tile_seg, seg_tiles, st);
}

}  // namespace

bool rows_supported(int dim, int cand_count_max, bool t3, int rl, bool norm) {
  return dim == kRDim && !t3 && cand_count_max > 0 && cand_count_max <= kRMaxCand && rl >= 0 && rl <= 2 &&
         !(rl == 1 && norm);
}

int launch_rows_screen(const AssignParams& p, int rl, bool norm, int32_t* tile_seg, int32_t* seg_tiles, int64_t cap,
                       hipStream_t st) {
  const int shape = rows_shape();
  const int R = shape == 88 ? 256 : 128;
  launch_tiling(p, R, tile_seg, seg_tiles, cap, st);
  const bool ok = shape == 88   ? launch_rows_w<8, 8>(p, rl, norm, tile_seg, seg_tiles, st)
                  : shape == 44 ? launch_rows_w<4, 4>(p, rl, norm, tile_seg, seg_tiles, st)
                                : launch_rows_w<4, 8>(p, rl, norm, tile_seg, seg_tiles, st);
  return ok ? RQSID_OK : fail(RQSID_E_LAUNCH, "assign: row-resident screen launch failed (device query / LDS attribute)");
}

}  // namespace rqsid
