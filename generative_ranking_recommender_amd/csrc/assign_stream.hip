// assign_stream.hip — the persistent, cross-tile pipelined screening kernel (rqsid_assign's fast path
// for single-pass segments of 512-d rows: every segment has <= NT*32 candidates).
//
// Same arithmetic as assign.hip's assign_screen_kernel<..., ONE = true> (fp16 MFMA screen, the
// collapsed per-candidate bound, pass bit masks, fp64 re-score of ambiguous rows), different data
// movement:
//  * One persistent 8-wave block per CU walks an XCD-contiguous run of 256-row tiles (twice the
//    rows per centre image of the per-tile kernel: the centre stream costs HBM-side bandwidth, see
//    tools/probe/dma_probe2.hip).  The LDS-DMA ring (kSS = 3 stages of 32-dim chunks: x 32 KiB with
//    the non-temporal hint + centres 2*NT KiB [+ lo 2*NT KiB]) never drains at a tile boundary: the
//    last two chunk slots of tile j already stream tile j+1's first chunks, so tile j's epilogue
//    (VALU only) overlaps tile j+1's HBM traffic.
//  * Tile j+1's header is fetched during tile j in two DMA levels (row / candidate indices and the
//    residual centre rows; then the candidates' |c|^2, |c| and the rows' den_in), counted on the same
//    vmcnt as the ring (every wait below is a counted vmcnt(N) for the exact number of younger ops).
//  * Outputs are written by a FIXED number of stores per wave (out_local, out_global [, den_out];
//    dummy targets for inactive lanes) so the next tile's counted waits stay exact; rows that need
//    the fp64 re-score get out_global = -2 and their work item at work[row] (a conditional store can
//    only make a later counted wait stronger, never weaker); a compaction pass lists them.
#include "assign_common.h"

#ifdef RQSID_STAMPS
__device__ unsigned long long g_stamps[8];  // (diagnostic build, see assign_common.h)
#endif

namespace rqsid {
namespace {

constexpr int kSC = 32;                   // dims per chunk (128-B row pieces: gathered rows stream at full rate)
constexpr int kSDim = 512;                // the stream kernel's row width
constexpr int kNch = kSDim / kSC;         // chunks per tile
constexpr int kSentinel = -2;             // out_global of a row left to the re-score

// W waves per block (32 rows each), S ring stages.  Shapes: 8 x 3 (one block per CU) and 4 x 2 (two
// blocks per CU: the other block's compute / epilogue covers this one's ring refill).
template <int NT, int RL, bool NORM, bool T3, int W, int S>
struct StreamLayout {
  static constexpr int kSR = W * 32;                              // rows per tile
  static constexpr int kSX = kSR * kSC * 4;                       // x stage: kSR rows x 128 B
  static constexpr int kCI = 2 * NT / W;                          // centre DMA ops per wave per table
  static constexpr int kCen = NT * 32 * kSC * 2;                  // one fp16 centre table image: NT*32 x 64 B
  static constexpr int kStage = kSX + kCen * (T3 ? 2 : 1);
  static constexpr int kRes = S * kStage;                         // [2 parities][RL rows] fp32 512
  static constexpr int kSoa = kRes + 2 * RL * kSDim * 4;          // [2 parities][csq | y][NT*32] f32
  static constexpr int kCidx = kSoa + 2 * 2 * NT * 32 * 4;        // [2 parities][NT*32] i32
  static constexpr int kLand = kCidx + 2 * NT * 32 * 4;           // [W waves][32] i32 (row idx, then den)
  static constexpr int kBytes = kLand + W * 32 * 4;
  static constexpr int kBlocks = W == 8 ? 1 : 2;                  // blocks per CU
  static constexpr int P = 4 + kCI * (T3 ? 2 : 1);                // ring DMA ops per chunk per wave
  static constexpr int E = 2 + (RL == 1 && NORM ? 1 : 0);         // fixed epilogue stores per wave
  static constexpr int H1 = 2 + (RL >= 1 ? 1 : 0);                // header level-1 DMA ops per wave
  static constexpr int H2 = 2 + (RL == 2 ? 1 : 0);                // header level-2 DMA ops per wave
  static constexpr int C1 = 2;                                    // chunk step issuing header level 1
  static constexpr int C2 = C1 + S;                               // ... reading it, issuing level 2
  static constexpr int C3 = C2 + S;                               // ... reading level 2
  static_assert(S >= 2 && C3 < kNch, "header steps must fit one tile");
  static_assert((2 * NT) % W == 0 && NT / 2 <= W && (RL < 2 || W >= 4), "header DMA: one op per wave");
  static_assert((S - 1) * P + E + H1 + H2 <= 63, "vmcnt field is 6 bits");
  static_assert(kBytes * kBlocks <= 160 * 1024, "LDS budget");
};

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

// s_load_dword issued from asm: an SMEM load (lgkmcnt), invisible to hipcc's vmcnt bookkeeping and
// never turned into a vector load.  The value is read only after a later wait_barrier (its
// lgkmcnt(0)) and an SGPR_PIN.
__device__ __forceinline__ int sload(const void* ptr) {
  const uint64_t a = reinterpret_cast<uint64_t>(ptr);  // uniform by construction; say so to hipcc
  const uint64_t u = ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(a >> 32)) << 32) |
                     (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)a);
  int v;
  asm volatile("s_load_dword %0, %1, 0x0" : "=s"(v) : "s"(u) : "memory");
  return v;
}
// (a macro, not a function taking int&: through a reference hipcc loses track of the SGPR)
#define SGPR_PIN(v) asm volatile("" : "+s"(v))

struct TileHdr {  // block-uniform (SGPRs)
  int T, s, t0, nrows, cnt, cbase, ca_row, cb_row;
  bool pen;   // penalty segment or no candidates: no screen, work items only
  bool flag;  // RQSID_SEG_PENALTY
};

__device__ __forceinline__ int uni(int v) { return __builtin_amdgcn_readfirstlane(v); }

template <int R>
__device__ __forceinline__ TileHdr tile_header(const AssignParams& p, const int32_t* tile_seg,
                                               const int32_t* seg_tiles, int T) {
  TileHdr H;
  H.T = T;
  H.s = uni(tile_seg[T]);
  const int s = H.s;
  const int r0 = uni(p.seg_row_off[s]), r1 = uni(p.seg_row_off[s + 1]), tb = uni(seg_tiles[s]);
  H.t0 = r0 + (T - tb) * R;
  H.nrows = min(R, r1 - H.t0);
  H.cnt = uni(p.cand_count[s]);
  H.cbase = uni(p.cand_base[s]);
  H.flag = p.seg_flags && (uni(p.seg_flags[s]) & RQSID_SEG_PENALTY);
  H.pen = H.flag || H.cnt <= 0;
  H.ca_row = p.seg_ca ? uni(p.seg_ca[s]) : s;
  H.cb_row = p.seg_cb ? uni(p.seg_cb[s]) : s;
  return H;
}

template <int NT, int RL, bool NORM, bool T3, int W, int S>
__global__ __launch_bounds__(W * 64, 2) void assign_stream_kernel(AssignParams p, const int32_t* tile_seg,
                                                                 const int32_t* seg_tile256) {
  using L = StreamLayout<NT, RL, NORM, T3, W, S>;
  constexpr int P = L::P;
  constexpr int kSS = S, kSR = L::kSR, kSX = L::kSX, kCI = L::kCI;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
#ifndef RQSID_AB_NO_FLUSH
  asm volatile("s_setreg_imm32_b32 hwreg(HW_REG_MODE, 6, 2), 0");  // fp16/fp64 denormals flushed (to_f16)
#endif
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = uni(tid >> 6);
  const int h = lane >> 5, r = lane & 31;
  const uint32_t lds0 = lds_addr(smem);

  // XCD-contiguous tile runs: block b runs on XCD b % 8; the G/8 blocks of an XCD walk one eighth of
  // the tile space together, so a segment's tiles (and its candidate centres) stay in one L2.
  const int ntiles = uni(seg_tile256[p.n_segments]);
  const int G8 = (int)(gridDim.x >> 3), xcd = (int)(blockIdx.x & 7), slot = (int)(blockIdx.x >> 3);
  const int xlo = (int)((int64_t)xcd * ntiles / 8), xhi = (int)((int64_t)(xcd + 1) * ntiles / 8);
  int T = xlo + slot;
  if (T >= xhi) return;

  // table-wide bound constants (meta row k)
  const float* trow = p.c_meta + 4 * (int64_t)p.n_centers;
  const float tscale = __uint_as_float(uni(__float_as_uint(trow[0])));
  const float tgz = __uint_as_float(uni(__float_as_uint(trow[1])));
  const float tgw = __uint_as_float(uni(__float_as_uint(trow[2])));
  const float tgy = __uint_as_float(uni(__float_as_uint(trow[3])));
  int* const dummy = p.work_count + 16;                 // sink of the fixed-count stores

  // ---- header pipeline pieces -------------------------------------------------------------
  // level 1: row indices (wave w: rows 32w..32w+31, lanes 0..31), candidate indices (wave w:
  // candidates (w % (NT/2))*64 + lane; later waves repeat), residual centre rows (RL >= 1)
  auto hdr_level1 = [&](const TileHdr& H, int par) {
    const int lr = min(32 * wave + r, H.nrows - 1);
    if (lane < 32)  // (exec-masked: still one vector-memory op of this wave)
      dma4(p.row_index ? (const void*)(p.row_index + H.t0 + lr) : (const void*)p.seg_row_off,
           uni(lds0 + L::kLand + wave * 128));
    const int k = (wave % (NT / 2)) * 64 + lane;
    const int kc = H.cnt > 0 ? min(k, H.cnt - 1) : 0;
    dma4(p.cand_idx && H.cnt > 0 ? (const void*)(p.cand_idx + H.cbase + kc) : (const void*)p.seg_row_off,
         uni(lds0 + L::kCidx + par * NT * 128 + (wave % (NT / 2)) * 256));
    if (RL >= 1) {  // RL1: ca halves by wave parity; RL2: waves w%4 = 0,1 ca, 2,3 cb (the rest repeat)
      const int half = wave & 1;
      const bool second = RL == 2 && (wave & 2);
      const float* src = second ? p.cb + (int64_t)H.cb_row * kSDim : p.ca + (int64_t)H.ca_row * kSDim;
      dma16(src + half * 256 + lane * 4,
            uni(lds0 + L::kRes + (par * RL + (second ? 1 : 0)) * kSDim * 4 + half * 1024));
    }
  };
  // read level 1 (after the barrier that retires it): this wave's row ids and DMA sources of the tile
  // DMA sources as 32-bit indices of 16-B units (row*128 + slot, candidate*64 + slot): the 64-bit
  // address is one v_mad_u64_u32 per DMA, and a tile's sources cost 4 + NT/4 VGPRs, not twice that.
  // Every DMA instruction moves whole 128-B row lines (8 lanes per row) or 64-B candidate pieces
  // (4 lanes per candidate): fragment-shaped (16-B-per-row) DMAs double the address-path work.
  struct Next {
    uint32_t xi[4];
    uint32_t ci[kCI];
    int my_row;
    float inv1;
  };
  auto cand_of = [&](const TileHdr& H, int par, int k) -> int {  // global centre of local candidate k
    if (H.pen) return 0;
    if (!p.cand_idx) return H.cbase + min(k, H.cnt - 1);
    return reinterpret_cast<const int*>(smem + L::kCidx + par * NT * 128)[min(k, NT * 32 - 1)];
  };
  auto hdr_read1 = [&](const TileHdr& H, int par, Next& n) {
    const int* land = reinterpret_cast<const int*>(smem + L::kLand + wave * 128);
    auto row_of = [&](int lr) {  // lr: row within this wave's 32
      return p.row_index ? land[lr] : H.t0 + min(32 * wave + lr, H.nrows - 1);
    };
    n.my_row = row_of(r);
    // x image of wave w (4 KiB per stage): row rr at rr*128 B, 16-B slot q stored at q ^ ((rr>>1)&7)
    // (conflict-free fragment reads); instruction i moves rows 8i + lane/8, physical slot lane%8
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int lr = 8 * i + (lane >> 3);
      const int sl = (lane & 7) ^ ((lr >> 1) & 7);
      n.xi[i] = (uint32_t)row_of(lr) * 128u + (uint32_t)sl;
    }
    // centre image: candidate k at k*64 B, slot q stored at q ^ ((k>>2)&3); instruction j of wave w
    // moves candidates (w*NT/4 + j)*16 + lane/4, physical slot lane%4 (sources: 2-KiB c16 rows)
#pragma unroll
    for (int j = 0; j < kCI; ++j) {
      const int k = (wave * kCI + j) * 16 + (lane >> 2);
      const int sl = (lane & 3) ^ ((k >> 2) & 3);
      n.ci[j] = (uint32_t)cand_of(H, par, k) * 128u + (uint32_t)sl;
    }
  };
  // level 2: |c|^2 and |c| of the candidates (SoA, gathered from meta), den_in of the rows (RL2 NORM)
  auto hdr_level2 = [&](const TileHdr& H, int par, const Next& n) {
    const int k = (wave % (NT / 2)) * 64 + lane;
    const float* m = p.c_meta + 4 * (int64_t)cand_of(H, par, k);
    dma4(m, uni(lds0 + L::kSoa + (par * 2 + 0) * NT * 128 + (wave % (NT / 2)) * 256));
    dma4(m + 1, uni(lds0 + L::kSoa + (par * 2 + 1) * NT * 128 + (wave % (NT / 2)) * 256));
    if (RL == 2 && lane < 32)
      dma4(NORM ? (const void*)(p.den_in + n.my_row) : (const void*)p.seg_row_off, uni(lds0 + L::kLand + wave * 128));
  };
  auto hdr_read2 = [&](Next& n) {
    if (RL == 2 && NORM) n.inv1 = 1.0f / reinterpret_cast<const float*>(smem + L::kLand + wave * 128)[r];
    else n.inv1 = 1.0f;
  };

  // ---- ring ------------------------------------------------------------------------------------
  const char* const xbase = reinterpret_cast<const char*>(p.x);
  const char* const cbase16 = reinterpret_cast<const char*>(p.c16);
  auto addr = [](const char* base, uint32_t unit) -> const void* {  // base + 16 unit (v_mad_u64_u32)
    return base + (uint64_t)unit * 16u;
  };
  auto issue = [&](const Next& n, int c, int st) {
    const uint32_t sb = lds0 + st * L::kStage;
    const char* xb = xbase + c * (kSC * 4);
#pragma unroll
    for (int i = 0; i < 4; ++i) dma16_nt(addr(xb, n.xi[i]), uni(sb + wave * 4096 + i * 1024));
    const char* cb = cbase16 + c * (kSC * 4);  // c16 row: per chunk 64 B hi then 64 B lo
#pragma unroll
    for (int j = 0; j < kCI; ++j) dma16(addr(cb, n.ci[j]), uni(sb + kSX + (wave * kCI + j) * 1024));
    if (T3) {
      const char* cl = cb + kSC * 2;
#pragma unroll
      for (int j = 0; j < kCI; ++j)
        dma16(addr(cl, n.ci[j]), uni(sb + kSX + L::kCen + (wave * kCI + j) * 1024));
    }
  };

  // ---- first tile: synchronous header --------------------------------------------------------
  TileHdr Hc = tile_header<kSR>(p, tile_seg, seg_tile256, T);
  Next cur{};
  hdr_level1(Hc, 0);
  wait_barrier<0>();
  hdr_read1(Hc, 0, cur);
  hdr_level2(Hc, 0, cur);
  wait_barrier<0>();
  hdr_read2(cur);
#pragma unroll
  for (int c = 0; c < kSS - 1; ++c) issue(cur, c, c);

  const f32x16 zero16 = {};
  bool first = true;
  int par = 0;
  int qb = 0;  // ring stage of this tile's chunk 0 (kNch % kSS != 0: the stage walks on across tiles)
  ST(uint64_t st_wait = 0; uint64_t st_epi = 0; uint64_t st_issue = 0; uint64_t st_hdr = 0; const uint64_t st_begin = ST_NOW();)
  for (;;) {
    const int Tn = T + G8;
    const bool more = Tn < xhi;
    TileHdr Hn{};
    Next nxt{};
    // raw header words of the next tile (SMEM loads in flight; plain scalars so they stay in SGPRs)
    int sN = 0, w_r0 = 0, w_r1 = 0, w_tb = 0, w_cnt = 0, w_cb = 0, w_fl = 0, w_ca = 0, w_cbr = 0;

    f32x16 acc[NT];
    f32x16 accl[T3 ? NT : 1];
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[t] = zero16;
#pragma unroll
    for (int t = 0; t < (T3 ? NT : 1); ++t) accl[t] = zero16;
    RowSums rs;
    const float* lds_ca = reinterpret_cast<const float*>(smem + L::kRes + (par * RL + 0) * kSDim * 4);
    const float* lds_cb = reinterpret_cast<const float*>(smem + L::kRes + (par * RL + (RL == 2 ? 1 : 0)) * kSDim * 4);
    const float inv1 = cur.inv1;
    const int xsw = (r >> 1) & 7;  // x image swizzle of this lane's row
    const int csw = (r >> 2) & 3;  // centre image swizzle of this lane's candidate rows

#pragma unroll 1
    for (int c = 0; c < kNch; ++c) {
      // wait for chunk c: the younger ops are chunks c+1 .. c+S-2 and the groups issued after chunk c.
      // After the first tile, chunk S-1 was issued at the start of the previous epilogue, before its E
      // stores: c = 0 sees chunks 1 .. S-1 + E, c = 1 .. S-1 see S-2 chunks + E.  Header level 1
      // (issued at step C1) is younger than chunks C1+1 .. C1+S-1, level 2 (step C2) than chunks
      // C2+1 .. C2+S-1.  The barrier then also frees stage (c-1) % S.
      constexpr int YP = (S - 2) * P;  // the S-2 chunks issued after chunk c
      ST(const uint64_t st_w0 = ST_NOW();)
      if (more || c + S - 2 < kNch) {
        if (!first && c == 0) wait_barrier<(S - 1) * P + L::E>();
        else if (!first && c <= S - 1) wait_barrier<YP + L::E>();
        else if (c > L::C1 && c <= L::C1 + S - 1 && more) wait_barrier<YP + L::H1>();
        else if (c > L::C2 && c <= L::C2 + S - 1 && more) wait_barrier<YP + L::H2>();
        else wait_barrier<YP>();
      } else {
        wait_barrier<0>();
      }
      ST(st_wait += ST_NOW() - st_w0;)
      const int st = (qb + c) % kSS;
      ST(const uint64_t st_i0 = ST_NOW();)
      if (c + kSS - 1 < kNch) {
        if (first || c != 0) issue(cur, c + kSS - 1, (qb + c + kSS - 1) % kSS);
      } else if (more) {
        issue(nxt, c + kSS - 1 - kNch, (qb + c + kSS - 1) % kSS);
      }
      ST(const uint64_t st_h0 = ST_NOW(); st_issue += st_h0 - st_i0;)
      if (more) {
        if (c == 0) sN = sload(tile_seg + Tn);
        if (c == 1) {  // this iteration's wait_barrier retired the tile_seg load (lgkmcnt(0))
          SGPR_PIN(sN);
          w_r0 = sload(p.seg_row_off + sN);
          w_r1 = sload(p.seg_row_off + sN + 1);
          w_tb = sload(seg_tile256 + sN);
          w_cnt = sload(p.cand_count + sN);
          w_cb = sload(p.cand_base + sN);
          if (p.seg_flags)  // the aligned dword holding byte sN
            w_fl = sload(reinterpret_cast<const void*>(reinterpret_cast<uintptr_t>(p.seg_flags + sN) & ~(uintptr_t)3));
          if (p.seg_ca) w_ca = sload(p.seg_ca + sN);
          if (p.seg_cb) w_cbr = sload(p.seg_cb + sN);
        }
        if (c == L::C1) {  // ... and this one the segment words
          SGPR_PIN(w_r0); SGPR_PIN(w_r1); SGPR_PIN(w_tb); SGPR_PIN(w_cnt);
          SGPR_PIN(w_cb); SGPR_PIN(w_fl); SGPR_PIN(w_ca); SGPR_PIN(w_cbr);
          Hn.T = Tn;
          Hn.s = sN;
          Hn.t0 = w_r0 + (Tn - w_tb) * kSR;
          Hn.nrows = min(kSR, w_r1 - Hn.t0);
          Hn.cnt = w_cnt;
          Hn.cbase = w_cb;
          Hn.flag = p.seg_flags && ((w_fl >> (8 * (sN & 3))) & RQSID_SEG_PENALTY);
          Hn.pen = Hn.flag || Hn.cnt <= 0;
          Hn.ca_row = p.seg_ca ? w_ca : sN;
          Hn.cb_row = p.seg_cb ? w_cbr : sN;
          hdr_level1(Hn, par ^ 1);
        }
        if (c == L::C2) {  // level 1 retired by this step's wait
          hdr_read1(Hn, par ^ 1, nxt);
          hdr_level2(Hn, par ^ 1, nxt);
        }
        if (c == L::C3) hdr_read2(nxt);
      }
      ST(st_hdr += ST_NOW() - st_h0;)
#if RQSID_AB_MODE < 3
      // compute chunk c (dims 32c .. 32c+31) in two k-steps: lane (r, h) owns row r of its wave and
      // dims 32c + 16ks + 8h + 0..7 (the per-tile kernel's fragment layout)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
      const unsigned char* xb = smem + st * L::kStage + (32 * wave + r) * 128;
      const int q0 = 4 * ks + 2 * h;
      const float4 xa = *reinterpret_cast<const float4*>(xb + ((q0 ^ xsw) << 4));
      const float4 xc = *reinterpret_cast<const float4*>(xb + (((q0 + 1) ^ xsw) << 4));
      const int d0 = c * kSC + 16 * ks + 8 * h;
      f16x8 bf, bl = {};
      row_frag<RL, NORM, T3, true>(xa, xc, lds_ca, lds_cb, d0, inv1, bf, bl, rs);
      const unsigned char* cimg = smem + st * L::kStage + kSX + r * 64 + (((2 * ks + h) ^ csw) << 4);
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        const f16x8 af = *reinterpret_cast<const f16x8*>(cimg + t * 32 * 64);
#if RQSID_AB_MODE >= 2
        acc[t][0] += (float)bf[0] + (float)af[0];
#else
        acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(af, bf, acc[t], 0, 0, 0);
        if (T3) {
          const f16x8 al = *reinterpret_cast<const f16x8*>(cimg + L::kCen + t * 32 * 64);
          accl[T3 ? t : 0] = __builtin_amdgcn_mfma_f32_32x32x16_f16(af, bl, accl[T3 ? t : 0], 0, 0, 0);
          accl[T3 ? t : 0] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, bf, accl[T3 ? t : 0], 0, 0, 0);
        }
#endif
      }
      }  // ks
#endif
    }

    // the next tile's chunk 2 goes into chunk 15's stage as soon as every wave is done with it, so
    // three chunks stream during the epilogue (VALU only) instead of two
    ST(const uint64_t st_e0 = ST_NOW();)
    if (more) {
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
      issue(nxt, kSS - 1, (qb + kNch - 1) % kSS);
    }
    // ---- epilogue (tile T): the single-pass bound of assign_screen_kernel<..., ONE> ----------
    const bool row_valid = 32 * wave + r < Hc.nrows;
    const int my_row = cur.my_row;
    float inv_den = 1.f, dr = 0.f, vn, en, en2 = 0.f;
    {
      const float se2 = rs.se2v.x + rs.se2v.y, sf2 = rs.sf2v.x + rs.sf2v.y;
      en = sqrtf(se2 + __shfl_xor(se2, 32)) * 1.001f + 1e-30f;
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
        if (RL == 1) {  // fixed-count store (dummy target for the other half / padding rows)
          float* dst = (h == 0 && row_valid) ? p.den_out + my_row : reinterpret_cast<float*>(dummy);
          *dst = den;
        }
        // RL2 also: the fp32 denominator's error, |v/den' - v/den| <= den_eps |v| / den'
        const float den_eps = (0.125f * (float)(kSDim) + 3.0f) * 5.97e-8f;
        dr = RL == 1 ? 2.0f * 5.97e-8f
                     : (4.0f * 2.39e-7f * (1.0f + nrm) * inv_den + 4.0f * 5.97e-8f + 1.01f * den_eps * nrm * inv_den);
      } else {
        nrm = sqrtf(sf2 + __shfl_xor(sf2, 32));
      }
      vn = nrm * 1.0001f + 1e-30f;
    }
    int out_l = kSentinel, out_g = kSentinel;
    bool need = false;
    WorkItem w{};
    w.row = my_row;
    w.seg = Hc.s;
    if (Hc.pen) {
      need = true;
      w.n = Hc.flag ? -2 : -3;
    } else {
#if RQSID_AB_MODE >= 1
      float sink = 0.f;
#pragma unroll
      for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int v = 0; v < 16; ++v) sink += acc[t][v] + (T3 ? accl[T3 ? t : 0][v] : 0.f);
      const int k = sink == -1.2345e38f ? 1 : (int)(((uint32_t)my_row * 2654435761u) >> 8) % Hc.cnt;
      out_l = p.cand_lid ? 0 : k;
      out_g = cand_of(Hc, par, k);
#else
      const float hn = vn + en;
      const float vr = vn * inv_den;
      const float ar = p.acc_rel, ar2 = 2.0f * p.acc_rel, k2 = 2.0f * inv_den * 1.000001f;
      const float A = T3 ? k2 * (en2 + ar * hn + ar2 * (en + en2)) + 2.0f * dr + 7.2e-7f * vr
                         : k2 * (en + ar * hn) + 2.0f * dr + 4.8e-7f * vr;
      const float B = T3 ? k2 * (hn * (1.0f + ar2) + 2.0f * (en + en2)) : k2 * hn * (1.0f + ar);
      const float C = T3 ? k2 * ((en + en2) + ar * hn + ar2 * (hn + en + en2)) : 0.0f;
      const float m2 = -2.0f * inv_den * tscale;
      const float A2 = (A + B * (T3 ? tgz : tgw) + C * tgw + 2.39e-7f * tgy) * 1.000001f;
      const f2 m2v = {m2, m2}, a2v = {A2, A2}, epsv = {1e-30f, 1e-30f};
      const float* m_csq = reinterpret_cast<const float*>(smem + L::kSoa + (par * 2 + 0) * NT * 128);
      const float* m_y = reinterpret_cast<const float*>(smem + L::kSoa + (par * 2 + 1) * NT * 128);
      float U = INFINITY;
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const float4 csq = *reinterpret_cast<const float4*>(m_csq + t * 32 + 8 * g + 4 * h);
          const float4 yy = *reinterpret_cast<const float4*>(m_y + t * 32 + 8 * g + 4 * h);
#pragma unroll
          for (int e = 0; e < 2; ++e) {
            const int v = 4 * g + 2 * e;
            f2 d = {acc[t][v], acc[t][v + 1]};
            if (T3) d = f2{accl[T3 ? t : 0][v], accl[T3 ? t : 0][v + 1]} * 0x1p-12f + d;
            const f2 P2 = m2v * d + (e ? f2{csq.z, csq.w} : f2{csq.x, csq.y});
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
      const f2 upv = {Up, Up};
      uint32_t pbits[NT / 2];
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
      // candidates beyond cnt (duplicates of the last one) never pass
      // (a lane half's candidates ascend with v, so a tile's valid values are a prefix of its 16 bits)
      if (Hc.cnt < NT * 32) {
#pragma unroll
        for (int wd = 0; wd < NT / 2; ++wd) {
          uint32_t m = 0;
#pragma unroll
          for (int q = 0; q < 2; ++q) {
            const int rem = Hc.cnt - 32 * (2 * wd + q) - 4 * h;  // valid iff (v&3) + 8(v>>2) < rem
            int nv = 0;
#pragma unroll
            for (int g = 0; g < 4; ++g) nv += min(4, max(0, rem - 8 * g));
            const uint32_t pre = (uint32_t)((0xFFFFull << (16 - nv)) & 0xFFFFull);
            m |= q == 0 ? pre << 16 : pre;
          }
          pbits[wd] &= m;
        }
      }
      int k = -1;
      if (pass_decide(pbits, h, k, w)) {
        out_l = k;
        out_g = cand_of(Hc, par, k);
      } else {
        need = true;
      }
#endif
    }
    {  // fixed-count output stores: exactly E per wave whatever the rows decided
      const bool mine = h == 0 && row_valid;
      int* dl = mine ? p.out_local + my_row : dummy;
      int* dg = mine ? p.out_global + my_row : dummy;
      *dl = out_l;
      *dg = out_g;
    }
    if (need && h == 0 && row_valid) p.work[my_row] = w;  // may only strengthen the next counted waits

    ST(st_epi += ST_NOW() - st_e0;)
    if (!more) break;
    T = Tn;
    Hc = Hn;
    cur = nxt;
    par ^= 1;
    qb = (qb + kNch) % kSS;
    first = false;
  }
#ifdef RQSID_STAMPS
  if (tid == 0) {
    atomicAdd(&g_stamps[0], (unsigned long long)(ST_NOW() - st_begin));
    atomicAdd(&g_stamps[1], (unsigned long long)st_wait);
    atomicAdd(&g_stamps[2], (unsigned long long)st_epi);
    atomicAdd(&g_stamps[3], (unsigned long long)st_issue);
    atomicAdd(&g_stamps[4], (unsigned long long)st_hdr);
  }
#endif
}

// ---- ping-pong form: the 8 waves of the block are two 4-wave groups (waves 0-3: rows 0-127 of the
// 256-row tile, waves 4-7: rows 128-255; one wave of each group per SIMD) that alternate roles every
// phase: while one group runs the MFMAs of chunk j, the other issues its share of the ring's DMAs
// (and the next tile's header loads).  The compute waves never stall on DMA issue (140-200 cycles per
// global_load_lds_dwordx4 under load, tools/stamps.py), and each SIMD runs one computing wave at a
// time.  Phases are barrier-separated; chunk j's centre image is shared by both groups (group 0
// computes it in phase 2j, group 1 in phase 2j+1).
//   phase 2j   : group 0 computes chunk j;   group 1 issues the centres of chunk j+1 and its rows of j+2
//   phase 2j+1 : group 1 computes chunk j;   group 0 issues its rows of chunk j+3
// (rows stream three chunks ahead from HBM, the L2-resident centres one).  Chunk numbers continue across
// tiles (16.. = the next tile's 0..).  LDS: rows [2 groups][3 stages] x 16 KiB, centres [2 stages].
// Group 0 runs its epilogue in phase 31 (after its issue), group 1 in the next tile's phase 0 (after
// its issue); both while the other group computes.
template <int NT, int RL, bool NORM, bool T3>
struct PPLayout {
  static constexpr int kCI = NT / 2;                       // centre DMA ops per group-1 wave per table
  static constexpr int kCen = NT * 32 * kSC * 2;           // one fp16 table image of a chunk
  static constexpr int kCStage = kCen * (T3 ? 2 : 1);
  static constexpr int kXG = 128 * kSC * 4;                // one group's rows of a chunk: 16 KiB
  static constexpr int kX = 0;                             // [2 groups][3 stages]
  static constexpr int kC = kX + 6 * kXG;                  // [2 stages]
  static constexpr int kRes = kC + 2 * kCStage;            // [2 parities][RL rows] fp32 512
  static constexpr int kSoa = kRes + 2 * RL * kSDim * 4;
  static constexpr int kCidx = kSoa + 2 * 2 * NT * 32 * 4;
  static constexpr int kLand = kCidx + 2 * NT * 32 * 4;
  static constexpr int kBytes = kLand + 8 * 32 * 4;
  static constexpr int PC = kCI * (T3 ? 2 : 1);            // centre ops per group-1 wave per chunk
  static constexpr int E = 2 + (RL == 1 && NORM ? 1 : 0);
  static constexpr int H1 = 2 + (RL >= 1 ? 1 : 0);
  static constexpr int H2 = 2 + (RL == 2 ? 1 : 0);
  static constexpr int C1 = 2, C2 = 6, C3 = 10;            // header steps (their phases: see the waits)
  static_assert(kBytes <= 160 * 1024, "LDS budget");
  static_assert(2 * (PC + 4) + E + H1 + H2 <= 63, "vmcnt field is 6 bits");
};

// Scalar loads that complete inside the asm (s_waitcnt lgkmcnt(0) before it returns): their outputs
// are valid SGPRs at once, so hipcc may copy or spill them freely (the ping-pong kernel's header
// steps sit in several inlined phase copies, where an asynchronous load's output would be copied
// before it lands).
__device__ __forceinline__ uint64_t uni64(const void* ptr) {
  const uint64_t a = reinterpret_cast<uint64_t>(ptr);
  return ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(a >> 32)) << 32) |
         (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)a);
}
__device__ __forceinline__ int sload_now(const void* ptr) {
  int v;
  asm volatile("s_load_dword %0, %1, 0x0\n\ts_waitcnt lgkmcnt(0)" : "=s"(v) : "s"(uni64(ptr)) : "memory");
  return v;
}
struct SegWords {
  int r0, r1, tb, cnt, cb, fl, ca, cbr;
};
// segment s's header words (seg_row_off[s], [s+1], seg_tiles[s], cand_count[s], cand_base[s], the
// aligned seg_flags word holding byte s, seg_ca[s], seg_cb[s]; absent arrays read a harmless word)
__device__ __forceinline__ SegWords seg_words(const AssignParams& p, const int32_t* seg_tiles, int s) {
  const void* fl = p.seg_flags ? reinterpret_cast<const void*>(reinterpret_cast<uintptr_t>(p.seg_flags + s) & ~(uintptr_t)3)
                               : (const void*)p.seg_row_off;
  const void* ca = p.seg_ca ? (const void*)(p.seg_ca + s) : (const void*)p.seg_row_off;
  const void* cb = p.seg_cb ? (const void*)(p.seg_cb + s) : (const void*)p.seg_row_off;
  SegWords w;
  asm volatile(
      "s_load_dword %0, %8, 0x0\n\t"
      "s_load_dword %1, %8, 0x4\n\t"
      "s_load_dword %2, %9, 0x0\n\t"
      "s_load_dword %3, %10, 0x0\n\t"
      "s_load_dword %4, %11, 0x0\n\t"
      "s_load_dword %5, %12, 0x0\n\t"
      "s_load_dword %6, %13, 0x0\n\t"
      "s_load_dword %7, %14, 0x0\n\t"
      "s_waitcnt lgkmcnt(0)"
      : "=&s"(w.r0), "=&s"(w.r1), "=&s"(w.tb), "=&s"(w.cnt), "=&s"(w.cb), "=&s"(w.fl),
        "=&s"(w.ca), "=&s"(w.cbr)
      : "s"(uni64(p.seg_row_off + s)), "s"(uni64(seg_tiles + s)), "s"(uni64(p.cand_count + s)),
        "s"(uni64(p.cand_base + s)), "s"(uni64(fl)), "s"(uni64(ca)), "s"(uni64(cb))
      : "memory");
  return w;
}

template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"i"(N) : "memory");
}
__device__ __forceinline__ void lgkm_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

template <int NT, int RL, bool NORM, bool T3>
__global__ __launch_bounds__(512, 2) void assign_pp_kernel(AssignParams p, const int32_t* tile_seg,
                                                           const int32_t* seg_tile256) {
  using L = PPLayout<NT, RL, NORM, T3>;
  constexpr int PC = L::PC, kCI = L::kCI, kSR = 256;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
#ifndef RQSID_AB_NO_FLUSH
  asm volatile("s_setreg_imm32_b32 hwreg(HW_REG_MODE, 6, 2), 0");  // fp16/fp64 denormals flushed (to_f16)
#endif
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = uni(tid >> 6);
  const int grp = wave >> 2, gw = wave & 3;
  const int h = lane >> 5, r = lane & 31;
  const uint32_t lds0 = lds_addr(smem);

  const int ntiles = uni(seg_tile256[p.n_segments]);
  const int G8 = (int)(gridDim.x >> 3), xcd = (int)(blockIdx.x & 7), slot = (int)(blockIdx.x >> 3);
  const int xlo = (int)((int64_t)xcd * ntiles / 8), xhi = (int)((int64_t)(xcd + 1) * ntiles / 8);
  int T = xlo + slot;
  if (T >= xhi) return;

  // table-wide bound constants (meta row k)
  const float* trow = p.c_meta + 4 * (int64_t)p.n_centers;
  const float tscale = __uint_as_float(uni(__float_as_uint(trow[0])));
  const float tgz = __uint_as_float(uni(__float_as_uint(trow[1])));
  const float tgw = __uint_as_float(uni(__float_as_uint(trow[2])));
  const float tgy = __uint_as_float(uni(__float_as_uint(trow[3])));
  int* const dummy = p.work_count + 16;                 // sink of the fixed-count stores
  const uint32_t cunits = (!T3 && p.c16h) ? 64u : 128u;  // 16-B units per centre row of the table gathered
#ifdef RQSID_AB_HALFROW
  constexpr int kXR = 2;  // row DMA ops per wave and chunk (the probe's 64-B fp16 row pieces)
#else
  constexpr int kXR = 4;  // row DMA ops per wave and chunk
#endif

  // ---- header pipeline pieces -------------------------------------------------------------
  // level 1: row indices (wave w: rows 32w..32w+31, lanes 0..31), candidate indices (wave w:
  // candidates (w % (NT/2))*64 + lane; later waves repeat), residual centre rows (RL >= 1)
  auto hdr_level1 = [&](const TileHdr& H, int par) {
    const int lr = min(32 * wave + r, H.nrows - 1);
    if (lane < 32)  // (exec-masked: still one vector-memory op of this wave)
      dma4(p.row_index ? (const void*)(p.row_index + H.t0 + lr) : (const void*)p.seg_row_off,
           uni(lds0 + L::kLand + wave * 128));
    const int k = (wave % (NT / 2)) * 64 + lane;
    const int kc = H.cnt > 0 ? min(k, H.cnt - 1) : 0;
    dma4(p.cand_idx && H.cnt > 0 ? (const void*)(p.cand_idx + H.cbase + kc) : (const void*)p.seg_row_off,
         uni(lds0 + L::kCidx + par * NT * 128 + (wave % (NT / 2)) * 256));
    if (RL >= 1) {  // RL1: ca halves by wave parity; RL2: waves w%4 = 0,1 ca, 2,3 cb (the rest repeat)
      const int half = wave & 1;
      const bool second = RL == 2 && (wave & 2);
      const float* src = second ? p.cb + (int64_t)H.cb_row * kSDim : p.ca + (int64_t)H.ca_row * kSDim;
      dma16(src + half * 256 + lane * 4,
            uni(lds0 + L::kRes + (par * RL + (second ? 1 : 0)) * kSDim * 4 + half * 1024));
    }
  };
  // read level 1 (after the barrier that retires it): this wave's row ids and DMA sources of the tile
  // DMA sources as 32-bit indices of 16-B units (row*128 + slot, candidate*64 + slot): the 64-bit
  // address is one v_mad_u64_u32 per DMA, and a tile's sources cost 4 + NT/4 VGPRs, not twice that.
  // Every DMA instruction moves whole 128-B row lines (8 lanes per row) or 64-B candidate pieces
  // (4 lanes per candidate): fragment-shaped (16-B-per-row) DMAs double the address-path work.
  struct Next {
    uint32_t xi[4];
    uint32_t ci[kCI];
    int my_row;
    float inv1;
  };
  auto cand_of = [&](const TileHdr& H, int par, int k) -> int {  // global centre of local candidate k
    if (H.pen) return 0;
    if (!p.cand_idx) return H.cbase + min(k, H.cnt - 1);
    return reinterpret_cast<const int*>(smem + L::kCidx + par * NT * 128)[min(k, NT * 32 - 1)];
  };
  auto hdr_read1 = [&](const TileHdr& H, int par, Next& n) {
    const int* land = reinterpret_cast<const int*>(smem + L::kLand + wave * 128);
    auto row_of = [&](int lr) {  // lr: row within this wave's 32
      return p.row_index ? land[lr] : H.t0 + min(32 * wave + lr, H.nrows - 1);
    };
    n.my_row = row_of(r);
    // x image of wave w (4 KiB per stage): row rr at rr*128 B, 16-B slot q stored at q ^ ((rr>>1)&7)
    // (conflict-free fragment reads); instruction i moves rows 8i + lane/8, physical slot lane%8
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int lr = 8 * i + (lane >> 3);
      const int sl = (lane & 7) ^ ((lr >> 1) & 7);
      n.xi[i] = (uint32_t)row_of(lr) * 128u + (uint32_t)sl;
    }
    // centre image: candidate k at k*64 B, slot q stored at q ^ ((k>>2)&3); instruction j of wave w
    // moves candidates (w*NT/4 + j)*16 + lane/4, physical slot lane%4 (sources: 2-KiB c16 rows)
#pragma unroll
    for (int j = 0; j < kCI; ++j) {
      const int k = (gw * kCI + j) * 16 + (lane >> 2);
      const int sl = (lane & 3) ^ ((k >> 2) & 3);
      n.ci[j] = (uint32_t)cand_of(H, par, k) * cunits + (uint32_t)sl;
    }
  };
  // level 2: |c|^2 and |c| of the candidates (SoA, gathered from meta), den_in of the rows (RL2 NORM)
  auto hdr_level2 = [&](const TileHdr& H, int par, const Next& n) {
    const int k = (wave % (NT / 2)) * 64 + lane;
    const float* m = p.c_meta + 4 * (int64_t)cand_of(H, par, k);
    dma4(m, uni(lds0 + L::kSoa + (par * 2 + 0) * NT * 128 + (wave % (NT / 2)) * 256));
    dma4(m + 1, uni(lds0 + L::kSoa + (par * 2 + 1) * NT * 128 + (wave % (NT / 2)) * 256));
    if (RL == 2 && lane < 32)
      dma4(NORM ? (const void*)(p.den_in + n.my_row) : (const void*)p.seg_row_off, uni(lds0 + L::kLand + wave * 128));
  };
  auto hdr_read2 = [&](Next& n) {
    if (RL == 2 && NORM) n.inv1 = 1.0f / reinterpret_cast<const float*>(smem + L::kLand + wave * 128)[r];
    else n.inv1 = 1.0f;
  };

  // ---- ring: this wave's share of chunk j (tile-relative; 16, 17 = the next tile's 0, 1) ----------
  const char* const xbase = reinterpret_cast<const char*>(p.x);
  // the 1-term screen gathers hi pieces: from the hi-only table when present (a 1-KiB row per centre, 64 B per
  // chunk), else from the interleaved table (2 KiB per centre, 128 B per chunk: hi then lo)
  const bool hi_tab = !T3 && p.c16h;
  const char* const cbase16 = reinterpret_cast<const char*>(hi_tab ? p.c16h : p.c16);
  const int cchunk = hi_tab ? kSC * 2 : kSC * 4;  // bytes per chunk of a centre row
  auto addr = [](const char* base, uint32_t unit) -> const void* { return base + (uint64_t)unit * 16u; };
  int qb = 0;  // row stage of this tile's chunk 0 (16 % 3 != 0: walks on across tiles)
  auto issue_c = [&](const Next& n, int j) __attribute__((always_inline)) {  // group 1: chunk j's centres
    const uint32_t sc = lds0 + L::kC + (j & 1) * L::kCStage;
    const char* cb = cbase16 + (j & 15) * cchunk;  // chunk j's piece of every centre row
#pragma unroll
    for (int q = 0; q < kCI; ++q) dma16(addr(cb, n.ci[q]), uni(sc + (gw * kCI + q) * 1024));
    if (T3) {
      const char* cl = cb + kSC * 2;
#pragma unroll
      for (int q = 0; q < kCI; ++q) dma16(addr(cl, n.ci[q]), uni(sc + L::kCen + (gw * kCI + q) * 1024));
    }
  };
  auto issue_x = [&](const Next& n, int j) __attribute__((always_inline)) {  // this group's rows of chunk j
    const uint32_t sx = lds0 + L::kX + (grp * 3 + (qb + j) % 3) * L::kXG + gw * 4096;
    const char* xb = xbase + (j & 15) * (kSC * 4);
#if defined(RQSID_AB_HALFROW)  // (timing probe only, wrong results: the DMA of 1-KiB fp16 rows, 64 B per row and chunk)
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int rr = 16 * i + (lane >> 2);
      const uint32_t xq = (lane >> 5) ? n.xi[2 * i + 1] : n.xi[2 * i];
      const uint32_t row = (uint32_t)__shfl((int)(xq >> 7), (rr & 7) * 8);
      dma16_nt(xbase + (uint64_t)row * 1024u + (j & 15) * 64 + (lane & 3) * 16, uni(sx + i * 1024));
    }
#elif !defined(RQSID_AB_NOROWDMA)  // (NOROWDMA: timing probe only, no row traffic, wrong results)
#pragma unroll
    for (int i = 0; i < 4; ++i) dma16_nt(addr(xb, n.xi[i]), uni(sx + i * 1024));
#endif
  };

  // ---- first tile: synchronous header ----------------------------------------------------------
  TileHdr Hc = tile_header<kSR>(p, tile_seg, seg_tile256, T);
  Next cur{};
  hdr_level1(Hc, 0);
  wait_barrier<0>();
  hdr_read1(Hc, 0, cur);
  hdr_level2(Hc, 0, cur);
  wait_barrier<0>();
  hdr_read2(cur);
  if (grp == 0) {
    issue_x(cur, 0);
    issue_x(cur, 1);
    issue_x(cur, 2);
  } else {
    issue_x(cur, 0);
    issue_c(cur, 0);
    issue_x(cur, 1);
  }

  const f32x16 zero16 = {};
  f32x16 acc[NT];
  f32x16 accl[T3 ? NT : 1];
#pragma unroll
  for (int t = 0; t < NT; ++t) acc[t] = zero16;
#pragma unroll
  for (int t = 0; t < (T3 ? NT : 1); ++t) accl[t] = zero16;
  RowSums rs;
  const int xsw = (r >> 1) & 7;  // x image swizzle of this lane's row
  const int csw = (r >> 2) & 3;  // centre image swizzle of this lane's candidate rows
  int par = 0;
  bool first = true;
  ST(uint64_t st_wait = 0; uint64_t st_comp = 0; uint64_t st_epi = 0; const uint64_t st_begin = ST_NOW();)
  TileHdr Hp{};  // group 1: the tile whose epilogue is still pending
  int row_p = 0, par_p = 0;

  auto epilogue = [&](const TileHdr& H_, int my_row_, int par_) __attribute__((always_inline)) {
      const bool row_valid = 32 * wave + r < H_.nrows;
      const int my_row = my_row_;
      float inv_den = 1.f, dr = 0.f, vn, en, en2 = 0.f;
      {
        const float se2 = rs.se2v.x + rs.se2v.y, sf2 = rs.sf2v.x + rs.sf2v.y;
        en = sqrtf(se2 + __shfl_xor(se2, 32)) * 1.001f + 1e-30f;
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
          if (RL == 1) {  // fixed-count store (dummy target for the other half / padding rows)
            float* dst = (h == 0 && row_valid) ? p.den_out + my_row : reinterpret_cast<float*>(dummy);
            *dst = den;
          }
          // RL2 also: the fp32 denominator's error, |v/den' - v/den| <= den_eps |v| / den'
          const float den_eps = (0.125f * (float)(kSDim) + 3.0f) * 5.97e-8f;
          dr = RL == 1 ? 2.0f * 5.97e-8f
                       : (4.0f * 2.39e-7f * (1.0f + nrm) * inv_den + 4.0f * 5.97e-8f + 1.01f * den_eps * nrm * inv_den);
        } else {
          nrm = sqrtf(sf2 + __shfl_xor(sf2, 32));
        }
        vn = nrm * 1.0001f + 1e-30f;
      }
      int out_l = kSentinel, out_g = kSentinel;
      bool need = false;
      WorkItem w{};
      w.row = my_row;
      w.seg = H_.s;
      if (H_.pen) {
        need = true;
        w.n = H_.flag ? -2 : -3;
      } else {
  #if RQSID_AB_MODE >= 1
        float sink = 0.f;
  #pragma unroll
        for (int t = 0; t < NT; ++t)
  #pragma unroll
          for (int v = 0; v < 16; ++v) sink += acc[t][v] + (T3 ? accl[T3 ? t : 0][v] : 0.f);
        const int k = sink == -1.2345e38f ? 1 : (int)(((uint32_t)my_row * 2654435761u) >> 8) % H_.cnt;
        out_l = p.cand_lid ? 0 : k;
        out_g = cand_of(Hc, par_, k);
  #else
        const float hn = vn + en;
        const float vr = vn * inv_den;
        const float ar = p.acc_rel, ar2 = 2.0f * p.acc_rel, k2 = 2.0f * inv_den * 1.000001f;
        const float A = T3 ? k2 * (en2 + ar * hn + ar2 * (en + en2)) + 2.0f * dr + 7.2e-7f * vr
                           : k2 * (en + ar * hn) + 2.0f * dr + 4.8e-7f * vr;
        const float B = T3 ? k2 * (hn * (1.0f + ar2) + 2.0f * (en + en2)) : k2 * hn * (1.0f + ar);
        const float C = T3 ? k2 * ((en + en2) + ar * hn + ar2 * (hn + en + en2)) : 0.0f;
        const float m2 = -2.0f * inv_den * tscale;
        const float A2 = (A + B * (T3 ? tgz : tgw) + C * tgw + 2.39e-7f * tgy) * 1.000001f;
        const f2 m2v = {m2, m2}, a2v = {A2, A2}, epsv = {1e-30f, 1e-30f};
        const float* m_csq = reinterpret_cast<const float*>(smem + L::kSoa + (par_ * 2 + 0) * NT * 128);
        const float* m_y = reinterpret_cast<const float*>(smem + L::kSoa + (par_ * 2 + 1) * NT * 128);
        float U = INFINITY;
  #pragma unroll
        for (int t = 0; t < NT; ++t) {
          __builtin_amdgcn_sched_barrier(0);
  #pragma unroll
          for (int g = 0; g < 4; ++g) {
            const float4 csq = *reinterpret_cast<const float4*>(m_csq + t * 32 + 8 * g + 4 * h);
            const float4 yy = *reinterpret_cast<const float4*>(m_y + t * 32 + 8 * g + 4 * h);
  #pragma unroll
            for (int e = 0; e < 2; ++e) {
              const int v = 4 * g + 2 * e;
              f2 d = {acc[t][v], acc[t][v + 1]};
              if (T3) d = f2{accl[T3 ? t : 0][v], accl[T3 ? t : 0][v + 1]} * 0x1p-12f + d;
              const f2 P2 = m2v * d + (e ? f2{csq.z, csq.w} : f2{csq.x, csq.y});
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
        const f2 upv = {Up, Up};
        // pass bits: NT independent 16-bit chains (one per candidate tile) the scheduler may interleave, then
        // paired into words (tile 2w in the high half).  One chain through all NT tiles, sched-barriered per tile,
        // was latency-bound on its dependent alignbits: 1.75 ms of the 7.5-ms PROD level 2 (tools/ab_build.sh
        // RQSID_AB_EPI probes)
        uint32_t pbt[NT];
  #pragma unroll
        for (int t = 0; t < NT; ++t) pbt[t] = 0u;
  #pragma unroll
        for (int v = 0; v < 16; v += 2)  // (v outer: the NT chains advance together)
  #pragma unroll
          for (int t = 0; t < NT; ++t) {
            const f2 d = f2{acc[t][v], acc[t][v + 1]} - upv;
            pbt[t] = __builtin_amdgcn_alignbit(pbt[t], __float_as_uint(d.x), 31);
            pbt[t] = __builtin_amdgcn_alignbit(pbt[t], __float_as_uint(d.y), 31);
          }
        uint32_t pbits[NT / 2];
  #pragma unroll
        for (int wd = 0; wd < NT / 2; ++wd) pbits[wd] = (pbt[2 * wd] << 16) | pbt[2 * wd + 1];
        // candidates beyond cnt (duplicates of the last one) never pass
        // (a lane half's candidates ascend with v, so a tile's valid values are a prefix of its 16 bits)
        if (H_.cnt < NT * 32) {
  #pragma unroll
          for (int wd = 0; wd < NT / 2; ++wd) {
            uint32_t m = 0;
  #pragma unroll
            for (int q = 0; q < 2; ++q) {
              const int rem = H_.cnt - 32 * (2 * wd + q) - 4 * h;  // valid iff (v&3) + 8(v>>2) < rem
              int nv = 0;
  #pragma unroll
              for (int g = 0; g < 4; ++g) nv += min(4, max(0, rem - 8 * g));
              const uint32_t pre = (uint32_t)((0xFFFFull << (16 - nv)) & 0xFFFFull);
              m |= q == 0 ? pre << 16 : pre;
            }
            pbits[wd] &= m;
          }
        }
        int k = -1;
#if defined(RQSID_AB_EPI)  // (timing probes only, wrong results: 1 = no pass bits, 2 = no list decision)
        uint32_t px = 0;
        for (int q = 0; q < NT / 2; ++q) px ^= pbits[q];
        if (RQSID_AB_EPI == 1) px = __float_as_uint(Up) | 1u;
        k = __builtin_ctz(px | 0x80000000u);
        if (true) {
#else
        if (pass_decide(pbits, h, k, w)) {
#endif
          out_l = k;
          out_g = cand_of(Hc, par_, k);
        } else {
          need = true;
        }
  #endif
      }
      {  // fixed-count output stores: exactly E per wave whatever the rows decided
        const bool mine = h == 0 && row_valid;
        int* dl = mine ? p.out_local + my_row : dummy;
        int* dg = mine ? p.out_global + my_row : dummy;
        *dl = out_l;
        *dg = out_g;
      }
      if (need && h == 0 && row_valid) p.work[my_row] = w;  // may only strengthen the next counted waits
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[t] = zero16;
#pragma unroll
    for (int t = 0; t < (T3 ? NT : 1); ++t) accl[t] = zero16;
    rs = RowSums{};
  };

  for (;;) {
    const int Tn = T + G8;
    const bool more = Tn < xhi;
    TileHdr Hn{};
    Next nxt{};
    int sN = 0, w_r0 = 0, w_r1 = 0, w_tb = 0, w_cnt = 0, w_cb = 0, w_fl = 0, w_ca = 0, w_cbr = 0;
    const float* lds_ca = reinterpret_cast<const float*>(smem + L::kRes + (par * RL + 0) * kSDim * 4);
    const float* lds_cb = reinterpret_cast<const float*>(smem + L::kRes + (par * RL + (RL == 2 ? 1 : 0)) * kSDim * 4);
    const float inv1 = cur.inv1;
    // header steps of this group's load phases: s = 0 tile_seg, 1 segment words, 2 level 1, 5 level 2, 8 read 2
    auto header_step = [&](int s) __attribute__((always_inline)) {
      if (!more) return;
      if (s == 0) sN = sload_now(tile_seg + Tn);
      if (s == 1) {
        const SegWords sw = seg_words(p, seg_tile256, sN);
        w_r0 = sw.r0; w_r1 = sw.r1; w_tb = sw.tb; w_cnt = sw.cnt;
        w_cb = sw.cb; w_fl = sw.fl; w_ca = sw.ca; w_cbr = sw.cbr;
      }
      if (s == L::C1) {
        Hn.T = Tn;
        Hn.s = sN;
        Hn.t0 = w_r0 + (Tn - w_tb) * kSR;
        Hn.nrows = min(kSR, w_r1 - Hn.t0);
        Hn.cnt = w_cnt;
        Hn.cbase = w_cb;
        Hn.flag = p.seg_flags && ((w_fl >> (8 * (sN & 3))) & RQSID_SEG_PENALTY);
        Hn.pen = Hn.flag || Hn.cnt <= 0;
        Hn.ca_row = p.seg_ca ? w_ca : sN;
        Hn.cb_row = p.seg_cb ? w_cbr : sN;
        hdr_level1(Hn, par ^ 1);
      }
      if (s == L::C2) {  // level 1 of both groups retired and barrier-ordered
        hdr_read1(Hn, par ^ 1, nxt);
        hdr_level2(Hn, par ^ 1, nxt);
      }
      if (s == L::C3) hdr_read2(nxt);
    };
    auto compute = [&](int j) __attribute__((always_inline)) {
#if RQSID_AB_MODE < 3
      const unsigned char* xrow = smem + L::kX + (grp * 3 + (qb + j) % 3) * L::kXG + (32 * gw + r) * 128;
      const unsigned char* cimg0 = smem + L::kC + (j & 1) * L::kCStage + r * 64;
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const int q0 = 4 * ks + 2 * h;
        const float4 xa = *reinterpret_cast<const float4*>(xrow + ((q0 ^ xsw) << 4));
        const float4 xc = *reinterpret_cast<const float4*>(xrow + (((q0 + 1) ^ xsw) << 4));
        const int d0 = j * kSC + 16 * ks + 8 * h;
        f16x8 bf, bl = {};
        row_frag<RL, NORM, T3, true>(xa, xc, lds_ca, lds_cb, d0, inv1, bf, bl, rs);
        const unsigned char* cimg = cimg0 + (((2 * ks + h) ^ csw) << 4);
#pragma unroll
        for (int t = 0; t < NT; ++t) {
          const f16x8 af = *reinterpret_cast<const f16x8*>(cimg + t * 32 * 64);
#if RQSID_AB_MODE >= 2
          acc[t][0] += (float)bf[0] + (float)af[0];
#else
          acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(af, bf, acc[t], 0, 0, 0);
          if (T3) {
            const f16x8 al = *reinterpret_cast<const f16x8*>(cimg + L::kCen + t * 32 * 64);
            accl[T3 ? t : 0] = __builtin_amdgcn_mfma_f32_32x32x16_f16(af, bl, accl[T3 ? t : 0], 0, 0, 0);
            accl[T3 ? t : 0] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, bf, accl[T3 ? t : 0], 0, 0, 0);
          }
#endif
        }
      }
#endif
    };

    // counted waits (ops per wave, in issue order; group 1 issues centres before rows, headers and the
    // epilogue's E stores come last in a phase): see the schedule above
    auto phase_even = [&](int j) __attribute__((always_inline)) {
      // ---- phase 2j: group 0 computes chunk j; group 1 issues centres(j+1), rows(j+2) ------------------
      const bool tail = !more && j >= 12;  // no next-tile traffic: the counted waits below would be too weak
      ST(const uint64_t st_w0 = ST_NOW();)
      if (tail) wait_vm<0>();
      else if (grp == 0) {  // rows(j): phase 2j-5; younger: rows(j+1), rows(j+2) [+ E, header]
        if (!first && j <= 2) wait_vm<2 * kXR + L::E>();
        else if (more && (j == 3 || j == 4)) wait_vm<2 * kXR + L::H1>();
        else if (more && (j == 7 || j == 8)) wait_vm<2 * kXR + L::H2>();
        else wait_vm<2 * kXR>();
      } else {  // centres(j): phase 2j-2; younger: rows(j+1) [+ E, header]
        if (!first && j == 1) wait_vm<kXR + L::E>();
        else if (more && j == 4) wait_vm<kXR + L::H1>();
        else if (more && j == 8) wait_vm<kXR + L::H2>();
        else wait_vm<kXR>();
      }
      lgkm_barrier();
      ST(const uint64_t st_w1 = ST_NOW(); st_wait += st_w1 - st_w0;)
      if (grp == 0) {
        compute(j);
        ST(st_comp += ST_NOW() - st_w1;)
      } else {
        if (j + 1 < kNch) issue_c(cur, j + 1);
        else if (more) issue_c(nxt, j + 1);
        if (j + 2 < kNch) issue_x(cur, j + 2);
        else if (more) issue_x(nxt, j + 2);
        if (j >= 1) header_step(j - 1);
      }
    };
    auto phase_odd = [&](int j) __attribute__((always_inline)) {
      // ---- phase 2j+1: group 1 computes chunk j; group 0 issues rows(j+3) -------------------------------
      const bool tail = !more && j >= 12;
      ST(const uint64_t st_w0 = ST_NOW();)
      if (grp == 1) {  // rows(j): phase 2j-4; younger: phases 2j-2, 2j [+ E, header]
        if (tail) wait_vm<0>();
        else if (!first && j <= 1) wait_vm<2 * (PC + kXR) + L::E>();
        else if (more && (j == 3 || j == 4)) wait_vm<2 * (PC + kXR) + L::H1>();
        else if (more && (j == 7 || j == 8)) wait_vm<2 * (PC + kXR) + L::H2>();
        else wait_vm<2 * (PC + kXR)>();
      }
      lgkm_barrier();
      ST(const uint64_t st_w1 = ST_NOW(); st_wait += st_w1 - st_w0;)
      if (grp == 1) {
        compute(j);
        ST(st_comp += ST_NOW() - st_w1;)
      } else {
        if (j + 3 < kNch) issue_x(cur, j + 3);
        else if (more) issue_x(nxt, j + 3);
        header_step(j);
      }
    };
    // chunk 0 and chunk 15 are peeled: the epilogues run outside the chunk loop (register pressure)
    phase_even(0);
    ST(const uint64_t st_e0 = ST_NOW();)
    if (grp == 1 && !first) epilogue(Hp, row_p, par_p);  // the previous tile's, after this phase's issue
    ST(st_epi += ST_NOW() - st_e0;)
    phase_odd(0);
#pragma unroll 1
    for (int j = 1; j < kNch - 1; ++j) {
      phase_even(j);
      phase_odd(j);
    }
    phase_even(kNch - 1);
    phase_odd(kNch - 1);
    ST(const uint64_t st_e1 = ST_NOW();)
    if (grp == 0) epilogue(Hc, cur.my_row, par);  // after this phase's issue, while group 1 computes
    ST(st_epi += ST_NOW() - st_e1;)
    if (grp == 1) {
      Hp = Hc;
      row_p = cur.my_row;
      par_p = par;
    }
    if (!more) break;
    T = Tn;
    Hc = Hn;
    cur = nxt;
    par ^= 1;
    qb = (qb + kNch) % 3;
    first = false;
  }
  if (grp == 1) epilogue(Hp, row_p, par_p);  // the last tile
#ifdef RQSID_STAMPS
  if (lane == 0 && (wave == 0 || wave == 4)) {
    const int o = wave == 0 ? 0 : 4;
    atomicAdd(&g_stamps[o + 0], (unsigned long long)(ST_NOW() - st_begin));
    atomicAdd(&g_stamps[o + 1], (unsigned long long)st_wait);
    atomicAdd(&g_stamps[o + 2], (unsigned long long)st_comp);
    atomicAdd(&g_stamps[o + 3], (unsigned long long)st_epi);
  }
#endif
}

// R-row tiling of the segments: seg_tile256[s] = sum_{s' < s} ceil(rows(s') / R) (one block).  The total,
// which every tiled screen takes as its tile count, is clamped to the tile maps' capacity max_tiles (the
// segment offsets of one call give at most rows / R + nseg tiles; more means a stale or doubled count): past
// it the error word's kErrTiles bit is raised, so no screen reads a tile map or descriptor past its slot.
__global__ __launch_bounds__(1024) void stream_tiles_kernel(const int32_t* __restrict__ seg_row_off, int nseg, int R,
                                                            int64_t max_tiles, int32_t* __restrict__ err,
                                                            int32_t* __restrict__ seg_tile256) {
  __shared__ int part[1024];
  const int tid = threadIdx.x;
  const int per = (nseg + 1023) / 1024, s0 = min(nseg, tid * per), s1 = min(nseg, s0 + per);
  int sum = 0;
  for (int s = s0; s < s1; ++s) sum += (seg_row_off[s + 1] - seg_row_off[s] + R - 1) / R;
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
    seg_tile256[s] = run;
    run += (seg_row_off[s + 1] - seg_row_off[s] + R - 1) / R;
  }
  if (tid == 1023) {
    int total = part[1023];
    if ((int64_t)total > max_tiles) {
      if (err) atomicOr(err, kErrTiles);
      total = (int)max_tiles;
    }
    seg_tile256[nseg] = total;
  }
}

// tile -> segment map (one thread per tile, binary search over seg_tile256)
__global__ __launch_bounds__(256) void tile_seg_kernel(const int32_t* __restrict__ seg_tile256, int nseg,
                                                       int64_t cap, int32_t* __restrict__ tile_seg) {
  const int ntiles = seg_tile256[nseg];
  for (int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x; t < ntiles && t < cap; t += (int64_t)gridDim.x * 256) {
    int lo = 0, hi = nseg;
    while (hi - lo > 1) {
      const int mid = (lo + hi) >> 1;
      if (seg_tile256[mid] <= t) lo = mid; else hi = mid;
    }
    tile_seg[t] = lo;
  }
}

template <int NT, int RL, bool NORM, bool T3, int W, int S>
bool launch_one(const AssignParams& p, const int32_t* tile_seg, const int32_t* seg_tiles, int64_t max_tiles,
                hipStream_t st) {
  using L = StreamLayout<NT, RL, NORM, T3, W, S>;
  static bool attr[kMaxDevices] = {};
  const int dev = current_device(), ncu = device_cu_count();
  if (dev < 0 || !ncu) return false;
  if (!attr[dev]) {
    if (hipFuncSetAttribute((const void*)assign_stream_kernel<NT, RL, NORM, T3, W, S>,
                            hipFuncAttributeMaxDynamicSharedMemorySize, L::kBytes) != hipSuccess)
      return false;
    attr[dev] = true;
  }
  int64_t g = (int64_t)ncu * L::kBlocks;  // persistent: every block resident at once
  if (g > max_tiles) g = max_tiles;
  g = g / 8 * 8;
  if (g < 8) g = 8;
  hipLaunchKernelGGL((assign_stream_kernel<NT, RL, NORM, T3, W, S>), dim3((unsigned)g), dim3(W * 64), L::kBytes, st,
                     p, tile_seg, seg_tiles);
  return true;
}

// block shape: RQSID_STREAM_SHAPE = 83 (8 waves x 3 stages, the default), 42 (4 waves x 2 stages) or
// 88 (the ping-pong 8-wave form)
int stream_shape() {
  const char* e = getenv("RQSID_STREAM_SHAPE");
  const int v = e ? atoi(e) : 83;
  return v == 42 || v == 88 ? v : 83;
}

template <int NT, int RL, bool NORM, bool T3>
bool launch_pp(const AssignParams& p, const int32_t* tile_seg, const int32_t* seg_tiles, int64_t max_tiles,
               hipStream_t st) {
  using L = PPLayout<NT, RL, NORM, T3>;
  static bool attr[kMaxDevices] = {};
  const int dev = current_device(), ncu = device_cu_count();
  if (dev < 0 || !ncu) return false;
  if (!attr[dev]) {
    if (hipFuncSetAttribute((const void*)assign_pp_kernel<NT, RL, NORM, T3>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            L::kBytes) != hipSuccess)
      return false;
    attr[dev] = true;
  }
  int64_t g = ncu;  // one persistent 8-wave block per CU
  if (g > max_tiles) g = max_tiles;
  g = g / 8 * 8;
  if (g < 8) g = 8;
  hipLaunchKernelGGL((assign_pp_kernel<NT, RL, NORM, T3>), dim3((unsigned)g), dim3(512), L::kBytes, st, p, tile_seg,
                     seg_tiles);
  return true;
}

bool launch_pp_shape(const AssignParams& p, int nt, bool t3, int rl, bool norm, int32_t* tile_seg, int32_t* seg_tiles,
                     int64_t cap, hipStream_t st) {
  constexpr int R = 256;
  hipLaunchKernelGGL(stream_tiles_kernel, dim3(1), dim3(1024), 0, st, p.seg_row_off, p.n_segments, R,
                     (int64_t)(cap / R + p.n_segments), p.work_count ? p.work_count + kErrSlot : (int32_t*)nullptr, seg_tiles);
  const int64_t max_tiles = cap / R + p.n_segments;
  const unsigned tg = (unsigned)(max_tiles / 256 + 1 < 4096 ? max_tiles / 256 + 1 : 4096);
  hipLaunchKernelGGL(tile_seg_kernel, dim3(tg), dim3(256), 0, st, seg_tiles, p.n_segments, cap, tile_seg);
#define RQ_L(NT, RL, NORM, T3) return launch_pp<NT, RL, NORM, T3>(p, tile_seg, seg_tiles, max_tiles, st)
  if (nt == 8) {
    if (rl == 0) RQ_L(8, 0, false, false);
    else if (rl == 1) { if (norm) RQ_L(8, 1, true, false); else RQ_L(8, 1, false, false); }
    else { if (norm) RQ_L(8, 2, true, false); else RQ_L(8, 2, false, false); }
  } else if (t3) {
    if (rl == 0) RQ_L(4, 0, false, true);
    else if (rl == 1) { if (norm) RQ_L(4, 1, true, true); else RQ_L(4, 1, false, true); }
    else { if (norm) RQ_L(4, 2, true, true); else RQ_L(4, 2, false, true); }
  } else {
    if (rl == 0) RQ_L(4, 0, false, false);
    else if (rl == 1) { if (norm) RQ_L(4, 1, true, false); else RQ_L(4, 1, false, false); }
    else { if (norm) RQ_L(4, 2, true, false); else RQ_L(4, 2, false, false); }
  }
#undef RQ_L
  return false;
}

template <int W, int S>
bool launch_shape(const AssignParams& p, int nt, bool t3, int rl, bool norm, int32_t* tile_seg, int32_t* seg_tiles,
                  int64_t cap, hipStream_t st) {
  constexpr int R = W * 32;
  hipLaunchKernelGGL(stream_tiles_kernel, dim3(1), dim3(1024), 0, st, p.seg_row_off, p.n_segments, R,
                     (int64_t)(cap / R + p.n_segments), p.work_count ? p.work_count + kErrSlot : (int32_t*)nullptr, seg_tiles);
  const int64_t max_tiles = cap / R + p.n_segments;  // bound on the R-row tiles
  const unsigned tg = (unsigned)(max_tiles / 256 + 1 < 4096 ? max_tiles / 256 + 1 : 4096);
  hipLaunchKernelGGL(tile_seg_kernel, dim3(tg), dim3(256), 0, st, seg_tiles, p.n_segments, cap, tile_seg);
#define RQ_L(NT, RL, NORM, T3) return launch_one<NT, RL, NORM, T3, W, S>(p, tile_seg, seg_tiles, max_tiles, st)
  if (nt == 8) {
    if (rl == 0) RQ_L(8, 0, false, false);
    else if (rl == 1) { if (norm) RQ_L(8, 1, true, false); else RQ_L(8, 1, false, false); }
    else { if (norm) RQ_L(8, 2, true, false); else RQ_L(8, 2, false, false); }
  } else if (t3) {
    if (rl == 0) RQ_L(4, 0, false, true);
    else if (rl == 1) { if (norm) RQ_L(4, 1, true, true); else RQ_L(4, 1, false, true); }
    else { if (norm) RQ_L(4, 2, true, true); else RQ_L(4, 2, false, true); }
  } else {
    if (rl == 0) RQ_L(4, 0, false, false);
    else if (rl == 1) { if (norm) RQ_L(4, 1, true, false); else RQ_L(4, 1, false, false); }
    else { if (norm) RQ_L(4, 2, true, false); else RQ_L(4, 2, false, false); }
  }
#undef RQ_L
  return false;
}

}  // namespace

bool stream_supported(int nt, bool t3, int rl, bool norm) {
  (void)norm;
  if (nt == 8) return !t3 && rl >= 0 && rl <= 2;
  if (nt == 4) return rl >= 0 && rl <= 2;
  return false;
}

void launch_tiling(const AssignParams& p, int R, int32_t* tile_seg, int32_t* seg_tiles, int64_t cap, hipStream_t st) {
  hipLaunchKernelGGL(stream_tiles_kernel, dim3(1), dim3(1024), 0, st, p.seg_row_off, p.n_segments, R,
                     (int64_t)(cap / R + p.n_segments), p.work_count ? p.work_count + kErrSlot : (int32_t*)nullptr, seg_tiles);
  const int64_t max_tiles = cap / R + p.n_segments;
  const unsigned tg = (unsigned)(max_tiles / 256 + 1 < 4096 ? max_tiles / 256 + 1 : 4096);
  hipLaunchKernelGGL(tile_seg_kernel, dim3(tg), dim3(256), 0, st, seg_tiles, p.n_segments, cap, tile_seg);
}

int launch_stream_screen(const AssignParams& p, int nt, bool t3, int rl, bool norm, int32_t* tile_seg,
                         int32_t* seg_tiles, int64_t cap, int shape, hipStream_t st) {
  if (shape == 0) shape = stream_shape();
  bool ok;
  if (shape == 88) ok = launch_pp_shape(p, nt, t3, rl, norm, tile_seg, seg_tiles, cap, st);
  else if (shape == 42) ok = launch_shape<4, 2>(p, nt, t3, rl, norm, tile_seg, seg_tiles, cap, st);
  else ok = launch_shape<8, 3>(p, nt, t3, rl, norm, tile_seg, seg_tiles, cap, st);
  return ok ? RQSID_OK : fail(RQSID_E_LAUNCH, "assign: stream screen launch failed (device query / LDS attribute)");
}

}  // namespace rqsid

#ifdef RQSID_STAMPS
extern "C" int rqsid_debug_stamps(unsigned long long* out8) {
  if (hipMemcpyFromSymbol(out8, HIP_SYMBOL(g_stamps), 8 * sizeof(unsigned long long)) != hipSuccess) return -1;
  const unsigned long long z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  return hipMemcpyToSymbol(HIP_SYMBOL(g_stamps), z, sizeof(z)) == hipSuccess ? 0 : -1;
}
#endif
