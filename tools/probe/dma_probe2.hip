// HBM + centre-stream probe (tools only): persistent blocks of W waves over (32W)-row tiles of 10M x
// 2 KiB rows (gathered by a permutation), ring of S stages of 32 dims: x (32W rows x 128 B) + a
// centre image of NC candidates x 64 B gathered from a 2560 x 1 KiB L2-resident fp16 table, with
// the tile-to-tile prefetch kept running (no drain at tile boundaries).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <algorithm>
#include <random>

__device__ __forceinline__ uint32_t lds_addr(const void* ptr) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)ptr;
}
template <bool NTL = false>
__device__ __forceinline__ void dma16(const void* gsrc, uint32_t lds_base) {
  uint32_t keep;
  if (NTL)
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off nt\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(gsrc), "s"(lds_base) : "memory");
  else
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(gsrc), "s"(lds_base) : "memory");
}
template <int N> __device__ __forceinline__ void waitb() {
  asm volatile("s_waitcnt vmcnt(%0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::"i"(N) : "memory");
}

template <int W, int S, int NC, bool NTX, int CP>
__global__ __launch_bounds__(W * 64) void probe(const char* __restrict__ x, const int* __restrict__ perm,
                                                const char* __restrict__ ctab, int ntiles) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  constexpr int R = 32 * W;               // rows per tile
  constexpr int XS = R * 128;             // x bytes per stage
  constexpr int CS = NC * 64;             // centre bytes per stage
  constexpr int PX = 4;                   // x DMAs per wave per stage (32 rows x 128 B)
  constexpr int PC = CS / 1024 / W;       // centre DMAs per wave per stage
  constexpr int P = PX + PC;
  constexpr int NCH = 16;
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t l0 = lds_addr(smem);
  int tile = blockIdx.x;
  if (tile >= ntiles) return;
  const char* xs[PX];
  const char* cs[PC > 0 ? PC : 1];
  auto setup = [&](int t, const char** xo, const char** co) {
#pragma unroll
    for (int i = 0; i < PX; ++i) {
      const int row = perm[t * R + wave * 32 + i * 8 + lane / 8];
      xo[i] = x + (size_t)row * 2048 + (lane % 8) * 16;
    }
#pragma unroll
    for (int j = 0; j < PC; ++j) {
      if (CP == 64) {  // 16 candidates x 64 B (32 fp16 dims) per op
        const int cand = ((t * 977) + (wave * PC + j) * 16 + lane / 4) % 2560;
        co[j] = ctab + (size_t)cand * 1024 + (lane % 4) * 16;
      } else {  // 8 candidates x 128 B (64 dims) per op; a chunk pair covers every candidate
        const int cand = ((t * 977) + (wave * PC + j) * 8 + lane / 8) % 2560;
        co[j] = ctab + (size_t)cand * 1024 + (lane % 8) * 16;
      }
    }
  };
  auto issue = [&](const char** xo, const char** co, int c, int st) {
    const uint32_t sb = l0 + st * (XS + CS);
#pragma unroll
    for (int i = 0; i < PX; ++i) dma16<NTX>(xo[i] + c * 128, __builtin_amdgcn_readfirstlane(sb + (wave * PX + i) * 1024));
#pragma unroll
    for (int j = 0; j < PC; ++j) {
      const size_t off = CP == 64 ? (size_t)c * 64 : (size_t)(c >> 1) * 128 + (size_t)(c & 1) * (NC / 2) * 1024;
      dma16(co[j] + off, __builtin_amdgcn_readfirstlane(sb + XS + (wave * PC + j) * 1024));
    }
  };
  const char* xc[PX]; const char* cc[PC > 0 ? PC : 1];
  const char* xn[PX]; const char* cn[PC > 0 ? PC : 1];
  setup(tile, xc, cc);
  for (int c = 0; c < S - 1; ++c) issue(xc, cc, c, c);
  int q = 0;
  for (;;) {
    const int next = tile + gridDim.x;
    const bool more = next < ntiles;
    if (more) setup(next, xn, cn);  // (plain loads: drained at the first wait, fine for a probe)
    for (int c = 0; c < NCH; ++c, ++q) {
      const int ahead = more ? S - 2 : min(S - 2, NCH - 1 - c);
      if (ahead >= 2) waitb<2 * P>(); else if (ahead == 1) waitb<P>(); else waitb<0>();
      const int st = (q + S - 1) % S;
      if (c + S - 1 < NCH) issue(xc, cc, c + S - 1, st);
      else if (more) issue(xn, cn, c + S - 1 - NCH, st);
    }
    if (!more) break;
    tile = next;
#pragma unroll
    for (int i = 0; i < PX; ++i) xc[i] = xn[i];
#pragma unroll
    for (int j = 0; j < PC; ++j) cc[j] = cn[j];
  }
}

template <int W, int S, int NC, bool NTX, int CP>
void run(const char* x, const int* perm, const char* ctab, int n, int ncu, int bpc) {
  const int R = 32 * W, ntiles = n / R;
  const int lds = S * (R * 128 + NC * 64);
  if (lds * bpc > 160 * 1024) { printf("W=%d S=%d NC=%d bpc=%d: LDS %d too big\n", (int)NTX, W, S, NC, bpc, lds); return; }
  const int alloc = std::max(lds, 160 * 1024 / bpc - 1024);
  hipFuncSetAttribute((const void*)probe<W, S, NC, NTX, CP>, hipFuncAttributeMaxDynamicSharedMemorySize, alloc);
  const int grid = std::min(ntiles, ncu * bpc);
  hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
  hipLaunchKernelGGL((probe<W, S, NC, NTX, CP>), dim3(grid), dim3(W * 64), alloc, 0, x, perm, ctab, ntiles);
  hipEventRecord(a);
  for (int i = 0; i < 3; ++i) hipLaunchKernelGGL((probe<W, S, NC, NTX, CP>), dim3(grid), dim3(W * 64), alloc, 0, x, perm, ctab, ntiles);
  hipEventRecord(b); hipEventSynchronize(b);
  float ms; hipEventElapsedTime(&ms, a, b); ms /= 3;
  if (hipGetLastError() != hipSuccess) { printf("error\n"); return; }
  const double bytes = (double)ntiles * R * 2048;
  printf("cp=%d nt=%d waves=%d S=%d cands=%d blocks/CU=%d x-inflight/CU=%3d KB lds=%3d KB  %.3f ms  %.0f GB/s (x)\n", CP, (int)NTX, W, S, NC, bpc,
         (S - 1) * R * 128 * bpc / 1024, lds / 1024, ms, bytes / ms / 1e6);
  fflush(stdout);
}

int main() {
  const int n = 10000000 / 256 * 256;
  char *x, *ctab; int* perm;
  hipMalloc(&x, (size_t)n * 2048); hipMalloc(&perm, (size_t)n * 4); hipMalloc(&ctab, 2560 * 1024);
  hipMemset(x, 0, (size_t)n * 2048); hipMemset(ctab, 0, 2560 * 1024);
  std::vector<int> p(n); for (int i = 0; i < n; ++i) p[i] = i;
  std::mt19937 g(1); std::shuffle(p.begin(), p.end(), g);
  hipMemcpy(perm, p.data(), (size_t)n * 4, hipMemcpyHostToDevice);
  hipDeviceProp_t prop; hipGetDeviceProperties(&prop, 0);
  const int ncu = prop.multiProcessorCount;
#define R(W, S, NC, B, T, CP) run<W, S, NC, T, CP>(x, perm, ctab, n, ncu, B);
  R(4, 2, 256, 2, true, 64) R(4, 2, 256, 2, true, 128) R(8, 3, 256, 1, true, 64) R(8, 3, 256, 1, true, 128)
  R(4, 2, 128, 3, true, 64) R(4, 2, 128, 3, true, 128) R(8, 3, 0, 1, true, 64) R(4, 2, 0, 3, true, 64)
  return 0;
}
