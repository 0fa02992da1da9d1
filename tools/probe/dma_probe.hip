// HBM read-pattern probe for the screen's x staging (tools only): LDS-DMA (global_load_lds_dwordx4)
// of 10M x 2 KiB rows, persistent 4-wave blocks over 128-row tiles, ring of S stages of `PIECE`
// bytes per row (a row is visited 2048/PIECE times), rows in order or gathered by a permutation.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>
#include <random>

__device__ __forceinline__ uint32_t lds_addr(const void* ptr) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)ptr;
}
__device__ __forceinline__ void dma16(const void* gsrc, uint32_t lds_base) {
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(gsrc), "s"(lds_base) : "memory");
}
template <int N> __device__ __forceinline__ void waitb() {
  asm volatile("s_waitcnt vmcnt(%0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::"i"(N) : "memory");
}

constexpr int ROWB = 2048;

// PIECE bytes per row per stage; stage = 128 rows x PIECE; each wave moves its 32 rows: 32*PIECE/1024 DMAs
template <int PIECE, int S, bool PERM>
__global__ __launch_bounds__(256) void probe(const char* __restrict__ x, const int* __restrict__ perm, int ntiles) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  constexpr int NI = 32 * PIECE / 1024;       // DMAs per wave per stage
  constexpr int LPR = PIECE / 16;             // lanes per row in one DMA
  constexpr int RPI = 64 / LPR;               // rows per DMA instruction
  constexpr int NCH = ROWB / PIECE;           // stages per tile
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t l0 = lds_addr(smem);
  const char* src[NI];
  int tile = blockIdx.x;
  auto setup = [&](int t) {
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      int row = t * 128 + wave * 32 + i * RPI + lane / LPR;
      if (PERM) row = perm[row];
      src[i] = x + (size_t)row * ROWB + (lane % LPR) * 16;
    }
  };
  setup(tile);
  int q = 0;  // global stage counter
  auto issue = [&](int c) {
    const uint32_t sb = l0 + ((q + S - 1) % S) * (128 * PIECE);
#pragma unroll
    for (int i = 0; i < NI; ++i) dma16(src[i] + c * PIECE, __builtin_amdgcn_readfirstlane(sb + (wave * NI + i) * 1024));
  };
  // simple per-tile ring (no cross-tile prefetch): S-1 stages ahead
  for (; tile < ntiles; tile += gridDim.x) {
    setup(tile);
    for (int c = 0; c < S - 1 && c < NCH; ++c) {
      const uint32_t sb = l0 + (c % S) * (128 * PIECE);
#pragma unroll
      for (int i = 0; i < NI; ++i) dma16(src[i] + c * PIECE, __builtin_amdgcn_readfirstlane(sb + (wave * NI + i) * 1024));
    }
    for (int c = 0; c < NCH; ++c) {
      const int younger = min(S - 2, NCH - 1 - c);
      if (younger >= 3) waitb<3 * NI>(); else if (younger == 2) waitb<2 * NI>(); else if (younger == 1) waitb<NI>(); else waitb<0>();
      if (c + S - 1 < NCH) {
        const uint32_t sb = l0 + ((c + S - 1) % S) * (128 * PIECE);
#pragma unroll
        for (int i = 0; i < NI; ++i) dma16(src[i] + (c + S - 1) * PIECE, __builtin_amdgcn_readfirstlane(sb + (wave * NI + i) * 1024));
      }
    }
  }
  (void)q; (void)issue;
}

template <int PIECE, int S, bool PERM>
void run(const char* x, const int* perm, int ntiles, int bpc, int ncu, double bytes) {
  const int lds = S * 128 * PIECE;
  if (lds > 160 * 1024 / bpc) { printf("PIECE=%d S=%d bpc=%d: LDS %d too big\n", PIECE, S, bpc, lds); return; }
  const int ldsalloc = std::max(lds, 160 * 1024 / bpc - 2048);
  hipFuncSetAttribute((const void*)probe<PIECE, S, PERM>, hipFuncAttributeMaxDynamicSharedMemorySize, ldsalloc);
  const int grid = std::min(ntiles, ncu * bpc);
  hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
  hipLaunchKernelGGL((probe<PIECE, S, PERM>), dim3(grid), dim3(256), ldsalloc, 0, x, perm, ntiles);
  hipEventRecord(a);
  for (int i = 0; i < 3; ++i) hipLaunchKernelGGL((probe<PIECE, S, PERM>), dim3(grid), dim3(256), ldsalloc, 0, x, perm, ntiles);
  hipEventRecord(b); hipEventSynchronize(b);
  float ms; hipEventElapsedTime(&ms, a, b); ms /= 3;
  printf("piece=%4d S=%d perm=%d blocks/CU=%d inflight/CU=%3d KB  %.3f ms  %.0f GB/s\n", PIECE, S, (int)PERM, bpc,
         (S - 1) * 128 * PIECE * bpc / 1024, ms, bytes / ms / 1e6);
  fflush(stdout);
}

int main() {
  const int n = 10000000 / 128 * 128, ntiles = n / 128;
  char* x; int* perm;
  hipMalloc(&x, (size_t)n * ROWB); hipMalloc(&perm, (size_t)n * 4);
  hipMemset(x, 0, (size_t)n * ROWB);
  std::vector<int> p(n); for (int i = 0; i < n; ++i) p[i] = i;
  std::mt19937 g(1); std::shuffle(p.begin(), p.end(), g);
  hipMemcpy(perm, p.data(), (size_t)n * 4, hipMemcpyHostToDevice);
  hipDeviceProp_t prop; hipGetDeviceProperties(&prop, 0);
  const int ncu = prop.multiProcessorCount;
  const double bytes = (double)n * ROWB;
#define R(PC, S, PM, B) run<PC, S, PM>(x, perm, ntiles, B, ncu, bytes);
  R(64, 4, false, 2) R(128, 2, false, 3) R(128, 3, false, 2) R(256, 2, false, 2)
  R(64, 4, true, 2) R(64, 4, true, 3) R(128, 2, true, 3) R(128, 3, true, 2) R(128, 4, true, 2) R(256, 2, true, 2)
  R(256, 3, true, 1) R(512, 2, true, 1) R(128, 2, true, 4) R(64, 4, true, 4)
  return 0;
}
