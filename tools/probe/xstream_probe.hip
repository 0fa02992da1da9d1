// Memory-pipeline probe for the register-streamed screen design (tools only, not the product):
// 10M x 512 fp32 rows, each lane streams ONE row (lane = row r, half h) into VGPRs with asm
// global_load_dwordx4 in 16-dim sub-chunks (32 B per lane), D sub-chunks ahead, persistent blocks
// over 128-row tiles; optional row gather (permutation) and an LDS-DMA centre stream (8 KB per
// sub-chunk per block from an L2-resident table) counted on the same vmcnt.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>
#include <random>
#include <utility>
#include <type_traits>

typedef float f4 __attribute__((ext_vector_type(4)));

template <int OFF> __device__ __forceinline__ void ld16(f4& d, const void* p) {
  asm volatile("global_load_dwordx4 %0, %1, off offset:%2" : "=v"(d) : "v"(p), "i"(OFF) : "memory");
}
__device__ __forceinline__ void ld4(int& d, const void* p) {
  asm volatile("global_load_dword %0, %1, off" : "=v"(d) : "v"(p) : "memory");
}
__device__ __forceinline__ uint32_t lds_addr(const void* ptr) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)ptr;
}
__device__ __forceinline__ void dma16(const void* gsrc, uint32_t lds_base) {
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(gsrc), "s"(lds_base) : "memory");
}
template <int N> __device__ __forceinline__ void waitv(f4& a, f4& b) {
  asm volatile("s_waitcnt vmcnt(%2)" : "+v"(a), "+v"(b) : "i"(N) : "memory");
}

constexpr int DIM = 512, SUB = 32;  // 16-dim sub-chunks per row

template <int D, bool PERM, int CEN>
__global__ __launch_bounds__(256) void probe(const float* __restrict__ x, const int* __restrict__ perm,
                                             const _Float16* __restrict__ ctab, int ntiles, float* out) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int r = lane & 31, h = lane >> 5;
  constexpr int P = 2 + CEN;  // VMEM ops per sub-chunk per wave
  f4 xr[D + 1][2];
  float acc = 0.f;
  int tile = blockIdx.x;
  if (tile >= ntiles) return;
  int row = tile * 128 + wave * 32 + r;
  if (PERM) row = perm[row];
  int nrow_next = 0;
  const float* src = x + (size_t)row * DIM + 8 * h;
  const float* src_next = src;
  const uint32_t cl = lds_addr(smem);
  auto issue = [&](auto slot_c, const float* s, auto k_c) {
    constexpr int slot = decltype(slot_c)::value, k = decltype(k_c)::value;
    ld16<64 * k>(xr[slot][0], s);
    ld16<64 * k + 16>(xr[slot][1], s);
    if (CEN) {
      const _Float16* c = ctab + (size_t)(((tile * 131) & 2047) + wave * 16 + (lane >> 2)) * DIM + 16 * k + (lane & 3) * 4;
#pragma unroll
      for (int j = 0; j < CEN; ++j)
        dma16(c + j * 64 * DIM, __builtin_amdgcn_readfirstlane(cl + ((slot * CEN + j) * 4 + wave) * 1024));
    }
  };
  // prologue: sub-chunks 0..D-1 of the first tile
  [&]<int... K>(std::integer_sequence<int, K...>) { (issue(std::integral_constant<int, K>{}, src, std::integral_constant<int, K>{}), ...); }(std::make_integer_sequence<int, D>{});
  for (;;) {
    const int next = tile + gridDim.x;
    const bool more = next < ntiles;
    auto body = [&](auto k_c) {
      constexpr int k = decltype(k_c)::value;
      constexpr int ka = k + D;  // sub-chunk to issue (this tile or the next)
      if constexpr (ka < SUB) issue(std::integral_constant<int, ka % (D + 1)>{}, src, std::integral_constant<int, ka>{});
      else if (more) issue(std::integral_constant<int, ka % (D + 1)>{}, src_next, std::integral_constant<int, ka - SUB>{});
      if (k == 0) {
        int rn = next * 128 + wave * 32 + r;
        if (PERM) { if (more) ld4(nrow_next, perm + rn); } else nrow_next = rn;
      }
      if (k == D + 1 || (D + 1 >= SUB && k == 0)) {
        asm volatile("" : "+v"(nrow_next));
        src_next = x + (size_t)(more ? nrow_next : 0) * DIM + 8 * h;
        asm volatile("" : "+v"(src_next));
      }
      // wait for sub-chunk k: younger = sub-chunks k+1..k+D (+1 perm op, over-waited by one op)
      if (ka < SUB || more) waitv<D * P>(xr[k % (D + 1)][0], xr[k % (D + 1)][1]);
      else waitv<0>(xr[k % (D + 1)][0], xr[k % (D + 1)][1]);
      if (CEN) __builtin_amdgcn_s_barrier();
      const f4 a = xr[k % (D + 1)][0], b = xr[k % (D + 1)][1];
      acc += a.x + a.y + a.z + a.w + b.x + b.y + b.z + b.w;
      __builtin_amdgcn_sched_barrier(0);
    };
    [&]<int... K>(std::integer_sequence<int, K...>) { (body(std::integral_constant<int, K>{}), ...); }(std::make_integer_sequence<int, SUB>{});
    if (!more) break;
    tile = next;
    src = src_next;
  }
  if (acc == 1.2345e-30f) out[threadIdx.x] = acc;
}

template <int D, bool PERM, int CEN>
float run(const float* x, const int* perm, const _Float16* ctab, int ntiles, float* out, int blocks_per_cu, int ncu) {
  int grid = std::min(ntiles, ncu * blocks_per_cu);
  size_t lds = CEN ? (size_t)(D + 1) * CEN * 4 * 1024 : 0;
  lds = std::max(lds, (size_t)(160 * 1024 / blocks_per_cu - 1024));  // occupancy by LDS
  hipFuncSetAttribute((const void*)probe<D, PERM, CEN>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  hipEvent_t a, b;
  hipEventCreate(&a); hipEventCreate(&b);
  for (int i = 0; i < 2; ++i) hipLaunchKernelGGL((probe<D, PERM, CEN>), dim3(grid), dim3(256), lds, 0, x, perm, ctab, ntiles, out);
  hipEventRecord(a);
  const int reps = 5;
  for (int i = 0; i < reps; ++i) hipLaunchKernelGGL((probe<D, PERM, CEN>), dim3(grid), dim3(256), lds, 0, x, perm, ctab, ntiles, out);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms; hipEventElapsedTime(&ms, a, b);
  if (hipGetLastError() != hipSuccess) { printf("launch error\n"); exit(1); }
  return ms / reps;
}

int main() {
  const int n = 10000000 / 128 * 128, ntiles = n / 128;
  float* x; int* perm; _Float16* ctab; float* out;
  hipMalloc(&x, (size_t)n * DIM * 4);
  hipMalloc(&perm, (size_t)n * 4);
  hipMalloc(&ctab, (size_t)4096 * DIM * 2);
  hipMalloc(&out, 4096);
  hipMemset(x, 0, (size_t)n * DIM * 4);
  hipMemset(ctab, 0, (size_t)4096 * DIM * 2);
  std::vector<int> p(n);
  for (int i = 0; i < n; ++i) p[i] = i;
  std::mt19937 g(1);
  std::shuffle(p.begin(), p.end(), g);
  hipMemcpy(perm, p.data(), (size_t)n * 4, hipMemcpyHostToDevice);
  hipDeviceProp_t prop; hipGetDeviceProperties(&prop, 0);
  const int ncu = prop.multiProcessorCount;
  const double bytes = (double)n * DIM * 4;
#define R(D, PM, C, B) { float ms = run<D, PM, C>(x, perm, ctab, ntiles, out, B, ncu); \
    printf("D=%d perm=%d cen=%d blocks/CU=%d  %.3f ms  %.0f GB/s\n", D, PM, C, B, ms, bytes / ms / 1e6); fflush(stdout); }
  R(1, false, 0, 2) R(3, false, 0, 2) R(7, false, 0, 2) R(3, false, 0, 3) R(7, false, 0, 3)
  R(1, true, 0, 2) R(3, true, 0, 2) R(7, true, 0, 2) R(3, true, 0, 3) R(7, true, 0, 3) R(15, true, 0, 2)
  R(3, true, 2, 2) R(7, true, 2, 2) R(3, true, 2, 3) R(3, true, 4, 2) R(7, true, 4, 2)
  return 0;
}
