// Row-staging probe (tools only): how fast can gathered 2-KiB fp32 rows (10M rows in a
// random permutation, the level-2 access pattern) be brought into LDS, chunk by chunk, beside the
// L2-resident centre stream of the screen (256 candidates x 64 B per 32-dim chunk)?
//   mode 0: rows by LDS-DMA (global_load_lds_dwordx4, 4 ops per wave per chunk), as the screens do
//   mode 1: rows by global_load_dwordx4 into VGPRs, then ds_write_b128 of the fp32 image
//   mode 2: as 1, converted to fp16 before ds_write_b64 (half the LDS bytes)
//   mode 3: rows by global_load_dwordx4 into VGPRs, converted to fp16 and kept there (a row-resident
//           screen: rows never touch LDS, only the centres are staged)
// Centres by LDS-DMA in every mode.  Each wave then reads its rows' fragments and one centre
// fragment per chunk from LDS (the consumer's LDS traffic) and folds them into a sink.
// Persistent blocks, one 32-row slice per wave, S ring stages, prefetch distance S-1 (mode 0) or
// one chunk in VGPRs + S-1 LDS stages (modes 1, 2).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <random>
#include <vector>

__device__ __forceinline__ uint32_t lds_addr(const void* ptr) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)ptr;
}
__device__ __forceinline__ void dma16(const void* gsrc, uint32_t lds_base, bool nt) {
  uint32_t keep;
  if (nt)
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off nt\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(gsrc), "s"(lds_base) : "memory");
  else
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(gsrc), "s"(lds_base) : "memory");
}
__device__ __forceinline__ float4 gload_nt(const float4* p) {
  typedef __attribute__((ext_vector_type(4))) float v4;
  const v4 v = __builtin_nontemporal_load(reinterpret_cast<const v4*>(p));
  return make_float4(v.x, v.y, v.z, v.w);
}

template <int W, int S, int MODE>
__global__ __launch_bounds__(W * 64) void probe(const float* __restrict__ x, const int* __restrict__ perm,
                                                const char* __restrict__ ctab, int ntiles, float* sink) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  constexpr int R = 32 * W;                      // rows per tile
  constexpr int XB = MODE == 3 ? 0 : MODE == 2 ? 64 : 128;  // LDS bytes per row per chunk
  constexpr int XS = R * XB;
  constexpr int CS = 256 * 64;                   // centre image per chunk
  constexpr int PC = CS / 1024 / W;              // centre DMAs per wave per chunk
  constexpr int NCH = 16;
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t l0 = lds_addr(smem);
  int tile = blockIdx.x;
  if (tile >= ntiles) return;
  // row sources of this wave: instruction i moves rows 8i + lane/8, 16-B slot lane%8 of the chunk
  int rc[4], rn[4], cc[PC], cn[PC];
  auto setup = [&](int t, int* r, int* cd) {
#pragma unroll
    for (int i = 0; i < 4; ++i) r[i] = perm[(size_t)t * R + wave * 32 + i * 8 + lane / 8];
#pragma unroll
    for (int j = 0; j < PC; ++j) cd[j] = ((t * 977) + (wave * PC + j) * 16 + lane / 4) % 2560;
  };
  auto stage_base = [&](int st) { return l0 + st * (XS + CS); };
  auto issue_c = [&](const int* cd, int c, int st) {
#pragma unroll
    for (int j = 0; j < PC; ++j)
      dma16(ctab + (size_t)cd[j] * 1024 + c * 64 + (lane % 4) * 16,
            __builtin_amdgcn_readfirstlane(stage_base(st) + XS + (wave * PC + j) * 1024), false);
  };
  auto issue_x_dma = [&](const int* r, int c, int st) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
      dma16(reinterpret_cast<const char*>(x) + (size_t)r[i] * 2048 + c * 128 + (lane % 8) * 16,
            __builtin_amdgcn_readfirstlane(stage_base(st) + (wave * 32 + i * 8) * XB), true);
  };
  float4 reg[4];
  auto load_x = [&](const int* r, int c) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
      reg[i] = gload_nt(reinterpret_cast<const float4*>(x + (size_t)r[i] * 512 + c * 32) + (lane % 8));
  };
  auto write_x = [&](int st) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int rr = wave * 32 + i * 8 + lane / 8;
      unsigned char* dst = smem + st * (XS + CS) + rr * XB;
      if (MODE == 1) {
        *reinterpret_cast<float4*>(dst + (lane % 8) * 16) = reg[i];
      } else {
        typedef __attribute__((ext_vector_type(4))) _Float16 h4;
        h4 v = {(_Float16)reg[i].x, (_Float16)reg[i].y, (_Float16)reg[i].z, (_Float16)reg[i].w};
        *reinterpret_cast<h4*>(dst + (lane % 8) * 8) = v;
      }
    }
  };
  float acc = 0.f, keep = 0.f;
  auto consume = [&](int st) {
    const unsigned char* b = smem + st * (XS + CS);
    const unsigned char* xr = b + (wave * 32 + (lane & 31)) * XB;
    if (MODE == 3) {
    } else if (MODE == 2) {
      const float2 a = *reinterpret_cast<const float2*>(xr + (lane >> 5) * 8);
      const float2 c = *reinterpret_cast<const float2*>(xr + 16 + (lane >> 5) * 8);
      acc += a.x + c.y;
    } else {
      const float4 a = *reinterpret_cast<const float4*>(xr + (lane >> 5) * 16);
      const float4 c = *reinterpret_cast<const float4*>(xr + 32 + (lane >> 5) * 16);
      acc += a.x + c.w;
    }
    const float4 cf = *reinterpret_cast<const float4*>(b + XS + ((lane & 31) + 32 * (wave & 7)) * 64 + (lane >> 5) * 16);
    acc += cf.y;
  };
  setup(tile, rc, cc);
  // prologue: chunks 0 .. S-2 in flight (mode 0: rows and centres by DMA; else centres by DMA and
  // chunk 0's rows in VGPRs)
  for (int c = 0; c < S - 1; ++c) {
    issue_c(cc, c, c);
    if (MODE == 0) issue_x_dma(rc, c, c);
  }
  if (MODE != 0) load_x(rc, 0);
  int q = 0;
  for (;;) {
    const int next = tile + gridDim.x;
    const bool more = next < ntiles;
    if (more) setup(next, rn, cn);
    for (int c = 0; c < NCH; ++c, ++q) {
      const int st = q % S;
      if (MODE == 0) {
        asm volatile("s_waitcnt vmcnt(%0)" ::"i"((S - 2) * (PC + 4)) : "memory");
      } else if (MODE == 3) {
        asm volatile("s_waitcnt vmcnt(%0)" ::"i"(S >= 3 ? PC : 0) : "memory");
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          typedef __attribute__((ext_vector_type(2))) _Float16 h2;
          const h2 v = {(_Float16)reg[i].x, (_Float16)reg[i].w};
          keep += (float)(v.x * v.y);
        }
      } else {
        // chunk c's rows (issued last iteration before its centre ops) and, older, chunk c's centres
        asm volatile("s_waitcnt vmcnt(%0)" ::"i"(S >= 3 ? PC : 0) : "memory");
        write_x(st);
      }
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
      const int ca = c + S - 1, sa = (q + S - 1) % S;
      if (MODE != 0) {
        if (c + 1 < NCH) load_x(rc, c + 1);
        else if (more) load_x(rn, 0);
      }
      if (ca < NCH) {
        issue_c(cc, ca, sa);
        if (MODE == 0) issue_x_dma(rc, ca, sa);
      } else if (more) {
        issue_c(cn, ca - NCH, sa);
        if (MODE == 0) issue_x_dma(rn, ca - NCH, sa);
      }
      consume(st);
    }
    if (!more) break;
    tile = next;
#pragma unroll
    for (int i = 0; i < 4; ++i) rc[i] = rn[i];
#pragma unroll
    for (int j = 0; j < PC; ++j) cc[j] = cn[j];
  }
  if (acc + keep == 1.2345f) sink[blockIdx.x] = acc;
}

template <int W, int S, int MODE>
void run(const float* x, const int* perm, const char* ctab, float* sink, int n, int ncu, int bpc) {
  const int R = 32 * W, ntiles = n / R;
  const int XB = MODE == 3 ? 0 : MODE == 2 ? 64 : 128;
  const int lds = S * (R * XB + 256 * 64);
  if (lds * bpc > 160 * 1024) {
    printf("mode=%d W=%d S=%d bpc=%d: LDS %d KB too big\n", MODE, W, S, bpc, lds / 1024);
    return;
  }
  hipFuncSetAttribute((const void*)probe<W, S, MODE>, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
  const int grid = std::min(ntiles, ncu * bpc);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  hipLaunchKernelGGL((probe<W, S, MODE>), dim3(grid), dim3(W * 64), lds, 0, x, perm, ctab, ntiles, sink);
  hipEventRecord(a);
  for (int i = 0; i < 3; ++i)
    hipLaunchKernelGGL((probe<W, S, MODE>), dim3(grid), dim3(W * 64), lds, 0, x, perm, ctab, ntiles, sink);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  ms /= 3;
  if (hipGetLastError() != hipSuccess) {
    printf("error\n");
    return;
  }
  const double bytes = (double)ntiles * R * 2048;
  printf("mode=%d (%s) waves=%2d S=%d blocks/CU=%d lds=%3d KB  %.3f ms  %.0f GB/s of rows\n", MODE,
         MODE == 0 ? "lds-dma   " : MODE == 1 ? "reg fp32  " : MODE == 2 ? "reg->fp16 " : "reg only  ", W, S, bpc, lds / 1024, ms, bytes / ms / 1e6);
  fflush(stdout);
}

int main() {
  const int n = 10000000 / 512 * 512;
  float* x;
  char* ctab;
  int* perm;
  float* sink;
  hipMalloc(&x, (size_t)n * 2048);
  hipMalloc(&perm, (size_t)n * 4);
  hipMalloc(&ctab, 2560 * 1024);
  hipMalloc(&sink, 1 << 20);
  hipMemset(x, 0, (size_t)n * 2048);
  hipMemset(ctab, 0, 2560 * 1024);
  std::vector<int> p(n);
  for (int i = 0; i < n; ++i) p[i] = i;
  std::mt19937 g(1);
  std::shuffle(p.begin(), p.end(), g);
  hipMemcpy(perm, p.data(), (size_t)n * 4, hipMemcpyHostToDevice);
  hipDeviceProp_t prop;
  hipGetDeviceProperties(&prop, 0);
  const int ncu = prop.multiProcessorCount;
#define RUN(W, S, M, B) run<W, S, M>(x, perm, ctab, sink, n, ncu, B);
  RUN(8, 3, 0, 1) RUN(8, 3, 1, 1) RUN(8, 3, 2, 1)
  RUN(4, 2, 0, 2) RUN(4, 2, 1, 2) RUN(4, 2, 2, 2)
  RUN(4, 3, 0, 2) RUN(4, 3, 1, 2) RUN(4, 3, 2, 2)
  RUN(8, 2, 0, 2) RUN(8, 2, 1, 2) RUN(8, 2, 2, 2)
  RUN(16, 2, 0, 1) RUN(16, 2, 1, 1) RUN(16, 2, 2, 1)
  RUN(4, 4, 2, 2) RUN(8, 4, 2, 1)
  RUN(4, 2, 3, 2) RUN(8, 2, 3, 1) RUN(8, 2, 3, 2) RUN(8, 3, 3, 1) RUN(16, 2, 3, 1)
  return 0;
}
