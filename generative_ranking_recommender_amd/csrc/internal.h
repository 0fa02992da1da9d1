// internal.h — shared helpers of the rqsid HIP translation units (not part of the C ABI).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "../../include/rqsid.h"

namespace rqsid {

// error text of the calling thread (rqsid_last_error) + status helpers
int fail(int code, const char* fmt, ...);
int check_launch(const char* what);
// hipMemsetAsync's job done by a kernel (the default): inside a captured HIP graph a kernel node is ordered
// like every other kernel of the stream.  RQSID_MEMSET_API=1 uses hipMemsetAsync (A/B, graph diagnosis).
hipError_t fill_async(void* p, int value, size_t bytes, hipStream_t st);

inline int64_t cdiv(int64_t a, int64_t b) { return (a + b - 1) / b; }

// Per-device one-time state (dynamic-LDS attributes, CU counts) is kept per HIP device: a kernel
// attribute set on one device says nothing about another.  current_device() is -1 on error or
// beyond kMaxDevices; device_cu_count() is cached per device (0 on error).
constexpr int kMaxDevices = 64;
int current_device();
int device_cu_count();
inline unsigned grid_cap(int64_t want, int64_t cap) {
  return (unsigned)(want < 1 ? 1 : (want > cap ? cap : want));
}

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

// rqsid_seg_auction_lap_half with a switch for the 8-byte-load sweeps (auction_seg.hip); vec is honoured
// only for one segment of N % 4 == 0 jobs with an 8-byte aligned score matrix.  single_layout: the caller laid
// the one segment out itself (seg_off = {0, n_jobs}, chunk_off = {0, chunks}: rqsid_auction_lap_half), so the
// round kernels may take that geometry without reading the tables (SegAuction::one_n)
int seg_auction_run(const uint16_t* scores, int32_t n_workers, int32_t n_seg, const int32_t* seg_off,
                    const int32_t* seg_chunk_off, int64_t total_chunks, int32_t n_multi, int64_t n_jobs,
                    const uint8_t* active, int32_t max_rounds, int32_t* out_assign, int32_t* out_rounds,
                    void* workspace, int64_t workspace_bytes, void* stream, bool vec, bool single_layout = false);

// exclusive-scan kernel shared by bucketing and the match-list builder (rqsid.hip)
__global__ __launch_bounds__(1024) void bucket_scan_kernel(const int32_t* __restrict__ counts, int S, int tile_rows,
                                   int32_t* __restrict__ row_off, int32_t* __restrict__ tile_off,
                                   int32_t* __restrict__ cursor);

}  // namespace rqsid
