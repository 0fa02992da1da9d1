// auction.hip — the balanced assignment of balancekmeans.auction_lap_half (balancekmeans/__init__.py:12-140,
// SURVEY.md §8a row A5) as a sequence of dense passes over the fp16 score matrix on gfx950.
//
// Reference round (workers w = clusters, jobs j = rows, W = fp16(-distance) stored worker-major):
//   value[w][j] = W[w][j] if (w, j) won the previous round, else fp16(W[w][j] - cost[j])
//   each worker bids on its top jobs_per_worker = N / K jobs of value (torch.topk(jpw + 1)):
//       bid = fp16(fp16(value - (jpw+1)-th largest value) + eps)
//   retention (round < 100): the previous winner of j bids exactly eps on j   (bids.view(-1)[index] = eps)
//   leftovers (round > 1000): worker 0 bids eps on every job that had no bidder last round
//   each job goes to its highest bidder; stop when every job has one; else cost[j] = fp16(cost[j] + bid)
//
// The only implementation-defined step of the reference is which of several EQUAL values torch.topk /
// torch.max keep at the selection boundary.  Here the rule is fixed and documented: among values equal
// to the (jpw+1)-th largest, the lowest job indices are kept; among equal highest bids, the lowest worker
// wins.  oracle/rq_oracle.py auction_lap_half(tie_rule="stable") restates exactly this rule and
// tests/test_gpu_training.py and tests/test_gpu_batched.py check the kernels against it bit for bit.
//
// The passes (auction_seg.hip; all are coalesced sweeps over W, job-side state read once per block of
// 16 workers), per round:
//   P1 histogram of the high byte of a 16-bit order key of value, per worker
//   P2 histogram of the low byte inside the selected high-byte bin -> exact threshold key T[w]
//   P3 per-(worker, job chunk) count of values equal to T[w] (tie ranks)
//   P4 bids + overwrites, reduced to one packed {fp16 bid, ~worker} atomicMax per job and block
//   P5 per job: winner, cost update, bookkeeping; count of jobs with a bidder
#include <cmath>

#include "internal.h"

using namespace rqsid;

namespace {
constexpr int64_t kSmallAlign = 256;

__global__ void single_layout_kernel(int32_t* seg_off, int32_t* chunk_off, int32_t n, int32_t nch) {
  seg_off[0] = 0;
  seg_off[1] = n;
  chunk_off[0] = 0;
  chunk_off[1] = nch;
}

int64_t single_ws(int64_t n_jobs, int32_t n_workers) {
  const int64_t ch = rqsid_seg_auction_chunk_jobs();
  const int64_t nch = (n_jobs + ch - 1) / ch;
  return 3 * kSmallAlign + rqsid_seg_auction_workspace_bytes(n_jobs, n_workers, 1, nch, nch > 1 ? 1 : 0);
}
}  // namespace

extern "C" {

int64_t rqsid_auction_workspace_bytes(int64_t n_jobs, int32_t n_workers) {
  if (n_jobs < 0 || n_workers <= 0) return -1;
  return single_ws(n_jobs, n_workers);
}

// One auction = the segmented auction (auction_seg.hip) over a single segment: the same kernels, the
// same graph-captured round blocks.
int rqsid_auction_lap_half(const uint16_t* scores_wj, int32_t n_workers, int64_t n_jobs, int32_t max_rounds,
                           int32_t* out_assign, int32_t* out_rounds, void* workspace, int64_t workspace_bytes,
                           void* stream) {
  if (!scores_wj || !out_assign || n_workers <= 0 || n_jobs < 0 || n_jobs > INT32_MAX)
    return fail(RQSID_E_ARG, "auction: bad arguments (K=%d N=%lld)", n_workers, (long long)n_jobs);
  if (!workspace || workspace_bytes < single_ws(n_jobs, n_workers))
    return fail(RQSID_E_WORKSPACE, "auction: workspace too small");
  hipStream_t st = (hipStream_t)stream;
  if (out_rounds) *out_rounds = 0;
  if (n_jobs == 0) return RQSID_OK;
  if (n_workers == 1 && n_jobs >= 1)  // torch.topk(N + 1) would raise in the reference
    return fail(RQSID_E_ARG, "auction: a single worker cannot bid on N + 1 jobs");
  const int64_t ch = rqsid_seg_auction_chunk_jobs();
  const int64_t nch = (n_jobs + ch - 1) / ch;
  char* p = (char*)workspace;
  int32_t* seg_off = (int32_t*)p;
  int32_t* chunk_off = (int32_t*)(p + kSmallAlign);
  int32_t* rounds_dev = (int32_t*)(p + 2 * kSmallAlign);
  hipLaunchKernelGGL(single_layout_kernel, dim3(1), dim3(1), 0, st, seg_off, chunk_off, (int32_t)n_jobs,
                     (int32_t)nch);
  int rc = check_launch("auction_layout");
  if (rc) return rc;
  rc = seg_auction_run(scores_wj, n_workers, 1, seg_off, chunk_off, nch, nch > 1 ? 1 : 0, n_jobs, nullptr,
                       max_rounds, out_assign, rounds_dev, p + 3 * kSmallAlign, workspace_bytes - 3 * kSmallAlign,
                       stream, true);
  if (rc) return rc;
  int32_t r = 0;
  if (hipMemcpyAsync(&r, rounds_dev, 4, hipMemcpyDeviceToHost, st) != hipSuccess ||
      hipStreamSynchronize(st) != hipSuccess)
    return fail(RQSID_E_LAUNCH, "auction: readback");
  if (out_rounds) *out_rounds = r;
  return RQSID_OK;
}

}  // extern "C"
