#!/bin/bash
# GPU box, round 4: multi-block list rounds: parity against the sweep / one-block form, then round times of
# the level-0 shapes (K=128 x 10M, K=256 x 6.25M: the XL per-rank share) with lists (default) and the sweep
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -v -s --timeout 300 --timeout-method thread -m gpu \
  "tests/test_gpu_training.py::test_auction_bid_list_equals_sweep" tests/test_gpu_reference_parity.py::test_candidate_fit_half_k1280_certified \
  > gpurun_out/r4_mlist_tests.log 2>&1 || { tail -30 gpurun_out/r4_mlist_tests.log; exit 1; }
grep -E "ms/round|passed|failed" gpurun_out/r4_mlist_tests.log
for shape in "--jobs 10000000 --workers 128" "--jobs 6250000 --workers 256"; do
  for mode in 1 0; do
    RQSID_AUCTION_LIST=$mode timeout -k 10 300 python tools/auction_bench.py $shape --reps 1 > gpurun_out/m.tmp 2>&1 || { tail -5 gpurun_out/m.tmp; exit 1; }
    tail -1 gpurun_out/m.tmp | sed "s/^{/{\"list_mode\": $mode, /" >> gpurun_out/r4_mlist_rounds.jsonl
  done
done
cat gpurun_out/r4_mlist_rounds.jsonl
