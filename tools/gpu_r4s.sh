#!/bin/bash
# GPU box, round 4: training suite (auction parity, list forms) after the tie radix select, then the
# candidate-fit auction shapes at full size, lists vs sweep
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -v -s --timeout 300 --timeout-method thread -m gpu tests/test_gpu_training.py \
  tests/test_gpu_reference_parity.py::test_candidate_fit_half_k1280_certified > gpurun_out/r4_train_suite2.log 2>&1 || { tail -30 gpurun_out/r4_train_suite2.log; exit 1; }
grep -E "ms/round|passed|failed" gpurun_out/r4_train_suite2.log
for shape in "--jobs 1000000 --workers 1280" "--jobs 10000000 --workers 1280" "--jobs 6250000 --workers 2560"; do
  for mode in 1 0; do
    RQSID_AUCTION_LIST=$mode timeout -k 10 200 python tools/auction_bench.py $shape --reps 1 > gpurun_out/s.tmp 2>&1 || { tail -5 gpurun_out/s.tmp; exit 1; }
    tail -1 gpurun_out/s.tmp | sed "s/^{/{\"list_mode\": $mode, /" >> gpurun_out/r4_cand_rounds2.jsonl
  done
done
cat gpurun_out/r4_cand_rounds2.jsonl
