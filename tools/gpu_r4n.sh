#!/bin/bash
# GPU box, round 4: the training suite (auction parity incl. both list forms) and the auction round times of
# every list shape, lists (default) vs sweep
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -v -s --timeout 300 --timeout-method thread -m gpu tests/test_gpu_training.py \
  > gpurun_out/r4_train_suite.log 2>&1 || { tail -30 gpurun_out/r4_train_suite.log; exit 1; }
grep -E "ms/round|passed|failed" gpurun_out/r4_train_suite.log
for shape in "--jobs 1000000 --workers 128" "--jobs 1000000 --workers 1280" "--jobs 1000000 --workers 128 --segments 128" \
             "--jobs 10000000 --workers 128" "--jobs 6250000 --workers 256"; do
  for mode in 1 0; do
    RQSID_AUCTION_LIST=$mode timeout -k 10 300 python tools/auction_bench.py $shape --reps 1 > gpurun_out/n.tmp 2>&1 || { tail -5 gpurun_out/n.tmp; exit 1; }
    tail -1 gpurun_out/n.tmp | sed "s/^{/{\"list_mode\": $mode, /" >> gpurun_out/r4_list_rounds_final.jsonl
  done
done
cat gpurun_out/r4_list_rounds_final.jsonl
