#!/bin/bash
# GPU box, round 4: the sweep kernels exit at once in rounds where every list held (lany); training suite
# (auction parity, list forms), then the candidate-fit shapes with list verdict counts, lists vs sweep
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -v -s --timeout 300 --timeout-method thread -m gpu tests/test_gpu_training.py \
  tests/test_gpu_batched.py tests/test_gpu_reference_parity.py::test_candidate_fit_half_k1280_certified > gpurun_out/r4_train_suite3.log 2>&1 || { grep -E "FAIL|Error|error" gpurun_out/r4_train_suite3.log | head -20; tail -30 gpurun_out/r4_train_suite3.log; exit 1; }
grep -E "ms/round|passed|failed" gpurun_out/r4_train_suite3.log
: > gpurun_out/r4_cand_rounds3.jsonl
for shape in "--jobs 1000000 --workers 1280" "--jobs 1000000 --workers 128" "--jobs 10000000 --workers 1280" "--jobs 6250000 --workers 2560" "--jobs 10000000 --workers 128"; do
  RQSID_LIST_STATS=1 timeout -k 10 200 python tools/auction_bench.py $shape --reps 1 > gpurun_out/u.tmp 2>&1 || { tail -5 gpurun_out/u.tmp; exit 1; }
  grep "list stats" gpurun_out/u.tmp | tail -1
  tail -1 gpurun_out/u.tmp | sed "s/^{/{\"list_mode\": 1, /" >> gpurun_out/r4_cand_rounds3.jsonl
done
cat gpurun_out/r4_cand_rounds3.jsonl
