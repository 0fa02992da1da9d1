#!/bin/bash
# GPU box, round 4: list-only round blocks (no sweep kernel launches while every list holds); training suite,
# candidate-fit shapes with list verdict counts, and a kernel trace of the K=2560 x 6.25M auction
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -v -s --timeout 300 --timeout-method thread -m gpu tests/test_gpu_training.py \
  tests/test_gpu_batched.py tests/test_gpu_reference_parity.py::test_candidate_fit_half_k1280_certified > gpurun_out/r4_train_suite5.log 2>&1 || { grep -E "FAIL|Error|error" gpurun_out/r4_train_suite5.log | head -20; tail -30 gpurun_out/r4_train_suite5.log; exit 1; }
grep -E "passed|failed" gpurun_out/r4_train_suite5.log
: > gpurun_out/r4_cand_rounds5.jsonl
for shape in "--jobs 1000000 --workers 1280" "--jobs 1000000 --workers 128" "--jobs 10000000 --workers 1280" "--jobs 6250000 --workers 2560" "--jobs 10000000 --workers 128" "--jobs 1280000 --workers 1280"; do
  RQSID_LIST_STATS=1 timeout -k 10 200 python tools/auction_bench.py $shape --reps 1 > gpurun_out/v.tmp 2>&1 || { tail -5 gpurun_out/v.tmp; exit 1; }
  grep "list stats" gpurun_out/v.tmp | tail -1
  tail -1 gpurun_out/v.tmp | sed "s/^{/{\"list_mode\": 1, /" >> gpurun_out/r4_cand_rounds5.jsonl
done
cat gpurun_out/r4_cand_rounds5.jsonl
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/r4_k2560_lonly
mkdir -p "$OUT"
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run -- python3 "$GRAFT_REPO_ROOT/tools/auction_bench.py" --jobs 6250000 --workers 2560 --reps 1 > "$OUT/prof.log" 2>&1) || { tail -5 "$OUT/prof.log"; exit 1; }
python tools/prof_summary.py "$OUT/prof/run_results.db" > "$OUT/kernels.txt" && head -16 "$OUT/kernels.txt"
rm -rf "$OUT/prof"
