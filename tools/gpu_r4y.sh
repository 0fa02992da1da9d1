#!/bin/bash
# GPU box, round 4 end: the whole GPU suite in one process, the default bench line (PMC traffic, kernel
# trace: gpurun_out/r4_final), then the candidate-fit auction shapes with the final list settings
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -q --timeout 400 --timeout-method thread -m gpu tests/ --durations=15 \
  > gpurun_out/r4_final2_gpu_tests.log 2>&1 || { tail -30 gpurun_out/r4_final2_gpu_tests.log; exit 1; }
tail -3 gpurun_out/r4_final2_gpu_tests.log
TAG=r4_final2 timeout -k 10 280 bash tools/gpu_bench.sh || { echo "bench failed"; exit 1; }
: > gpurun_out/r4_cand_rounds_final.jsonl
for shape in "--jobs 6250000 --workers 2560" "--jobs 10000000 --workers 1280" "--jobs 1000000 --workers 1280" "--jobs 1280000 --workers 1280" "--jobs 1000000 --workers 128"; do
  timeout -k 10 200 python tools/auction_bench.py $shape --reps 1 > gpurun_out/y.tmp 2>&1 || { tail -5 gpurun_out/y.tmp; exit 1; }
  tail -1 gpurun_out/y.tmp >> gpurun_out/r4_cand_rounds_final.jsonl
done
cat gpurun_out/r4_cand_rounds_final.jsonl
