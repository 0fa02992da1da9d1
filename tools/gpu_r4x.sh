#!/bin/bash
# GPU box, round 4: first list-building round (RQSID_LIST_START 32 / 16 / 8) on the candidate-fit shapes,
# a settling auction (N % K == 0) and K=128
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
: > gpurun_out/r4_list_start.jsonl
for shape in "--jobs 6250000 --workers 2560" "--jobs 10000000 --workers 1280" "--jobs 1000000 --workers 1280" "--jobs 1280000 --workers 1280" "--jobs 1000000 --workers 128"; do
  for ls in 32 16 8; do
    RQSID_LIST_STATS=1 RQSID_LIST_START=$ls timeout -k 10 200 python tools/auction_bench.py $shape --reps 1 > gpurun_out/x.tmp 2>&1 || { tail -5 gpurun_out/x.tmp; exit 1; }
    grep "list stats" gpurun_out/x.tmp | tail -1 | sed "s/^/start $ls: /"
    tail -1 gpurun_out/x.tmp | sed "s/^{/{\"list_start\": $ls, /" >> gpurun_out/r4_list_start.jsonl
  done
done
cat gpurun_out/r4_list_start.jsonl
