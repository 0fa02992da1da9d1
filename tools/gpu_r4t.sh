#!/bin/bash
# GPU box, round 4: why the large candidate-fit auctions still sweep: list verdict counts (RQSID_LIST_STATS)
# and round times for list margins of 64, 96 and 128 keys (RQSID_LIST_DELTA)
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
: > gpurun_out/r4_list_delta.jsonl
for shape in "--jobs 1000000 --workers 1280" "--jobs 6250000 --workers 2560" "--jobs 10000000 --workers 1280"; do
  for d in 64 128 96; do
    RQSID_LIST_STATS=1 RQSID_LIST_DELTA=$d timeout -k 10 200 python tools/auction_bench.py $shape --reps 1 > gpurun_out/t.tmp 2>&1 || { tail -5 gpurun_out/t.tmp; exit 1; }
    grep "list stats" gpurun_out/t.tmp | tail -1 | sed "s/^/delta $d: /"
    tail -1 gpurun_out/t.tmp | sed "s/^{/{\"delta\": $d, /" >> gpurun_out/r4_list_delta.jsonl
  done
done
cat gpurun_out/r4_list_delta.jsonl
