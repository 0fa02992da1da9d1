#!/bin/bash
# GPU box, round 4: single auction K=128 x 10M jobs (level 0 of 10M training): sweep vs bid lists forced on
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for mode in 0 2 1; do
  RQSID_AUCTION_LIST=$mode timeout -k 10 300 python tools/auction_bench.py --jobs 10000000 --workers 128 --reps 1 > gpurun_out/k.tmp 2>&1 || { tail -5 gpurun_out/k.tmp; exit 1; }
  tail -1 gpurun_out/k.tmp | sed "s/^{/{\"list_mode\": $mode, /" >> gpurun_out/r4_auction_10m.jsonl
done
cat gpurun_out/r4_auction_10m.jsonl
