#!/bin/bash
# GPU box, round 4: the bench line with PMC traffic and its kernel-trace summary (gpurun_out/r4), then the
# auction bid-list round times (gpurun_out/r4_auction).
set -u
cd "$GRAFT_REPO_ROOT"
TAG=r4 timeout -k 10 780 bash tools/gpu_bench.sh || { echo "bench failed"; exit 1; }
TAG=r4_auction timeout -k 10 360 bash tools/gpu_auction_list.sh || { echo "auction list failed"; exit 1; }
