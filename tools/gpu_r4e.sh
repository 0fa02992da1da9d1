#!/bin/bash
# GPU box, round 4: XL encode (configs[4] per-rank share, 6.25M rows): kernel-trace summary of the default
# bench, then the row-resident screen at the 512-candidate last level (A/B line).
set -u
cd "$GRAFT_REPO_ROOT"
TAG=r4_xltrace timeout -k 10 480 bash tools/gpu_xl_trace.sh || { echo "xl trace failed"; exit 1; }
cat gpurun_out/r4_xltrace/bench.json
TAG=r4_xl_rows BENCH_ARGS="--preset xl" STEPS=5 AB="rows883:RQSID_SCREEN_VARIANT=8,RQSID_ROWS_SHAPE=883 rows443:RQSID_SCREEN_VARIANT=8,RQSID_ROWS_SHAPE=443" \
  PARITY=2048 timeout -k 10 420 bash tools/gpu_ab_env.sh > gpurun_out/r4_xl_rows_ab.txt 2>&1 || { echo "xl ab failed"; cat gpurun_out/r4_xl_rows_ab.txt; exit 1; }
cat gpurun_out/r4_xl_rows_ab.txt
