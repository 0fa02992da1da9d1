#!/bin/bash
# GPU box, round 4: PROD training (10M rows, [128,128,256]) after the list-only auction blocks
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 1000 python -u tools/train_bench.py --rows 10000000 --data bench --out gpurun_out/r4_train_bench_10m_listonly.json \
  > gpurun_out/r4_train_10m_listonly.log 2>&1
rc=$?
tail -3 gpurun_out/r4_train_10m_listonly.log
exit $rc
