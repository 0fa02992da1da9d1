#!/bin/bash
# GPU box, round 4: PROD training end to end at 10M rows (bench rows), per-layer / per-phase seconds.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 1120 python -u tools/train_bench.py --rows 10000000 --data bench --out gpurun_out/r4_train_bench_10m.json \
  > gpurun_out/r4_train_10m.log 2>&1
rc=$?
tail -3 gpurun_out/r4_train_10m.log
exit $rc
