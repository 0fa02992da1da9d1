#!/bin/bash
# GPU box, round 4 end: the whole GPU suite in one process, then the default bench line with PMC traffic and
# its kernel trace (gpurun_out/r4_final).
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -q --timeout 400 --timeout-method thread -m gpu tests/ --durations=15 \
  > gpurun_out/r4_final_gpu_tests.log 2>&1 || { tail -30 gpurun_out/r4_final_gpu_tests.log; exit 1; }
tail -3 gpurun_out/r4_final_gpu_tests.log
TAG=r4_final timeout -k 10 280 bash tools/gpu_bench.sh || { echo "bench failed"; exit 1; }
