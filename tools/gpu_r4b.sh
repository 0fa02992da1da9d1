#!/bin/bash
# GPU box, round 4: reference / match-matrix parity and the training suites (auction list rounds, sharded
# resume, graph replay).
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 1100 python -u -m pytest -v -s --timeout 400 --timeout-method thread -m gpu \
  tests/test_gpu_match_parity.py tests/test_gpu_training.py tests/test_gpu_reference_parity.py \
  tests/test_gpu_sharded_train.py tests/test_gpu_batched.py tests/test_gpu_graph.py --durations=30 > gpurun_out/r4_parity_b.log 2>&1
rc=$?
grep -E "passed|failed|error" gpurun_out/r4_parity_b.log | tail -5
exit $rc
