#!/bin/bash
# GPU box, round 4: row-staging probe, bench A/B of the row-resident screen, then the encode parity suite.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 150 ./tools/probe/stage_probe > gpurun_out/r4_stage_probe.txt 2>&1 || { echo "probe failed"; exit 1; }
TAG=r4_rows AB="default:- rows443:RQSID_SCREEN_VARIANT=8,RQSID_ROWS_SHAPE=443 rows482:RQSID_SCREEN_VARIANT=8,RQSID_ROWS_SHAPE=482 rows883:RQSID_SCREEN_VARIANT=8,RQSID_ROWS_SHAPE=883" \
  PARITY=2048 timeout -k 10 420 bash tools/gpu_ab_env.sh > gpurun_out/r4_rows_ab.txt 2>&1 || { echo "ab failed"; cat gpurun_out/r4_rows_ab.txt; exit 1; }
cat gpurun_out/r4_rows_ab.txt
timeout -k 10 580 python -u -m pytest -v -s --timeout 400 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  --durations=20 > gpurun_out/r4_parity_a.log 2>&1
rc=$?
tail -5 gpurun_out/r4_parity_a.log
exit $rc
