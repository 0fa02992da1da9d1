#!/bin/bash
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/diag_rescreen.py > gpurun_out/r4_diag_rescreen.txt 2>&1
rc=$?
cat gpurun_out/r4_diag_rescreen.txt | tail -8
exit $rc
