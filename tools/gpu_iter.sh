#!/bin/bash
# GPU box, one development iteration: (1) the GPU tests selected by $K (pytest -k; empty = all),
# (2) the per-level screen sweep for every variant in $VARIANTS (RQSID_SCREEN_VARIANT).
# Every GPU step has its own time limit; any failure ends the script.  Output: gpurun_out/$TAG.
set -u
OUT=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-iter}
mkdir -p "$OUT"
export TMPDIR=/tmp SWEEP_CB=/tmp/sweep_cb.npz SWEEP_REPS=${SWEEP_REPS:-5}
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 ${TEST_T:-600} python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread \
    ${K:+-k "$K"} > "$OUT/tests.log" 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -15 "$OUT/tests.log"
  [ $rc -ne 0 ] && exit $rc
fi
for v in ${VARIANTS:-0}; do
  RQSID_SCREEN_VARIANT=$v timeout -k 10 300 python tools/screen_sweep.py > "$OUT/sweep_v$v.log" 2>&1 || { tail -20 "$OUT/sweep_v$v.log"; exit 1; }
  tail -1 "$OUT/sweep_v$v.log"
done
