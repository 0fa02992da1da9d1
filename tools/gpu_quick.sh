#!/bin/bash
# GPU box: parity tests (gpu marker) then the per-level screen sweep (default library + any A/B libs in $LIBS).
set -u
OUT=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-quick}
mkdir -p "$OUT"
export TMPDIR=/tmp SWEEP_CB=/tmp/sweep_cb.npz SWEEP_REPS=${SWEEP_REPS:-5}
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 ${TEST_T:-600} python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} > "$OUT/tests.log" 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -15 "$OUT/tests.log"
  [ $rc -ne 0 ] && exit $rc
fi
timeout -k 10 300 python tools/screen_sweep.py > "$OUT/sweep.log" 2>&1 || { tail -20 "$OUT/sweep.log"; exit 1; }
tail -1 "$OUT/sweep.log"
for v in ${VARIANTS:-}; do
  RQSID_SCREEN_VARIANT=$v timeout -k 10 300 python tools/screen_sweep.py > "$OUT/sweep_v$v.log" 2>&1 || { tail -20 "$OUT/sweep_v$v.log"; exit 1; }
  tail -1 "$OUT/sweep_v$v.log"
done
for lib in ${LIBS:-}; do
  n=$(basename $lib .so)
  RQSID_LIB=$lib timeout -k 10 300 python tools/screen_sweep.py > "$OUT/$n.log" 2>&1 || { tail -20 "$OUT/$n.log"; exit 1; }
  tail -1 "$OUT/$n.log"
done
