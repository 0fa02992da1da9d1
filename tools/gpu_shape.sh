#!/bin/bash
# GPU box: stream-kernel parity tests for each block shape, then the per-level sweep of the per-tile
# kernel (variant 0) and of the stream kernel per shape.  Output in gpurun_out/$TAG.
set -u
OUT=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-shape}
mkdir -p "$OUT"
export TMPDIR=/tmp SWEEP_CB=/tmp/sweep_cb.npz SWEEP_REPS=${SWEEP_REPS:-5}
for sh in ${SHAPES:-42 83}; do
  RQSID_STREAM_SHAPE=$sh timeout -k 10 ${TEST_T:-400} python -u -m pytest tests -m gpu -x -q -rf --timeout 200 --timeout-method thread -k "${TESTK:-stream}" > "$OUT/tests_$sh.log" 2>&1
  rc=$?; echo "shape $sh pytest rc=$rc"; tail -3 "$OUT/tests_$sh.log"
  [ $rc -ne 0 ] && exit $rc
done
timeout -k 10 300 python tools/screen_sweep.py > "$OUT/sweep_v0.log" 2>&1 || { tail -20 "$OUT/sweep_v0.log"; exit 1; }
tail -1 "$OUT/sweep_v0.log"
for sh in ${SHAPES:-42 83}; do
  RQSID_SCREEN_VARIANT=5 RQSID_STREAM_SHAPE=$sh timeout -k 10 300 python tools/screen_sweep.py > "$OUT/sweep_s$sh.log" 2>&1 || { tail -20 "$OUT/sweep_s$sh.log"; exit 1; }
  echo "shape $sh: $(tail -1 $OUT/sweep_s$sh.log)"
done
