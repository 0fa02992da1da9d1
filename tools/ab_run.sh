#!/bin/bash
# GPU box: screen_sweep with the default library (fits + caches the codebooks), then each A/B build.
set -u
OUT=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-ab}
mkdir -p "$OUT"
export SWEEP_CB=/tmp/sweep_cb.npz SWEEP_REPS=${SWEEP_REPS:-5}
timeout -k 10 300 python tools/screen_sweep.py > "$OUT/base.log" 2>&1 || { tail -20 "$OUT/base.log"; exit 1; }
tail -1 "$OUT/base.log"
for lib in ${LIBS:-tools/ab/librqsid_ab1.so tools/ab/librqsid_ab2.so tools/ab/librqsid_ab3.so}; do
  n=$(basename $lib .so)
  RQSID_LIB=$lib timeout -k 10 300 python tools/screen_sweep.py > "$OUT/$n.log" 2>&1 || { tail -20 "$OUT/$n.log"; exit 1; }
  tail -1 "$OUT/$n.log"
done
