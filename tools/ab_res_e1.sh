#!/bin/bash
# GPU box: A/B of the centre-resident screen's epilogue-1 variants (tools/ab/librqsid_e1v{0,1}.so, built
# with -DRQ_E1V2=0/1) against the default dispatch, per encode level (tools/screen_sweep.py), then the
# resident-form parity tests under the new variant.  Output in gpurun_out/$TAG.
set -u
OUT=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-ab_e1}
mkdir -p "$OUT"
export TMPDIR=/tmp SWEEP_CB=/tmp/sweep_cb.npz SWEEP_REPS=${SWEEP_REPS:-5}
timeout -k 10 300 python tools/screen_sweep.py > "$OUT/default.log" 2>&1 || { tail -5 "$OUT/default.log"; exit 1; }
tail -1 "$OUT/default.log"
for v in 0 1 1la7; do
  RQSID_SCREEN_VARIANT=6 RQSID_LIB=tools/ab/librqsid_e1v$v.so timeout -k 10 300 python tools/screen_sweep.py > "$OUT/res_e1v$v.log" 2>&1 || { tail -5 "$OUT/res_e1v$v.log"; exit 1; }
  tail -1 "$OUT/res_e1v$v.log"
done
RQSID_LIB=tools/ab/librqsid_e1v1.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k "res" -q --timeout 300 --timeout-method thread > "$OUT/parity_e1v1.log" 2>&1
rc=$?; tail -3 "$OUT/parity_e1v1.log"; exit $rc
