#!/bin/bash
# GPU box: per-level rqsid_assign times (tools/screen_sweep.py) of the default library and of each A/B
# build in $VARIANTS (tools/ab/librqsid_<v>.so), default again at the end (box noise), then the
# screen parity tests under the first variant.  Output in gpurun_out/$TAG.
set -u
OUT=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-screen_ab}
mkdir -p "$OUT"
export TMPDIR=/tmp SWEEP_CB=/tmp/sweep_cb.npz SWEEP_REPS=${SWEEP_REPS:-5}
for v in default ${VARIANTS:-} default2; do
  lib=generative_ranking_recommender_amd/librqsid.so
  case $v in default|default2) ;; *) lib=tools/ab/librqsid_$v.so ;; esac
  RQSID_LIB=$lib timeout -k 10 300 python tools/screen_sweep.py > "$OUT/$v.log" 2>&1 || { tail -5 "$OUT/$v.log"; exit 1; }
  echo "$v: $(tail -1 "$OUT/$v.log")"
done
first=$(echo ${VARIANTS:-} | awk '{print $1}')
if [ -n "$first" ] && [ "${PARITY:-1}" = 1 ]; then
  RQSID_LIB=tools/ab/librqsid_$first.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -q --timeout 300 --timeout-method thread > "$OUT/parity_$first.log" 2>&1
  rc=$?; tail -2 "$OUT/parity_$first.log"; exit $rc
fi
