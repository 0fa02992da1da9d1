#!/bin/bash
# GPU box: auction parity tests (default library), then per-round auction timing of the default library
# and of each A/B build named in $VARIANTS (tools/ab/librqsid_<v>.so), K=128 and K=1280 at 1M jobs and the
# segmented forms (128 segments x K=128: the middle layer; 1666 x K=256: the last layer's groups),
# then a kernel-trace summary of the default.  Output in gpurun_out/$TAG.
set -u
OUT=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-auc_ab}
mkdir -p "$OUT"
export TMPDIR=/tmp
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu ${TEST_FILES:-tests/test_gpu_training.py tests/test_gpu_batched.py tests/test_gpu_reference_parity.py tests/test_gpu_sharded_train.py} > "$OUT/tests.log" 2>&1
  rc=$?; tail -3 "$OUT/tests.log"; [ $rc -ne 0 ] && exit $rc
fi
for v in default ${VARIANTS:-}; do
  lib=""; [ "$v" != default ] && lib=tools/ab/librqsid_$v.so
  for cfg in "128 0" "1280 0" "128 128" "256 1666"; do
    set -- $cfg
    RQSID_LIB=${lib:-generative_ranking_recommender_amd/librqsid.so} timeout -k 10 200 python tools/auction_bench.py --jobs 1000000 --workers $1 --segments $2 --reps 2 > "$OUT/t_${v}_k$1_s$2.log" 2>&1 || { tail -5 "$OUT/t_${v}_k$1_s$2.log"; exit 1; }
    echo "$v $(tail -1 "$OUT/t_${v}_k$1_s$2.log")"
  done
done
[ "${PROF:-1}" = 1 ] && TAG=${TAG:-auc_ab} PMC=0 bash tools/gpu_auction_prof.sh
exit 0
