set -u
OUT=$GRAFT_REPO_ROOT/gpurun_out/ab2
mkdir -p $OUT
export SWEEP_CB=/tmp/sweep_cb.npz SWEEP_REPS=5
timeout -k 10 300 python tools/screen_sweep.py > $OUT/base.log 2>&1 || exit 1
tail -1 $OUT/base.log
for v in 1 3; do
 for lib in tools/ab/librqsid_ab3.so tools/ab/librqsid_ab1.so generative_ranking_recommender_amd/librqsid.so; do
  RQSID_SCREEN_VARIANT=$v RQSID_LIB=$lib timeout -k 10 300 python tools/screen_sweep.py > $OUT/v$v.log 2>&1 || exit 1
  tail -1 $OUT/v$v.log
 done
done
