set -u
export TMPDIR=/tmp SWEEP_CB=/tmp/sweep_cb.npz SWEEP_REPS=3
O=gpurun_out/${TAG:-st}; mkdir -p $O
timeout -k 10 300 python tools/screen_sweep.py > $O/sweep.log 2>&1 || { tail $O/sweep.log; exit 1; }
tail -1 $O/sweep.log
for lib in ${LIBS}; do
  echo "== $lib"
  RQSID_SCREEN_VARIANT=6 RQSID_LIB=$lib timeout -k 10 300 python tools/res_stamps.py > $O/$(basename $lib).log 2>&1 || { tail $O/$(basename $lib).log; exit 1; }
  grep L2 $O/$(basename $lib).log
done
