# GPU box: rocprofv3 kernel-trace summaries of the screen sweep for each library in $LIBS (variant $V)
set -u
export TMPDIR=/tmp SWEEP_CB=/tmp/sweep_cb.npz SWEEP_REPS=2
O=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-proflibs}; mkdir -p $O
timeout -k 10 300 python tools/screen_sweep.py > $O/warm.log 2>&1 || { tail $O/warm.log; exit 1; }
for lib in $LIBS; do
  n=$(basename $lib .so)
  (cd /tmp && RQSID_LIB=$GRAFT_REPO_ROOT/$lib RQSID_SCREEN_VARIANT=${V:-6} timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/$n -o run -- python3 $GRAFT_REPO_ROOT/tools/screen_sweep.py > $O/$n.log 2>&1) || { tail $O/$n.log; exit 1; }
  python tools/prof_summary.py $O/$n/run_results.db > $O/$n.txt
  echo "== $n"; grep -E "assign_resident|assign_screen" $O/$n.txt
done
