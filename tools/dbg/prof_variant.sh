# GPU box: rocprofv3 kernel-trace summary of the screen sweep for RQSID_SCREEN_VARIANT=$V
set -u
export TMPDIR=/tmp SWEEP_CB=/tmp/sweep_cb.npz SWEEP_REPS=3
O=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-profv}; mkdir -p $O
timeout -k 10 300 python tools/screen_sweep.py > $O/warm.log 2>&1 || { tail $O/warm.log; exit 1; }
(cd /tmp && RQSID_SCREEN_VARIANT=${V:-0} timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 $GRAFT_REPO_ROOT/tools/screen_sweep.py > $O/prof.log 2>&1) || { tail $O/prof.log; exit 1; }
python tools/prof_summary.py $O/prof/run_results.db > $O/kernels.txt && head -20 $O/kernels.txt
