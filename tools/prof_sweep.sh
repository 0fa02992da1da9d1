#!/bin/bash
# GPU box: rocprofv3 kernel trace of the per-level sweep (codebooks cached in /tmp), summary to gpurun_out/$TAG
set -u
OUT=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-profsweep}
mkdir -p "$OUT"
export TMPDIR=/tmp SWEEP_CB=/tmp/sweep_cb.npz SWEEP_REPS=${SWEEP_REPS:-3}
timeout -k 10 300 python tools/screen_sweep.py > "$OUT/warm.log" 2>&1 || { tail -5 "$OUT/warm.log"; exit 1; }
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run -- python3 "$GRAFT_REPO_ROOT/tools/screen_sweep.py" > "$OUT/prof.log" 2>&1
rc=$?; echo "prof rc=$rc"; tail -2 "$OUT/prof.log"
cd "$GRAFT_REPO_ROOT" && python tools/prof_summary.py "$OUT/prof/run_results.db" > "$OUT/kernels.txt" && head -25 "$OUT/kernels.txt"
