#!/bin/bash
# GPU box, round 4: encode parity suite (duplicate centres, re-screen, re-score passes), the re-score cliff
# diagnostic, and a kernel trace of the default bench (the longest re-screen / re-score launches).
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  > gpurun_out/r4_parity_i.log 2>&1 || { tail -20 gpurun_out/r4_parity_i.log; exit 1; }
tail -2 gpurun_out/r4_parity_i.log
timeout -k 10 300 python -u tools/diag_rescreen.py > gpurun_out/r4_diag_rescreen2.txt 2>&1 || { tail -5 gpurun_out/r4_diag_rescreen2.txt; exit 1; }
cat gpurun_out/r4_diag_rescreen2.txt
OUT=$GRAFT_REPO_ROOT/gpurun_out/r4_trace2
mkdir -p $OUT
(cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --no-cpu > "$OUT/bench.json" 2> "$OUT/prof.err") || { tail -20 "$OUT/prof.err"; exit 1; }
python tools/prof_summary.py "$OUT/prof/run_results.db" > "$OUT/kernels.txt" && head -20 "$OUT/kernels.txt"
rm -rf "$OUT/prof/"*.db "$OUT/prof/"*/ 2>/dev/null
