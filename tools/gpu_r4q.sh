#!/bin/bash
# GPU box, round 4: the candidate-fit auction shapes at full size (K=1280 x 10M PROD, K=2560 x 6.25M XL per-rank
# share), lists vs sweep, and a kernel trace of the XL shape with lists
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
for shape in "--jobs 10000000 --workers 1280" "--jobs 6250000 --workers 2560"; do
  for mode in 1 0; do
    RQSID_AUCTION_LIST=$mode timeout -k 10 200 python tools/auction_bench.py $shape --reps 1 > gpurun_out/q.tmp 2>&1 || { tail -5 gpurun_out/q.tmp; exit 1; }
    tail -1 gpurun_out/q.tmp | sed "s/^{/{\"list_mode\": $mode, /" >> gpurun_out/r4_cand_rounds.jsonl
  done
done
cat gpurun_out/r4_cand_rounds.jsonl
OUT=$GRAFT_REPO_ROOT/gpurun_out/r4_cand_trace
mkdir -p $OUT
(cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run -- python3 "$GRAFT_REPO_ROOT/tools/auction_bench.py" --jobs 6250000 --workers 2560 --reps 1 > "$OUT/out.txt" 2> "$OUT/err.txt") || { tail -5 "$OUT/err.txt"; exit 1; }
python tools/prof_summary.py "$OUT/prof/run_results.db" > "$OUT/kernels.txt" && head -16 "$OUT/kernels.txt"
rm -rf "$OUT/prof/"*.db "$OUT/prof/"*/ 2>/dev/null
