#!/bin/bash
# GPU box: single-auction and lockstep round times with the bid lists (RQSID_AUCTION_LIST=1, default) and the
# sweep (0), then a kernel-trace summary of the K=1280 x 1M list run.  Output in gpurun_out/$TAG.
set -u
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-auction_list}
mkdir -p "$OUT"
for mode in 1 0; do
  for shape in "--jobs 1000000 --workers 128" "--jobs 1000000 --workers 1280" "--jobs 1000000 --workers 128 --segments 128"; do
    RQSID_AUCTION_LIST=$mode timeout -k 10 300 python tools/auction_bench.py $shape --reps 2 > "$OUT/run.tmp" 2>&1 || { tail -5 "$OUT/run.tmp"; exit 1; }
    tail -1 "$OUT/run.tmp" | sed "s/^{/{\"list\": $mode, /" >> "$OUT/rounds.jsonl"
  done
done
cat "$OUT/rounds.jsonl"
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run -- python3 "$GRAFT_REPO_ROOT/tools/auction_bench.py" --jobs 1000000 --workers 1280 --reps 1 > "$OUT/prof.out" 2> "$OUT/prof.err") || { tail -20 "$OUT/prof.err"; exit 1; }
python tools/prof_summary.py "$OUT/prof/run_results.db" > "$OUT/kernels_k1280.txt" && head -16 "$OUT/kernels_k1280.txt"
rm -rf "$OUT/prof/"*.db "$OUT/prof/"*/ 2>/dev/null
