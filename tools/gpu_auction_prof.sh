#!/bin/bash
# GPU box: kernel-trace summaries of one auction at K=128 x 1M and K=1280 x 1M jobs, then PMC passes of
# the K=128 x 1M auction's sweep kernels.  Output in gpurun_out/$TAG.
set -u
OUT=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-aprof}
mkdir -p "$OUT"
export TMPDIR=/tmp
for kw in "1000000 128" "1000000 1280"; do
  set -- $kw
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_k$2" -o run -- python3 "$GRAFT_REPO_ROOT/tools/auction_bench.py" --jobs $1 --workers $2 --reps 1 > "$OUT/prof_k$2.log" 2>&1) || { tail -5 "$OUT/prof_k$2.log"; exit 1; }
  python tools/prof_summary.py "$OUT/prof_k$2/run_results.db" > "$OUT/kernels_k$2.txt" && head -14 "$OUT/kernels_k$2.txt"
  tail -1 "$OUT/prof_k$2.log"
  rm -rf "$OUT/prof_k$2"
done
[ "${PMC:-1}" = 1 ] && TAG=${TAG:-aprof}/pmc CMD="tools/auction_bench.py --jobs 1000000 --workers 128 --reps 1" KREGEX="sa_bid|sa_hist|sa_resolve" bash tools/pmc_cmd.sh
exit 0
