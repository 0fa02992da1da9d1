#!/bin/bash
# GPU box: kernel-trace summary of one auction (K=$K x 1M) under the default library and each A/B build in
# $VARIANTS (tools/ab/librqsid_<v>.so).  Timing only: A/B builds may compute wrong results.
set -u
OUT=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-abprof}
mkdir -p "$OUT"
export TMPDIR=/tmp
for v in default ${VARIANTS:-}; do
  lib=$GRAFT_REPO_ROOT/generative_ranking_recommender_amd/librqsid.so; [ "$v" != default ] && lib=$GRAFT_REPO_ROOT/tools/ab/librqsid_$v.so
  (cd /tmp && RQSID_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/p_$v" -o run -- python3 "$GRAFT_REPO_ROOT/tools/auction_bench.py" --jobs 1000000 --workers ${K:-128} --segments ${S:-0} --reps 1 > "$OUT/p_$v.log" 2>&1) || { tail -5 "$OUT/p_$v.log"; exit 1; }
  python tools/prof_summary.py "$OUT/p_$v/run_results.db" > "$OUT/k_$v.txt" && echo "== $v" && sed -n 3,8p "$OUT/k_$v.txt" | cut -c1-100
  rm -rf "$OUT/p_$v"
done
exit 0
