#!/bin/bash
# GPU box, round 4: XL encode (configs[4] per-rank share, 6.25M rows): PMC traffic of the default kernels
# (now the row-resident screen at level 2), the bench line with it, and its kernel-trace summary.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/r4_xl
mkdir -p "$OUT"
TAG=r4_xl/traffic BENCH_ARGS="--preset xl" timeout -k 10 500 bash tools/pmc_traffic.sh > "$OUT/traffic.log" 2>&1 || { tail -20 "$OUT/traffic.log"; exit 1; }
timeout -k 10 400 python bench.py --preset xl --no-cpu --traffic-json "$OUT/traffic/traffic.json" > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -20 "$OUT/bench.err"; exit 1; }
cat "$OUT/bench.json"
rm -rf "$OUT/traffic/p1" "$OUT/traffic/p2" 2>/dev/null
