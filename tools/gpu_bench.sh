#!/bin/bash
# GPU box: PMC traffic passes, the default bench line (with that traffic), and the rocprofv3 kernel-trace
# summary of the same bench command.  Output in gpurun_out/$TAG.
set -u
OUT=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-bench}
mkdir -p "$OUT"
export TMPDIR=/tmp
TAG=${TAG:-bench}/traffic bash tools/pmc_traffic.sh > "$OUT/traffic.log" 2>&1 || { tail -20 "$OUT/traffic.log"; exit 1; }
timeout -k 10 600 python bench.py --traffic-json "$OUT/traffic/traffic.json" > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -20 "$OUT/bench.err"; exit 1; }
cat "$OUT/bench.json"
(cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --no-cpu --traffic-json "$OUT/traffic/traffic.json" > "$OUT/prof_bench.json" 2> "$OUT/prof.err") || { tail -20 "$OUT/prof.err"; exit 1; }
python tools/prof_summary.py "$OUT/prof/run_results.db" > "$OUT/kernels.txt" && head -12 "$OUT/kernels.txt"
# keep gpurun_out small (the merge back is capped at 64 MiB): drop the raw databases once summarised
rm -rf "$OUT/prof/"*.db "$OUT/prof/"*/ "$OUT/traffic/p1" "$OUT/traffic/p2" 2>/dev/null
du -sh "$OUT"
