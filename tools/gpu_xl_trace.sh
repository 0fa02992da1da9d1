#!/bin/bash
# GPU box: rocprofv3 kernel-trace summary of the XL encode bench (no CPU leg).  Output in gpurun_out/$TAG.
set -u
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-xltrace}
mkdir -p "$OUT"
(cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --preset xl --no-cpu --config0 0 --steps 5 --warmup 2 ${BENCH_EXTRA:-} > "$OUT/bench.json" 2> "$OUT/prof.err") || { tail -20 "$OUT/prof.err"; exit 1; }
python tools/prof_summary.py "$OUT/prof/run_results.db" > "$OUT/kernels.txt" && head -24 "$OUT/kernels.txt"
rm -rf "$OUT/prof/"*.db "$OUT/prof/"*/ 2>/dev/null
