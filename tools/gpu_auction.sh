#!/bin/bash
# GPU box: auction parity tests, auction timings and a kernel-trace of one auction.  Output in gpurun_out/$TAG.
set -u
OUT=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-auction}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 ${TEST_T:-600} python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_batched.py tests/test_gpu_training.py > "$OUT/tests.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 "$OUT/tests.log"
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/auction_bench.py --jobs 1000000 --workers 128 > "$OUT/bench_k128.json" 2>&1 || exit 1
timeout -k 10 300 python tools/auction_bench.py --jobs 100000 --workers 1280 > "$OUT/bench_k1280.json" 2>&1 || exit 1
cat "$OUT"/bench_k*.json
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run -- python3 "$GRAFT_REPO_ROOT/tools/auction_bench.py" --jobs 1000000 --workers 128 --reps 1 > "$OUT/prof.log" 2>&1 || exit 1
cd "$GRAFT_REPO_ROOT" && python tools/prof_summary.py "$OUT/prof/run_results.db" > "$OUT/kernels.txt" && head -16 "$OUT/kernels.txt"
