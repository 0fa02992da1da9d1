#!/bin/bash
# GPU box, one call: the full GPU suite (with smoke), then tools/gpu_bench.sh (PMC traffic passes, the
# bench line with that traffic, the kernel-trace summary of the same bench command).  Output in
# gpurun_out/$TAG.  A crash or time-out (anything but pytest's "tests failed" = 1) ends the script.
set -u
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-round}
mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rA --timeout 120 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" "$OUT/gpu_tests.log" | tail -3
[ $rc -ne 0 ] && exit $rc
TAG=${TAG:-round} bash tools/gpu_bench.sh
