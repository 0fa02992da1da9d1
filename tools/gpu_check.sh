#!/bin/bash
# GPU-box driver: parity tests, then a short bench, then a rocprofv3 kernel-trace of the bench.
# Every GPU step has its own time limit; a crash/timeout (anything but pytest's "tests failed" = 1)
# ends the script so nothing more touches the GPU.
set -u
OUT=gpurun_out/${TAG:-run}
mkdir -p "$OUT"
export TMPDIR=/tmp
fatal() { case "$1" in 0|1) return 1;; *) return 0;; esac; }
timeout -k 10 ${TEST_T:-900} python -m pytest tests -m gpu -q -rA ${PYTEST_ARGS:-} > "$OUT/gpu_tests.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -30 "$OUT/gpu_tests.log"
if fatal $rc; then exit $rc; fi
[ "${SKIP_BENCH:-0}" = 1 ] && exit $rc
timeout -k 10 ${BENCH_T:-600} python bench.py ${BENCH_ARGS:-} > "$OUT/bench.log" 2>&1
rc2=$?; echo "bench rc=$rc2"; tail -5 "$OUT/bench.log"
if [ $rc2 -ne 0 ]; then exit $rc2; fi
[ "${SKIP_PROF:-0}" = 1 ] && exit $rc
cd /tmp && timeout -k 10 ${PROF_T:-600} rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$OUT/prof" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --no-cpu ${BENCH_ARGS:-} > "$GRAFT_REPO_ROOT/$OUT/prof.log" 2>&1
rc3=$?; echo "prof rc=$rc3"; tail -5 "$GRAFT_REPO_ROOT/$OUT/prof.log"
exit $rc3
