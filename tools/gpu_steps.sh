#!/bin/bash
# GPU box: run a list of steps, each under its own time limit, stopping at the first failure.
#   bash tools/gpu_steps.sh TAG 'name|seconds|command' ['name|seconds|command' ...]
# Output of step `name` goes to gpurun_out/TAG/name.log (its last lines are echoed).  A step that fails, times
# out or crashes ends the script with its status, so nothing more runs on the GPU after a fault.  Replaces the
# one-off per-experiment call scripts of rounds 1-4 (their commands are in git history).
set -u
TAG=$1
shift
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
for step in "$@"; do
  name=${step%%|*}
  rest=${step#*|}
  secs=${rest%%|*}
  cmd=${rest#*|}
  echo "== $name ($secs s): $cmd"
  timeout -k 10 "$secs" bash -c "$cmd" > "$OUT/$name.log" 2>&1
  rc=$?
  tail -${TAIL:-8} "$OUT/$name.log"
  if [ $rc -ne 0 ]; then
    echo "== $name failed: rc=$rc"
    exit $rc
  fi
done
