#!/bin/bash
# GPU box: the bench's encode step under several kernel-selection environments (A/B), one line each.
# Usage: AB="NAME1:VAR=1,VAR2=3 NAME2:..." [BENCH_ARGS=...] bash tools/gpu_ab_env.sh
set -u
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-ab}
mkdir -p "$OUT"
ARGS="--steps ${STEPS:-10} --warmup 2 --no-cpu --balanced-rows 0 --train-iters 0 --parity-rows ${PARITY:-0} --config0 0 ${BENCH_ARGS:-}"
for spec in $AB; do
  name=${spec%%:*}; envs=${spec#*:}
  env_args=""; [ "$envs" != "-" ] && env_args=$(echo "$envs" | tr ',' ' ')
  timeout -k 10 300 env $env_args python bench.py $ARGS > "$OUT/$name.json" 2> "$OUT/$name.err" || { echo "$name failed"; tail -5 "$OUT/$name.err"; exit 1; }
  python - "$OUT/$name.json" "$name" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], "%.3e" % d["value"], d["ms_per_step"], {k: v.get("ms") for k, v in d["kernels"].items()}, d.get("parity"))
PY
done
