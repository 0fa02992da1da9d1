#!/bin/bash
# GPU box: HBM traffic of the screening kernels of the bench command, from PMC counters as
# MI355X_MICROARCH.md prescribes (separate --pmc passes for FETCH_SIZE and WRITE_SIZE, kernel trace
# only; FETCH_SIZE doubled for gfx950's wide streaming reads).  Output: gpurun_out/$TAG/traffic.json
# (bench.py --traffic-json reads it).
set -u
OUT=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-traffic}
mkdir -p "$OUT"
export TMPDIR=/tmp
ARGS="--steps 2 --warmup 1 --no-cpu --balanced-rows 0 --train-iters 0 --parity-rows 0 --config0 0 ${BENCH_ARGS:-}"
i=0
for c in FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  (cd /tmp && timeout -s KILL 300 rocprofv3 --pmc $c --kernel-include-regex "assign_screen|assign_stream|assign_pp|assign_pc|assign_resident|assign_rows|assign_rescreen|assign_rescore" \
     --output-format csv -d "$OUT/p$i" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" $ARGS > "$OUT/p$i.log" 2>&1)
  rc=$?; echo "pass $c rc=$rc"
  [ $rc -ne 0 ] && { tail -5 "$OUT/p$i.log"; exit $rc; }
done
# rows per launch of the profiled bench (bench.py compares it with its own --rows before using the bytes)
ROWS=$(python3 - "$OUT/p1.log" <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith("{"):
        print(json.loads(l)["config"]["rows_per_gpu"])
PY
)
python3 "$GRAFT_REPO_ROOT/tools/pmc_traffic.py" "$OUT" $ROWS > "$OUT/traffic.json" && cat "$OUT/traffic.json"
