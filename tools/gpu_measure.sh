#!/bin/bash
# GPU box: XL-preset PMC traffic + the XL bench line with it, then the per-phase training cost at 10M rows
# (tools/train_scale.py).  Output in gpurun_out/$TAG.  Any failure ends the script.
set -u
OUT=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-measure}
mkdir -p "$OUT"
export TMPDIR=/tmp
if [ "${SKIP_XL:-0}" != 1 ]; then
  TAG=${TAG:-measure}/xl_traffic BENCH_ARGS="--preset xl" bash tools/pmc_traffic.sh > "$OUT/xl_traffic.log" 2>&1 || { tail -20 "$OUT/xl_traffic.log"; exit 1; }
  timeout -k 10 400 python bench.py --preset xl --no-cpu --config0 0 --traffic-json "$OUT/xl_traffic/traffic.json" > "$OUT/xl_bench.json" 2> "$OUT/xl_bench.err" || { tail -20 "$OUT/xl_bench.err"; exit 1; }
  tail -c 700 "$OUT/xl_bench.json"
  rm -rf "$OUT/xl_traffic/p1" "$OUT/xl_traffic/p2"
fi
if [ "${SKIP_SCALE:-0}" != 1 ]; then
  timeout -k 10 600 python tools/train_scale.py --rows ${SCALE_ROWS:-10000000} --out "$OUT/train_scale.json" > "$OUT/train_scale.log" 2>&1 || { tail -20 "$OUT/train_scale.log"; exit 1; }
  cat "$OUT/train_scale.json"
fi
if [ "${TRAIN_ROWS:-0}" != 0 ]; then
  timeout -k 10 900 python -u tools/train_bench.py --rows $TRAIN_ROWS --out "$OUT/train_bench.json" > "$OUT/train_bench.log" 2>&1 || { tail -20 "$OUT/train_bench.log"; exit 1; }
  cat "$OUT/train_bench.json"
fi
