#!/bin/bash
# GPU box: candidate-split screen checks (new parity tests + the XL encode, split vs multi-pass).
set -u
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-cw}
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -rA --timeout 120 --timeout-method thread \
  -k "${TESTK:-candidate_split}" > "$OUT/tests.log" 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|Error" "$OUT/tests.log" | tail -5
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --preset xl --no-cpu --config0 0 --steps 5 --warmup 2 > "$OUT/xl_split.json" 2> "$OUT/xl_split.err" || { tail -20 "$OUT/xl_split.err"; exit 1; }
RQSID_SCREEN_VARIANT=7 timeout -k 10 300 python bench.py --preset xl --no-cpu --config0 0 --steps 5 --warmup 2 > "$OUT/xl_multi.json" 2> "$OUT/xl_multi.err" || { tail -20 "$OUT/xl_multi.err"; exit 1; }
python - "$OUT" <<'PY'
import json, sys
for n in ("xl_split", "xl_multi"):
    d = json.loads(open(f"{sys.argv[1]}/{n}.json").read().strip().splitlines()[-1])
    print(n, d["value"], d["ms_per_step"], {k: v.get("ms") for k, v in d["kernels"].items()})
PY
