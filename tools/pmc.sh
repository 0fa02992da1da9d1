#!/bin/bash
# PMC passes (one rocprofv3 run per counter group, kernel-trace only: never combined with sys/runtime
# traces) over the screen-sweep workload (PROD encode levels), or with XL=1 over the XL bench (the
# [256,256,512] encode).  Usage: TAG=x [XL=1] tools/pmc.sh
set -u
OUT=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-pmc}
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
i=0
for grp in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
           "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM" \
           "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_LDS_BANK_CONFLICT" \
           "FETCH_SIZE" "TCC_HIT_sum TCC_MISS_sum" "SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_LDS_IDX_ACTIVE"; do
  i=$((i+1))
  if [ "${XL:-0}" = "1" ]; then
    timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d "$OUT/p$i" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" \
      --preset xl --steps 2 --warmup 1 --no-cpu --balanced-rows 0 --train-iters 0 --parity-rows 0 --config0 0 > "$OUT/p$i.log" 2>&1
  else
    timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d "$OUT/p$i" -o run -- python3 "$GRAFT_REPO_ROOT/tools/screen_sweep.py" > "$OUT/p$i.log" 2>&1
  fi
  rc=$?
  echo "pass $i ($grp) rc=$rc"
  if [ $rc -ne 0 ]; then tail -20 "$OUT/p$i.log"; exit $rc; fi
done
python3 "$GRAFT_REPO_ROOT/tools/pmc_summary.py" "$OUT" > "$OUT/summary.csv" && cat "$OUT/summary.csv"
rm -rf "$OUT"/p*/  # the raw per-dispatch csvs exceed gpurun's merge-back cap
