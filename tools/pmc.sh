#!/bin/bash
# PMC passes (one rocprofv3 run per counter group, kernel-trace only: never combined with sys/runtime
# traces) over the screen-sweep workload.  Usage: TAG=x tools/pmc.sh
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
  timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d "$OUT/p$i" -o run -- python3 "$GRAFT_REPO_ROOT/tools/screen_sweep.py" > "$OUT/p$i.log" 2>&1
  rc=$?
  echo "pass $i ($grp) rc=$rc"
  if [ $rc -ne 0 ]; then tail -20 "$OUT/p$i.log"; exit $rc; fi
done
python3 "$GRAFT_REPO_ROOT/tools/pmc_summary.py" "$OUT" > "$OUT/summary.csv" && cat "$OUT/summary.csv"
rm -rf "$OUT"/p*/  # the raw per-dispatch csvs exceed gpurun's merge-back cap
