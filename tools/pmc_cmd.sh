#!/bin/bash
# PMC passes (one rocprofv3 run per counter group, kernel trace only) over an arbitrary python command:
#   TAG=x CMD="tools/auction_bench.py --jobs 1000000 --workers 128 --reps 1" KREGEX="sa_bid|sa_hist" tools/pmc_cmd.sh
# then python tools/pmc_summary.py gpurun_out/x > summary.csv
set -u
OUT=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-pmc}
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
i=0
for grp in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
           "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM" \
           "SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAVES" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $grp --kernel-include-regex "${KREGEX:-.}" --output-format csv -d "$OUT/p$i" -o run \
    -- python3 $GRAFT_REPO_ROOT/$CMD > "$OUT/p$i.log" 2>&1
  rc=$?
  echo "pass $i ($grp) rc=$rc"
  if [ $rc -ne 0 ]; then tail -20 "$OUT/p$i.log"; exit $rc; fi
done
python3 $GRAFT_REPO_ROOT/tools/pmc_summary.py "$OUT" > "$OUT/summary.csv" && cat "$OUT/summary.csv"
rm -rf "$OUT"/p*/
