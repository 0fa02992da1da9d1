#!/bin/bash
# GPU box: two PMC passes (kernel-trace only) over the cached-codebook sweep, for the default library
# and optionally $LIB2; summaries in gpurun_out/$TAG/{a,b}.txt
set -u
OUT=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-pmc2}
mkdir -p "$OUT"
export TMPDIR=/tmp SWEEP_CB=/tmp/sweep_cb.npz SWEEP_REPS=2
timeout -k 10 300 python tools/screen_sweep.py > "$OUT/warm.log" 2>&1 || { tail -5 "$OUT/warm.log"; exit 1; }
run() {  # $1 = name, $2 = lib or empty
  i=0
  for grp in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_MFMA" \
             "SQ_INSTS_VMEM SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"; do
    i=$((i+1))
    (cd /tmp && RQSID_LIB=${2:-$GRAFT_REPO_ROOT/generative_ranking_recommender_amd/librqsid.so} timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d "$OUT/$1/p$i" -o run -- python3 "$GRAFT_REPO_ROOT/tools/screen_sweep.py" > "$OUT/$1_p$i.log" 2>&1)
    rc=$?; echo "$1 pass $i rc=$rc"
    [ $rc -ne 0 ] && { tail -5 "$OUT/$1_p$i.log"; exit $rc; }
  done
  python tools/pmc_summary.py "$OUT/$1" > "$OUT/$1.txt"
}
run a "" || exit 1
[ -n "${LIB2:-}" ] && { run b "$GRAFT_REPO_ROOT/$LIB2" || exit 1; }
grep -i "stream\|screen\|rescore\|kernel,\|compact" "$OUT/a.txt" | head -12
[ -f "$OUT/b.txt" ] && grep -i "stream\|screen\|rescore\|kernel,\|compact" "$OUT/b.txt" | head -12
exit 0
