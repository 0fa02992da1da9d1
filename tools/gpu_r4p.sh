#!/bin/bash
# GPU box, round 4: PMC summaries (mfma_busy, wait_any, SALU / VALU, FETCH_SIZE x2, ...) of the default
# encode kernels: PROD levels (screen sweep) and the XL encode (its level 2 on the row-resident screen).
set -u
cd "$GRAFT_REPO_ROOT"
TAG=r4_pmc_prod timeout -k 10 560 bash tools/pmc.sh > gpurun_out/r4_pmc_prod.log 2>&1 || { tail -20 gpurun_out/r4_pmc_prod.log; exit 1; }
TAG=r4_pmc_xl XL=1 timeout -k 10 600 bash tools/pmc.sh > gpurun_out/r4_pmc_xl.log 2>&1 || { tail -20 gpurun_out/r4_pmc_xl.log; exit 1; }
grep -E "assign_|kernel," gpurun_out/r4_pmc_prod/summary.csv gpurun_out/r4_pmc_xl/summary.csv | cut -c1-200
