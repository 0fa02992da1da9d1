#!/bin/bash
# GPU box, round 4: XL training (configs[4] per-rank share: 6.25M rows, [256,2560,2560] / need [256,256,512])
# through the row-sharded trainer at world size 1 over RCCL, after the list-only auction blocks.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 1120 python -u tools/train_bench.py --preset xl --sharded --rows 6250000 --data bench \
  --out gpurun_out/r4_train_xl_6250k_listonly.json > gpurun_out/r4_train_xl_listonly.log 2>&1
rc=$?
tail -3 gpurun_out/r4_train_xl_listonly.log
exit $rc
