#!/bin/bash
# A/B timing builds of librqsid.so (RQSID_AB_MODE 1..3 strip the screen's epilogue / MFMA / compute;
# results are WRONG, timing only).  Use: RQSID_LIB=tools/ab/librqsid_ab<N>.so python tools/screen_sweep.py
set -eu
cd "$(dirname "$0")/.."
C=generative_ranking_recommender_amd/csrc
for m in ${MODES:-1 2 3}; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fno-slp-vectorize -shared -fPIC -DRQSID_AB_MODE=$m ${EXTRA:-} \
    -o tools/ab/librqsid_ab$m${SUFFIX:-}.so $C/rqsid.hip $C/assign.hip $C/assign_stream.hip $C/assign_resident.hip $C/assign_rows.hip $C/assign_pc.hip $C/auction.hip $C/auction_seg.hip &
done
for j in $(jobs -p); do wait $j || { echo "ab_build failed"; exit 1; }; done
