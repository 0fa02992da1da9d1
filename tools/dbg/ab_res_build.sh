#!/bin/bash
# Timing-only A/B builds of librqsid.so with stamps: tools/ab/librqsid_<name>.so for each NAME=FLAGS pair in $ABS
set -eu
cd "$(dirname "$0")/../.."
C=generative_ranking_recommender_amd/csrc
for pair in $ABS; do
  name=${pair%%=*}; flags=${pair#*=}
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fno-slp-vectorize -shared -fPIC ${STAMPS--DRQSID_STAMPS} ${flags//,/ } \
    -o tools/ab/librqsid_$name.so $C/rqsid.hip $C/assign.hip $C/assign_stream.hip $C/assign_resident.hip $C/auction.hip &
done
for j in $(jobs -p); do wait $j || { echo "build failed"; exit 1; }; done
