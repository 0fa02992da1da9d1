set -u
TAG=segprof_g K=256 S=1666 bash tools/gpu_ab_prof.sh && TAG=segprof_m K=128 S=128 bash tools/gpu_ab_prof.sh
