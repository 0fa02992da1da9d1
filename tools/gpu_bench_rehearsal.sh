#!/bin/bash
# GPU box: (1) the side-measurement watchdog (a 1-s budget prints the encode line without the side fields);
# (2) the N=2 path of bench.py through torchrun on one GPU (gloo, ranks share the device).
set -u
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-rehearsal}
mkdir -p "$OUT"
timeout -k 10 300 python bench.py --no-cpu --config0 0 --side-budget 1 --rows 2000000 > "$OUT/watchdog.json" 2> "$OUT/watchdog.err" || { tail -5 "$OUT/watchdog.err"; exit 1; }
tail -c 300 "$OUT/watchdog.json"; echo
RQSID_BENCH_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --rows 2000000 --steps 3 --warmup 1 --balanced-rows 200000 > "$OUT/n2.json" 2> "$OUT/n2.err" || { tail -20 "$OUT/n2.err"; exit 1; }
tail -c 600 "$OUT/n2.json"
