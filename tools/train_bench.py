"""Time HierarchicalRQKMeans.train at the PROD shape (layer_clusters [128,1280,1280], need [128,128,256]) or
the XL shape (configs[4]: [256,2560,2560], need [256,256,512]) on synthetic rows, per layer, with the
lockstep sub-fits (default) or the reference's sequential order; --sharded runs the row-sharded trainer
(one process per GPU) at world size 1 over RCCL, i.e. the code path of one rank of the 8-GPU job.

    python tools/train_bench.py --rows 200000 [--sequential] [--preset xl] [--sharded] [--out f.json]

Prints one JSON line: rows, per-layer seconds, total seconds, sub-fit mode."""
import argparse
import json
import logging
import sys
import threading
import time
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from generative_ranking_recommender_amd import synth  # noqa: E402
from generative_ranking_recommender_amd.hierarchical_rq_kmeans import (HierarchicalRQKMeans,  # noqa: E402
                                                                       HierarchicalRQKMeansConfig)


class LayerTimes(logging.Handler):
    def __init__(self):
        super().__init__()
        self.t0 = time.time()
        self.marks = []

    def emit(self, record):
        msg = record.getMessage()
        if msg.startswith("[LAYER"):
            self.marks.append((msg, time.time() - self.t0))
            print(msg, flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=200000)
    ap.add_argument("--sequential", action="store_true")
    ap.add_argument("--iter-limit", type=int, default=100)
    ap.add_argument("--preset", choices=("prod", "xl"), default="prod")
    ap.add_argument("--sharded", action="store_true",
                    help="row-sharded trainer through a world-size-1 RCCL process group")
    ap.add_argument("--sharded-auction", action="store_true",
                    help="with --sharded: the balanced fits run the row-sharded auction protocol (rqsid_dauction_*, "
                         "per-round collectives, row-sharded bid lists) even at world 1 (RQSID_SHARDED_AUCTION=1), "
                         "i.e. what every rank of a larger world runs")
    ap.add_argument("--out", default="")
    ap.add_argument("--data", choices=("small", "bench"), default="small",
                    help="small: synth.small_mixture (host); bench: bench.make_rows (the encode bench's rows, "
                         "generated on the device, for 10M-row runs)")
    a = ap.parse_args()
    t_start = time.time()

    def heartbeat():  # long phases log nothing for minutes; say the run is alive once a minute
        while True:
            time.sleep(60)
            print(f"[heartbeat] {time.time() - t_start:.0f} s", flush=True)

    threading.Thread(target=heartbeat, daemon=True).start()
    if a.data == "bench":
        import bench  # noqa: E402  (tools/ run from the repo root)
        x = bench.make_rows(a.rows, 0, torch.device("cuda", 0)).cpu().numpy()
    else:
        x = synth.small_mixture(a.rows, m=4096, seed=5)
    lc, need = ([256, 2560, 2560], [256, 256, 512]) if a.preset == "xl" else ([128, 1280, 1280], [128, 128, 256])
    cfg = HierarchicalRQKMeansConfig(layer_clusters=lc, need_clusters=need, embedding_dim=512,
                                     iter_limit=a.iter_limit)
    group = None
    if a.sharded_auction:
        import os
        os.environ["RQSID_SHARDED_AUCTION"] = "1"
    if a.sharded:
        import os
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29531")
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
        group = dist.group.WORLD
    h = LayerTimes()
    lg = logging.getLogger("generative_ranking_recommender_amd.hierarchical_rq_kmeans")
    lg.setLevel(logging.INFO)
    lg.addHandler(h)
    np.random.seed(42)
    torch.manual_seed(42)
    model = HierarchicalRQKMeans(cfg, device=torch.device("cuda", 0), group=group)
    model.batched_sub_fits = not a.sequential
    t = time.time()
    res = model.train(x)
    torch.cuda.synchronize()
    total = time.time() - t
    ids = np.stack([r.cpu().numpy() for r in res["cluster_ids"]], 1)
    consistent = bool((model.predict(x, reference_quirks=False) == ids).all())
    line = {"rows": a.rows, "data": a.data, "preset": a.preset, "layer_clusters": lc, "need_clusters": need,
            "path": ("sharded (world 1, RCCL)" + (", row-sharded auction protocol" if a.sharded_auction else ""))
                    if a.sharded else "single process",
            "dauction_lists": __import__("os").environ.get("RQSID_DAUCTION_LIST", "1"),
            "mode": "sequential" if a.sequential else "lockstep",
            "total_s": round(total, 2),
            "layers": [m for m in h.marks], "unique_ids": int(len(np.unique(ids, axis=0))),
            "train_encode_consistent": consistent}
    print(json.dumps(line), flush=True)
    if a.out:
        Path(a.out).write_text(json.dumps(line) + "\n")


if __name__ == "__main__":
    main()
