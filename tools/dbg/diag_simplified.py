"""Debug: simplified-semantics encode, fused vs materialised vs per-tile vs exact oracle, per level."""
import os
import sys
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
from generative_ranking_recommender_amd import synth  # noqa: E402
from generative_ranking_recommender_amd.encode import SIMPLIFIED, HIERARCHICAL_TRAIN, RQEncoder  # noqa: E402
from oracle import rq_oracle as O  # noqa: E402

DEV = torch.device("cuda", 0)
sem_name = sys.argv[1] if len(sys.argv) > 1 else "simplified"
sem = {"simplified": SIMPLIFIED, "train": HIERARCHICAL_TRAIN}[sem_name]
cb = synth.encode_codebooks(seed=99)
xn = synth.mixture_rows(0, 30000)
x = torch.from_numpy(xn).to(DEV)
enc = RQEncoder([torch.from_numpy(cb[k]) for k in ("c0", "c1", "c2")], [128, 128, 256],
                match=torch.from_numpy(cb["match"]), semantics=sem, device=DEV)
res = {}
for v in ["0", "6", "1"]:
    os.environ["RQSID_SCREEN_VARIANT"] = v
    enc.force_materialized = False
    res["fused_v" + v] = enc.encode(x, count_rescored=True).cpu().numpy()
    print("v", v, "rescored", enc.last_rescored, flush=True)
    enc.force_materialized = True
    res["mat_v" + v] = enc.encode(x).cpu().numpy()
kw = dict(normalize=sem.normalize_residual, remap_last=sem.remap_last, last_group_mult=sem.last_group_mult,
          residual_from_weighted=True, exact=True)
ref = O.encode(xn, [cb["c0"], cb["c1"], cb["c2"]], [128, 128, 256], cb["match"], **kw)
for k, a in res.items():
    d = (a != ref)
    print(k, "rows differing per level:", d.sum(0), "first rows:", np.nonzero(d.any(1))[0][:8])
    if d.any():
        i = np.nonzero(d.any(1))[0][0]
        print("   row", i, "got", a[i], "ref", ref[i])
