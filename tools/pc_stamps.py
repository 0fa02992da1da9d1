#!/usr/bin/env python3
"""Diagnostics (GPU, stamps build: EXTRA=-DRQSID_STAMPS MODES=0 SUFFIX=_st tools/ab_build.sh, loaded through
RQSID_LIB): per encode level, the producer/consumer screen's (assign_pc.hip) cycles per wave and role --
consumer {barrier, compute, epilogue}, row producer {DMA issue, vmcnt wait, build, finish, barrier},
loader {DMA issue, vmcnt wait, barrier} -- as shares of the role's total and as cycles per chunk phase.
The wide form (assign_pcw_kernel, 256-row tiles, RQSID_PCW unset or 1): consumer {barrier, compute,
epilogue}, feeder {DMA issue, build, vmcnt wait, barrier}; PCW=1 in the environment selects that table."""
import ctypes
import os
import sys
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import bench  # noqa: E402
from generative_ranking_recommender_amd import _lib, ops, synth  # noqa: E402
import generative_ranking_recommender_amd.encode as encmod  # noqa: E402
from generative_ranking_recommender_amd.encode import HIERARCHICAL_TRAIN, RQEncoder  # noqa: E402


def main(n=int(os.environ.get("SWEEP_ROWS", 10_000_000))):
    dev = torch.device("cuda", 0)
    cache = os.environ.get("SWEEP_CB")
    if cache and os.path.exists(cache):
        z = np.load(cache)
        cb = {k: z[k] for k in z.files}
    else:
        cb = synth.encode_codebooks(seed=99)
    enc = RQEncoder([torch.from_numpy(cb[k]) for k in ("c0", "c1", "c2")], [128, 128, 256],
                    match=torch.from_numpy(cb["match"]), semantics=HIERARCHICAL_TRAIN, device=dev)
    x = bench.make_rows(n, 0, dev)
    lib = _lib.load()
    fn = lib.rqsid_debug_pc_stamps
    fn.argtypes = [ctypes.c_void_p]
    buf = (ctypes.c_ulonglong * 24)()
    enc.encode(x)
    torch.cuda.synchronize()
    fn(buf)
    orig = ops.assign
    res = []

    def hook(*a, **k):
        out = orig(*a, **k)
        torch.cuda.synchronize()
        fn(buf)
        res.append((a[2], list(buf)))
        return out

    encmod.ops.assign = hook
    enc.encode(x)
    encmod.ops.assign = orig
    wide = os.environ.get("PCW", "0") == "1"
    rows_t, ph_t, ncons = (256, 32, 8) if wide else (128, 16, 4)
    names = {0: ("consumer", {1: "barrier", 5: "compute", 3: "epilogue", 2: "  epi:mfma-drain", 6: "  epi:bound+U",
                              7: "  epi:pass-bits", 23: "  epi:decide+stores"}),
             8: ("producer", {6: "issue", 2: "vmcnt", 5: "build", 3: "finish", 1: "barrier"}),
             16: ("loader", {6: "issue", 2: "vmcnt", 1: "barrier"})}
    if wide:
        names = {0: ("consumer", {1: "barrier", 5: "compute", 3: "epilogue"}),
                 8: ("feeder", {6: "issue", 5: "build", 2: "vmcnt", 1: "barrier"})}
    for lvl, (b, v) in enumerate(res):
        waves = v[4]
        if not waves:
            print(f"L{lvl}: producer/consumer screen not used")
            continue
        rows = int(b.seg_row_off[-1].item())
        tiles = int(((b.seg_row_off[1:] - b.seg_row_off[:-1] + rows_t - 1) // rows_t).sum().item())
        phases = ph_t * tiles / (waves / ncons)  # phases per block
        line = [f"L{lvl}: rows={rows} tiles={tiles} blocks={waves // ncons} phases/block={phases:.0f}"]
        for base, (role, parts) in names.items():
            w = v[base + 4]
            tot = v[base] / w
            seg = " ".join(f"{nm}={100 * v[base + o] / w / tot:.1f}%" for o, nm in parts.items())
            line.append(f"  {role}: {tot / phases:.0f} cycles/phase  {seg}")
        print("\n".join(line), flush=True)


if __name__ == "__main__":
    main()
