#!/usr/bin/env python3
"""Diagnostics (GPU, stamps build: EXTRA=-DRQSID_STAMPS MODES=0 SUFFIX=_st tools/ab_build.sh, loaded through
RQSID_LIB): BASELINE configs[0]'s GPU fit (bench.config0, 100 balanced iterations at K=128 over 100k rows), then
the list round's per-block cycles by phase (sa_list_round_kernel: pass 1 + first select, pass 2 + second
select, tie rank, bids) and the resolve blocks' cycles (s_memtime ticks, thread 0 of each block)."""
import ctypes
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import bench  # noqa: E402
from generative_ranking_recommender_amd import _lib  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    lib = _lib.load()
    fn = lib.rqsid_debug_al_stamps
    fn.argtypes = [ctypes.c_void_p]
    buf = (ctypes.c_ulonglong * 16)()
    fn(buf)
    out = bench.config0(dev, cpu_rounds=0)
    torch.cuda.synchronize()
    fn(buf)
    v = list(buf)
    print(out["gpu"], flush=True)
    nb = max(v[4], 1)
    names = ["pass1+select1", "pass2+select2", "tie rank", "bids"]
    tot = sum(v[:4]) / nb
    print(f"list-round blocks {v[4]}  with ties ranked {v[5]} ({100 * v[5] / nb:.1f}%)  mean list {v[6] / nb:.0f} "
          f"entries  mean block {tot:.0f} cycles")
    print("  " + "  ".join(f"{nm}={v[i] / nb:.0f} ({100 * v[i] / nb / max(tot, 1):.0f}%)" for i, nm in enumerate(names)))
    print(f"resolve blocks {v[9]}  mean block {v[8] / max(v[9], 1):.0f} cycles")


if __name__ == "__main__":
    main()
