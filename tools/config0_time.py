"""Time BASELINE configs[0] on the GPU alone (bench.py's config0 field without the CPU leg).

    python tools/config0_time.py [--reps 2]"""
import argparse
import json
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=2)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    for _ in range(a.reps):
        out = bench.config0(dev, cpu_rounds=0)
        print(json.dumps({"gpu": out["gpu"], "parity": out["parity"]}), flush=True)


if __name__ == "__main__":
    main()
