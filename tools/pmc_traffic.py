#!/usr/bin/env python3
"""Per-kernel HBM bytes per launch from the PMC passes of tools/pmc_traffic.sh.

FETCH_SIZE / WRITE_SIZE are in KiB per dispatch (summed over the XCD instances).  gfx950 tallies a
wide (16 B/lane) streaming read at half its bytes (MI355X_MICROARCH.md, HBM section), so FETCH_SIZE
is doubled; WRITE_SIZE is exact for stores of that width.  Launches are numbered per kernel in
dispatch order, so encode level l of step s is launch 3s + l of its kernel when levels differ in
template arguments (they do: RL = 0, 1, 2)."""
import csv
import glob
import json
import re
import sys
from collections import defaultdict


def short(n):
    n = re.sub(r"\(anonymous namespace\)::|rqsid::|void ", "", n)
    return n.split("(")[0]


def main(root, rows):
    vals = defaultdict(lambda: defaultdict(list))
    for f in sorted(glob.glob(f"{root}/p*/run_counter_collection.csv")):
        per = defaultdict(float)
        names = {}
        for r in csv.DictReader(open(f)):
            key = (int(r["Dispatch_Id"]), r["Counter_Name"])
            per[key] += float(r["Counter_Value"])
            names[int(r["Dispatch_Id"])] = short(r["Kernel_Name"])
        for (d, c), v in sorted(per.items()):
            vals[names[d]][c].append(v)
    out = {}
    for k, cs in vals.items():
        fetch = cs.get("FETCH_SIZE", [])
        write = cs.get("WRITE_SIZE", [])
        # the last launch of each kernel is a timed-step launch (warm-up and count passes come first); the
        # re-score runs as two launches per level after the fp32 re-screen (listed rows, then the overflow
        # pass): its level bytes are the last two launches
        last = 2 if "assign_rescore_half_kernel" in k else 1
        out[k] = {"launches": max(len(fetch), len(write)), "launches_per_level": last,
                  "fetch_bytes": 2 * 1024 * sum(fetch[-last:]) if fetch else None,
                  "write_bytes": 1024 * sum(write[-last:]) if write else None}
        if fetch and write:
            out[k]["hbm_bytes"] = out[k]["fetch_bytes"] + out[k]["write_bytes"]
    print(json.dumps({"source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes), FETCH_SIZE x2 (gfx950)",
                      "rows": rows, "kernels": out}, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else None)
