#!/usr/bin/env python3
"""Merge rocprofv3 --pmc CSV passes (tools/pmc.sh) into one per-kernel table: counters summed per
dispatch, averaged over the dispatches of each kernel; FETCH_SIZE doubled per MI355X_MICROARCH.md
(gfx950 reports half the bytes of wide streaming reads) and reported in bytes per dispatch."""
import csv
import glob
import re
import sys
from collections import defaultdict


def short(n):
    n = re.sub(r"\(anonymous namespace\)::|rqsid::|void |at::native::", "", n)
    n = n.split("(")[0] if not n.startswith("(") else n
    return n.replace(", ", ".").replace(",", ".")[:48]


def main(root):
    per = defaultdict(lambda: defaultdict(list))  # kernel -> counter -> [per-dispatch values]
    durs = defaultdict(dict)
    for f in sorted(glob.glob(f"{root}/p*/run_counter_collection.csv")):
        acc = defaultdict(float)
        meta = {}
        for r in csv.DictReader(open(f)):
            key = (r["Dispatch_Id"], r["Counter_Name"])
            acc[key] += float(r["Counter_Value"])
            meta[r["Dispatch_Id"]] = (short(r["Kernel_Name"]), int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
        for (d, c), v in acc.items():
            k, dur = meta[d]
            per[k][c].append(v)
            durs[k][(f, d)] = dur
    cols = ["dur_us", "SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES", "GRBM_GUI_ACTIVE", "wait_any%", "wait_inst%", "active%",
            "SQ_INSTS_VALU", "SQ_INSTS_MFMA", "SQ_INSTS_LDS", "SQ_INSTS_VMEM", "mfma_busy%", "lds_conflict%",
            "FETCH_bytes", "WRITE_bytes", "TCC_hit%", "clock_GHz", "SQ_INSTS_SALU", "SQ_WAVES"]
    print("kernel," + ",".join(cols))
    for k, cs in sorted(per.items()):
        avg = {c: sum(v) / len(v) for c, v in cs.items()}
        dur = sum(durs[k].values()) / max(len(durs[k]), 1) / 1e3
        wc = avg.get("SQ_WAVE_CYCLES", 0) or 1
        row = {"dur_us": dur, "SQ_WAVE_CYCLES": avg.get("SQ_WAVE_CYCLES"), "SQ_BUSY_CYCLES": avg.get("SQ_BUSY_CYCLES"),
               "GRBM_GUI_ACTIVE": avg.get("GRBM_GUI_ACTIVE"),
               "wait_any%": 100 * avg.get("SQ_WAIT_ANY", 0) / wc, "wait_inst%": 100 * avg.get("SQ_WAIT_INST_ANY", 0) / wc,
               "active%": 100 * avg.get("SQ_ACTIVE_INST_ANY", 0) / wc,
               "SQ_INSTS_VALU": avg.get("SQ_INSTS_VALU"), "SQ_INSTS_MFMA": avg.get("SQ_INSTS_MFMA"),
               "SQ_INSTS_LDS": avg.get("SQ_INSTS_LDS"), "SQ_INSTS_VMEM": avg.get("SQ_INSTS_VMEM"),
               "mfma_busy%": 100 * avg.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / max(avg.get("GRBM_GUI_ACTIVE", 1) / 8 * 1024, 1),
               "lds_conflict%": 100 * avg.get("SQ_LDS_BANK_CONFLICT", 0) / max(avg.get("SQ_LDS_IDX_ACTIVE", 1), 1),
               "FETCH_bytes": 2 * 1024 * avg.get("FETCH_SIZE", 0), "WRITE_bytes": 1024 * avg.get("WRITE_SIZE", 0),
               "SQ_INSTS_SALU": avg.get("SQ_INSTS_SALU"), "SQ_WAVES": avg.get("SQ_WAVES"),
               "TCC_hit%": 100 * avg.get("TCC_HIT_sum", 0) / max(avg.get("TCC_HIT_sum", 0) + avg.get("TCC_MISS_sum", 0), 1),
               "clock_GHz": avg.get("GRBM_GUI_ACTIVE", 0) / 8 / (dur * 1e3) if dur else 0}
        print(k + "," + ",".join("" if row[c] is None else f"{row[c]:.4g}" for c in cols))


if __name__ == "__main__":
    main(sys.argv[1])
