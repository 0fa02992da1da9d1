#!/usr/bin/env python3
"""Summarise a rocprofv3 kernel-trace database (``-d DIR -o run`` → run_results.db) into the
per-kernel stats table committed under profiles/ (calls, average/total duration, VGPR/SGPR, LDS).

usage: python tools/prof_summary.py gpurun_out/<tag>/prof/run_results.db > profiles/<name>.txt
"""
import re
import sqlite3
import sys


def short(name: str) -> str:
    name = re.sub(r"\(anonymous namespace\)::", "", name)
    if name.startswith("void at::native::"):
        return "torch:" + name[len("void at::native::"):].split("<")[0].split("(")[0]
    return name.replace("void ", "").split("(")[0] if "AssignParams" in name else name.split("(")[0]


def main(path):
    c = sqlite3.connect(path)
    rows = c.execute("select name, count(*), avg(duration), sum(duration), min(duration), max(duration), "
                     "max(vgpr_count), max(accum_vgpr_count), max(sgpr_count), max(lds_size), max(grid_x) "
                     "from kernels group by name order by sum(duration) desc").fetchall()
    tot = sum(r[3] for r in rows)
    print(f"# rocprofv3 --kernel-trace summary of {path}")
    print(f"# {'kernel':<58} {'calls':>5} {'avg_us':>10} {'min_us':>10} {'max_us':>10} {'total_ms':>9} {'pct':>6} "
          f"{'vgpr':>4} {'agpr':>4} {'sgpr':>4} {'lds':>6} {'grid':>9}")
    for n, cnt, avg, s, mn, mx, vg, ag, sg, lds, gx in rows:
        print(f"{short(n)[:60]:<60} {cnt:>5} {avg/1e3:>10.1f} {mn/1e3:>10.1f} {mx/1e3:>10.1f} {s/1e6:>9.3f} "
              f"{100*s/tot:>5.1f}% {vg:>4} {ag:>4} {sg:>4} {lds:>6} {gx:>9}")


if __name__ == "__main__":
    main(sys.argv[1])
