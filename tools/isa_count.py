"""Static instruction mix per kernel of a gfx950 .s file (hipcc --save-temps):

    python tools/isa_count.py /tmp/isa/auction_seg-hip-amdgcn-amd-amdhsa-gfx950.s [name-regex]

Counts SALU (s_*, excluding memory/branch/waitcnt), VALU (v_*), scalar and vector memory, LDS, branches
and waitcnts, plus VGPR/SGPR counts from the kernel descriptors.  A first look at the instruction stream
of a sweep kernel; PMC SQ_INSTS_* give the dynamic counts.
"""
import re
import sys
from collections import Counter


def classify(op):
    if op.startswith("s_waitcnt"):
        return "waitcnt"
    if op.startswith(("s_cbranch", "s_branch", "s_setpc", "s_endpgm")):
        return "branch"
    if op.startswith(("s_load", "s_buffer_load")):
        return "smem"
    if op.startswith("s_barrier"):
        return "barrier"
    if op.startswith("s_"):
        return "salu"
    if op.startswith(("global_", "buffer_", "flat_")):
        return "vmem"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith("v_"):
        return "valu"
    return "other"


def main():
    path = sys.argv[1]
    pat = re.compile(sys.argv[2]) if len(sys.argv) > 2 else None
    kernels = {}
    cur = None
    for line in open(path):
        m = re.match(r"^(_Z\S+):\s*(;.*)?$", line)
        if m:
            cur = m.group(1)
            kernels[cur] = Counter()
            continue
        if cur is None:
            continue
        if line.startswith(".Lfunc_end"):
            cur = None
            continue
        s = line.strip()
        if not s or s.startswith((";", ".")) or s.endswith(":"):
            continue
        op = s.split()[0]
        kernels[cur][classify(op)] += 1
        kernels[cur]["op:" + op] += 1
    for k, c in kernels.items():
        if pat and not pat.search(k):
            continue
        top = sorted(((v, o[3:]) for o, v in c.items() if o.startswith("op:")), reverse=True)[:8]
        print(f"{k[:70]:70s} salu {c['salu']:5d} valu {c['valu']:5d} vmem {c['vmem']:4d} lds {c['lds']:4d} "
              f"smem {c['smem']:3d} br {c['branch']:4d} wait {c['waitcnt']:4d}")
        print("    top:", ", ".join(f"{o} {v}" for v, o in top))


if __name__ == "__main__":
    main()
