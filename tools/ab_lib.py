"""A/B builds of librqsid.so with extra compile flags (e.g. -DRQ_BID_WAVES=6), same sources as
_lib.build(), into tools/ab/librqsid_<name>.so; load one with RQSID_LIB=tools/ab/librqsid_<name>.so.

    python tools/ab_lib.py w6 -DRQ_BID_WAVES=6
"""
import subprocess
import sys
import tempfile
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO))
from generative_ranking_recommender_amd import _lib  # noqa: E402


def main():
    name, extra = sys.argv[1], sys.argv[2:]
    out = REPO / "tools" / "ab" / f"librqsid_{name}.so"
    out.parent.mkdir(exist_ok=True)
    flags = [f for f in _lib.HIPCC_FLAGS if f != "-shared"] + extra
    with tempfile.TemporaryDirectory() as d:
        objs = [Path(d) / (s.stem + ".o") for s in _lib.SRCS]
        procs = [subprocess.Popen(["/opt/rocm/bin/hipcc", *flags, "-c", "-o", str(o), str(s)])
                 for s, o in zip(_lib.SRCS, objs)]
        if any(p.wait() for p in procs):
            sys.exit("ab_lib: compile failed")
        subprocess.run(["/opt/rocm/bin/hipcc", *_lib.HIPCC_FLAGS, "-o", str(out), *map(str, objs)], check=True)
    print(out)


if __name__ == "__main__":
    main()
