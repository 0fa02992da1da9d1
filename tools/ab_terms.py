#!/usr/bin/env python3
"""A/B (GPU): the bench with every rqsid_assign call forced to a screen-term count
(RQSID_AB_TERMS = 1 or 3; 0 = the library's automatic choice).  Prints bench.py's JSON line."""
import os
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from generative_ranking_recommender_amd import ops  # noqa: E402
import bench  # noqa: E402

TERMS = int(os.environ.get("RQSID_AB_TERMS", "0"))
_orig = ops.assign


def _forced(*a, **k):
    k["screen_terms"] = TERMS
    return _orig(*a, **k)


ops.assign = _forced
if __name__ == "__main__":
    sys.argv = ["bench.py", "--no-cpu", *sys.argv[1:]]
    bench.main()
