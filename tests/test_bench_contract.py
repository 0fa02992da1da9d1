"""bench.py's roofline traffic lookup: every kernel name LEVEL_KERNELS lists for a preset must be a
kernel of the committed PMC traffic file that preset reads, or the bench line silently loses its
traffic (the names carry template arguments that change with the kernels)."""
import ast
import json
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent


def _level_kernels():
    tree = ast.parse((REPO / "bench.py").read_text())
    for node in tree.body:
        if isinstance(node, ast.Assign) and any(getattr(t, "id", None) == "LEVEL_KERNELS" for t in node.targets):
            return ast.literal_eval(node.value)
    raise AssertionError("LEVEL_KERNELS not found in bench.py")


def test_level_kernels_match_committed_traffic():
    lk = _level_kernels()
    for preset, path in (("prod", "bench_data/traffic.json"), ("xl", "bench_data/traffic_xl.json")):
        names = set(json.loads((REPO / path).read_text())["kernels"])
        for lvl, ks in lk[preset].items():
            missing = [k for k in ks if k not in names]
            assert not missing, f"{preset} level {lvl}: {missing} not in {path}"
