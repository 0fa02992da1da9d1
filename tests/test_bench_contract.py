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


def test_side_watchdog_prints_the_encode_line_and_exits_nonzero(capsys):
    """a hang in the side measurements after the timed region ends with the encode line
    printed (marked stopped) and a NON-ZERO exit status, so the driver sees the failure."""
    import sys
    import time
    sys.path.insert(0, str(REPO))
    import bench
    codes = []
    line = {"metric": "vectors quantized/sec (3-level RQ, 512-d)", "value": 1.0}
    dog = bench.SideWatchdog(line, 0.05, rank=0, exit_fn=codes.append).start()
    dog.thread.join(5)
    assert codes == [bench.SideWatchdog.EXIT_CODE] and codes[0] != 0
    out = capsys.readouterr().out.strip().splitlines()
    assert len(out) == 1
    got = json.loads(out[0])
    assert got["value"] == 1.0 and got["side_measurements"].startswith("stopped")
    assert dog.done() is False  # the main thread's late print is suppressed: one line only
    assert capsys.readouterr().out == ""


def test_side_watchdog_quiet_when_done_in_time(capsys):
    import sys
    sys.path.insert(0, str(REPO))
    import bench
    codes = []
    dog = bench.SideWatchdog({"value": 2.0}, 30.0, rank=0, exit_fn=codes.append).start()
    assert dog.done() is True
    dog.thread.join(5)
    assert codes == [] and json.loads(capsys.readouterr().out)["value"] == 2.0
