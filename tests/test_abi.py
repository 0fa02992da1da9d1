"""The C-ABI library builds for gfx950, loads, and exports every symbol include/rqsid.h declares."""
import re
import subprocess
from pathlib import Path

import pytest

from generative_ranking_recommender_amd import _lib

REPO = Path(__file__).resolve().parent.parent


def declared_symbols():
    text = (REPO / "include" / "rqsid.h").read_text()
    return sorted(set(re.findall(r"^\s*(?:const\s+)?[a-z0-9_]+\*?\s+\*?(rqsid_[a-z0-9_]+)\s*\(", text, re.M)))


def test_header_and_binding_agree():
    assert set(declared_symbols()) == set(_lib.SIGNATURES), "ctypes table out of sync with include/rqsid.h"


def test_library_exports_every_declared_symbol():
    _lib.build()
    lib = _lib.load()
    for name in declared_symbols():
        assert hasattr(lib, name), name
    out = subprocess.run(["nm", "-D", "--defined-only", str(_lib.LIB_PATH)], capture_output=True, text=True).stdout
    exported = set(re.findall(r"\bT (rqsid_\w+)", out))
    assert set(declared_symbols()) <= exported


def test_library_is_gfx950_code_object():
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-readelf", "-n", str(_lib.LIB_PATH)], capture_output=True,
                         text=True)
    blob = _lib.LIB_PATH.read_bytes()
    assert b"gfx950" in blob


def test_host_only_queries_need_no_gpu():
    lib = _lib.load()
    assert lib.rqsid_version() >= 1
    assert lib.rqsid_assign_tile_rows() == 128
    assert lib.rqsid_assign_workspace_bytes(1000) >= 1000 * 32
    assert lib.rqsid_bucket_workspace_bytes(10, 16384) >= 16384 * 8


def test_argument_errors_map_to_value_error():
    lib = _lib.load()
    rc = lib.rqsid_prepare_centers(None, 4, 48, None, None, None)  # dim not a multiple of 32
    assert rc == -1
    assert "prepare_centers" in lib.rqsid_last_error().decode()
    with pytest.raises(ValueError):
        _lib.check(rc, "rqsid_prepare_centers")


def test_product_build_has_no_probe_flags():
    """a timing-probe build (RQSID_AB_*, RQSID_STAMPS) returns wrong IDs by design; the in-tree
    library must report none, and the loader refuses one unless RQSID_LIB names it explicitly."""
    assert _lib.load().rqsid_build_flags() == 0


def test_pc_kernel_keeps_nothing_in_m0():
    """assign_pc.hip drops the M0 save/restore around its LDS-DMA asm (RQ_M0_KEEP 0): valid only while hipcc
    itself neither reads nor writes M0 anywhere in assign_pc_kernel outside those asm blocks."""
    import shutil
    import tempfile
    hipcc = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    if not Path(hipcc).exists():
        pytest.skip("hipcc not available")
    src = REPO / "generative_ranking_recommender_amd" / "csrc" / "assign_pc.hip"
    with tempfile.TemporaryDirectory() as d:
        asm = Path(d) / "pc.s"
        subprocess.run([hipcc, "--offload-arch=gfx950", "-O3", "-std=c++17", "-fno-slp-vectorize", "--cuda-device-only",
                        "-S", "-o", str(asm), str(src)], check=True, capture_output=True)
        text = asm.read_text()
    kernels = re.findall(r"^(_Z\w*assign_pc_kernel\w*):", text, re.M)
    assert kernels
    for k in kernels:
        body = text[text.index(k + ":"):text.index(".Lfunc_end", text.index(k + ":"))]
        inside, bad = False, []
        for line in body.splitlines():
            if "ASMSTART" in line:
                inside = True
            elif "ASMEND" in line:
                inside = False
            elif not inside and re.search(r"\bm0\b", line.split(";")[0]):
                bad.append(line.strip())
        assert not bad, (k, bad[:5])
