"""Loader for the in-tree HIP library ``librqsid.so`` (C ABI: ``include/rqsid.h``).

The product path has no CPU fallback: if the library is missing or no GPU is
visible the calls below raise.  ``build()`` compiles ``csrc/*.hip`` for
gfx950 with hipcc into the package directory, so the ``.so`` travels with the
repository snapshot to the GPU box (it is git-ignored, not gpurun-ignored).
"""
from __future__ import annotations

import contextlib
import ctypes
import fcntl
import os
import subprocess
import tempfile
from pathlib import Path

PKG = Path(__file__).resolve().parent
REPO = PKG.parent
LIB_PATH = PKG / "librqsid.so"
SRCS = [PKG / "csrc" / "rqsid.hip", PKG / "csrc" / "assign.hip", PKG / "csrc" / "assign_stream.hip",
        PKG / "csrc" / "assign_resident.hip", PKG / "csrc" / "assign_rows.hip", PKG / "csrc" / "assign_pc.hip",
        PKG / "csrc" / "auction.hip",
        PKG / "csrc" / "auction_seg.hip"]
DEPS = SRCS + [PKG / "csrc" / "internal.h", PKG / "csrc" / "assign_common.h"]
HEADER = REPO / "include" / "rqsid.h"
# host-only I/O library (CSV reader): plain g++, no GPU code
IO_LIB_PATH = PKG / "librqsid_io.so"
IO_SRCS = [PKG / "csrc" / "csv_loader.cpp"]
IO_HEADER = REPO / "include" / "rqsid_io.h"
IO_FLAGS = ["-O3", "-std=c++17", "-Wall", "-shared", "-fPIC", "-pthread"]

HIPCC_FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fno-slp-vectorize", "-shared", "-fPIC"]

c_i32, c_i64, c_f32, c_vp, c_char_p = ctypes.c_int32, ctypes.c_int64, ctypes.c_float, ctypes.c_void_p, ctypes.c_char_p

# name -> (restype, argtypes); mirrors include/rqsid.h one to one
SIGNATURES = {
    "rqsid_version": (c_i32, []),
    "rqsid_last_error": (c_char_p, []),
    "rqsid_build_flags": (c_i32, []),
    "rqsid_prepare_centers": (c_i32, [c_vp, c_i64, c_i32, c_vp, c_vp, c_vp]),
    "rqsid_prepare_centers_hi": (c_i32, [c_vp, c_i64, c_i32, c_vp, c_vp]),
    "rqsid_bucket_workspace_bytes": (c_i64, [c_i64, c_i32]),
    "rqsid_bucket": (c_i32, [c_vp, c_i64, c_i32, c_i32, c_vp, c_vp, c_vp, c_vp, c_i64, c_vp]),
    "rqsid_assign_tile_rows": (c_i32, []),
    "rqsid_assign_workspace_bytes": (c_i64, [c_i64]),
    "rqsid_assign": (c_i32, [c_vp, c_i64, c_i32, c_vp, c_i32, c_vp, c_vp, c_i64,
                             c_vp, c_vp, c_vp, c_vp, c_i32,
                             c_vp, c_vp, c_i32, c_vp, c_vp, c_vp,
                             c_i32, c_i32, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp,
                             c_vp, c_vp, c_i32, c_vp, c_i64, c_vp]),
    "rqsid_residual": (c_i32, [c_vp, c_i64, c_i32, c_vp, c_i32, c_vp, c_vp, c_i32, c_i32, c_vp, c_vp]),
    "rqsid_scale_groups": (c_i32, [c_vp, c_i64, c_i32, c_vp, c_i32, c_vp, c_vp, c_vp]),
    "rqsid_centroid_tile_rows": (c_i32, []),
    "rqsid_centroid_accumulate": (c_i32, [c_vp, c_i32, c_vp, c_i32, c_vp, c_vp, c_i64, c_vp, c_vp]),
    "rqsid_centroid_finalize": (c_i32, [c_vp, c_vp, c_i32, c_i32, c_vp, c_vp]),
    "rqsid_match_workspace_bytes": (c_i64, [c_i32]),
    "rqsid_match_to_candidates": (c_i32, [c_vp, c_i32, c_i32, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_vp]),
    "rqsid_pairwise_distance": (c_i32, [c_vp, c_i64, c_i32, c_vp, c_i32, c_vp, c_vp]),
    "rqsid_auction_scores": (c_i32, [c_vp, c_i64, c_i32, c_vp, c_i32, c_i32, c_vp, c_vp]),
    "rqsid_auction_workspace_bytes": (c_i64, [c_i64, c_i32]),
    "rqsid_auction_lap_half": (c_i32, [c_vp, c_i32, c_i64, c_i32, c_vp, c_vp, c_vp, c_i64, c_vp]),
    "rqsid_auction_full_workspace_bytes": (c_i64, [c_i64, c_i32]),
    "rqsid_auction_lap_full": (c_i32, [c_vp, c_i32, c_i64, c_i32, c_vp, c_vp, c_vp, c_i64, c_vp]),
    "rqsid_seg_auction_scores": (c_i32, [c_vp, c_i64, c_i32, c_vp, c_i32, c_i32, c_vp, c_vp, c_i64, c_i32, c_vp,
                                         c_vp]),
    "rqsid_seg_auction_chunk_jobs": (c_i32, []),
    "rqsid_seg_auction_workspace_bytes": (c_i64, [c_i64, c_i32, c_i32, c_i64, c_i32]),
    "rqsid_seg_auction_lap_half": (c_i32, [c_vp, c_i32, c_i32, c_vp, c_vp, c_i64, c_i32, c_i64, c_vp, c_i32, c_vp,
                                           c_vp, c_vp, c_i64, c_vp]),
    "rqsid_pairwise_cosine": (c_i32, [c_vp, c_i64, c_i32, c_vp, c_i32, c_vp, c_vp, c_vp]),
    "rqsid_dauction_workspace_bytes": (c_i64, [c_i64, c_i32]),
    "rqsid_dauction_layout": (c_i32, [c_i64, c_i32, c_vp]),
    "rqsid_dauction_begin": (c_i32, [c_vp, c_i32, c_i64, c_i64, c_vp, c_vp, c_i64, c_vp]),
    "rqsid_dauction_eps": (c_i32, [c_vp, c_i32, c_i64, c_i64, c_vp, c_i64, c_vp]),
    "rqsid_dauction_hist": (c_i32, [c_vp, c_i32, c_i64, c_i64, c_i32, c_vp, c_i64, c_vp]),
    "rqsid_dauction_select": (c_i32, [c_vp, c_i32, c_i64, c_i64, c_i32, c_vp, c_i64, c_vp]),
    "rqsid_dauction_eqcount": (c_i32, [c_vp, c_i32, c_i64, c_i64, c_vp, c_i64, c_vp]),
    "rqsid_dauction_bid": (c_i32, [c_vp, c_i32, c_i64, c_i64, c_vp, c_vp, c_i64, c_vp]),
    "rqsid_dauction_resolve": (c_i32, [c_vp, c_i32, c_i64, c_i64, c_vp, c_vp, c_i64, c_vp]),
    "rqsid_dauction_end_round": (c_i32, [c_vp, c_i32, c_i64, c_i64, c_vp, c_i64, c_vp]),
    "rqsid_dauction_debug": (c_i32, [c_vp, c_i32, c_i64, c_i64, c_vp, c_vp, c_i64, c_vp]),
    "rqsid_dauction_list_pass": (c_i32, [c_vp, c_i32, c_i64, c_i64, c_i32, c_vp, c_vp, c_i64, c_vp]),
    "rqsid_greedy_match": (c_i32, [c_vp, c_vp, c_i32, c_i32, c_i32, c_vp, c_vp, c_vp]),
    "rqsid_mfma_probe": (c_i32, [c_i32, c_vp, c_vp, c_vp, c_vp, c_vp]),
}

IO_SIGNATURES = {
    "rqsid_csv_open": (c_i32, [c_char_p, c_i32, c_i64, c_i32, c_vp]),
    "rqsid_csv_rows": (c_i64, [c_vp]),
    "rqsid_csv_id_bytes": (c_i64, [c_vp]),
    "rqsid_csv_nonnumeric": (c_i64, [c_vp]),
    "rqsid_csv_records": (c_i64, [c_vp]),
    "rqsid_csv_copy": (c_i32, [c_vp, c_vp, c_vp, c_vp]),
    "rqsid_csv_copy_f16": (c_i32, [c_vp, c_vp]),
    "rqsid_csv_close": (None, [c_vp]),
    "rqsid_io_last_error": (c_char_p, []),
}

_lib = None
_io_lib = None


def _stale(lib: Path, deps) -> bool:
    return not lib.exists() or lib.stat().st_mtime < max(f.stat().st_mtime for f in deps)


@contextlib.contextmanager
def _build_lock():
    """One builder at a time (torchrun ranks or test workers may all find the library stale)."""
    lockdir = PKG / "build"
    lockdir.mkdir(exist_ok=True)
    with open(lockdir / ".lock", "w") as f:
        fcntl.flock(f, fcntl.LOCK_EX)
        try:
            yield
        finally:
            fcntl.flock(f, fcntl.LOCK_UN)


def build(force: bool = False, verbose: bool = False) -> Path:
    """Compile the HIP library for gfx950 (hipcc cross-compiles without a GPU)."""
    if not force and not _stale(LIB_PATH, DEPS + [HEADER]):
        return LIB_PATH
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    with _build_lock():
        if not force and not _stale(LIB_PATH, DEPS + [HEADER]):
            return LIB_PATH  # another process built it while this one waited
        compile_flags = [f for f in HIPCC_FLAGS if f != "-shared"]
        with tempfile.TemporaryDirectory(dir=PKG / "build") as objdir:
            objs = [Path(objdir) / (src.stem + ".o") for src in SRCS]
            cmds = [[hipcc, *compile_flags, "-c", "-o", str(o), str(src)] for src, o in zip(SRCS, objs)]
            if verbose:
                for c in cmds:
                    print(" ".join(c))
            # one hipcc per translation unit, in parallel (the kernels are template-heavy: minutes serially)
            procs = [subprocess.Popen(c) for c in cmds]
            bad = [c for c, pr in zip(cmds, procs) if pr.wait() != 0]
            if bad:
                raise subprocess.CalledProcessError(1, bad[0])
            tmp = Path(objdir) / LIB_PATH.name
            subprocess.run([hipcc, *HIPCC_FLAGS, "-o", str(tmp), *map(str, objs)], check=True)
            os.replace(tmp, LIB_PATH)
    return LIB_PATH


def build_io(force: bool = False, verbose: bool = False) -> Path:
    """Compile the host I/O library (g++)."""
    if not force and not _stale(IO_LIB_PATH, IO_SRCS + [IO_HEADER]):
        return IO_LIB_PATH
    with _build_lock():
        if not force and not _stale(IO_LIB_PATH, IO_SRCS + [IO_HEADER]):
            return IO_LIB_PATH
        with tempfile.TemporaryDirectory(dir=PKG / "build") as d:
            tmp = Path(d) / IO_LIB_PATH.name
            cmd = [os.environ.get("CXX", "g++"), *IO_FLAGS, "-o", str(tmp), *map(str, IO_SRCS)]
            if verbose:
                print(" ".join(cmd))
            subprocess.run(cmd, check=True)
            os.replace(tmp, IO_LIB_PATH)
    return IO_LIB_PATH


def load_io():
    """Load librqsid_io.so and bind every symbol of include/rqsid_io.h (raises if absent)."""
    global _io_lib
    if _io_lib is not None:
        return _io_lib
    if not IO_LIB_PATH.exists():
        raise RuntimeError(f"host I/O library {IO_LIB_PATH} is missing: run "
                           "`python -c 'import __graft_entry__ as g; g.build()'`")
    lib = ctypes.CDLL(str(IO_LIB_PATH))
    for name, (res, args) in IO_SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _io_lib = lib
    return lib


def load():
    """Load librqsid.so and bind every symbol of include/rqsid.h (raises if absent)."""
    global _lib
    if _lib is not None:
        return _lib
    path = Path(os.environ.get("RQSID_LIB", LIB_PATH))  # A/B builds of the same ABI (tools/)
    if not path.exists():
        raise RuntimeError(
            f"HIP library {path} is missing: run `python -c 'import __graft_entry__ as g; g.build()'` "
            "(there is no CPU fallback for the semantic-ID kernels)")
    lib = ctypes.CDLL(str(path))
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    flags = int(lib.rqsid_build_flags())
    if flags and "RQSID_LIB" not in os.environ:
        # a timing-probe build (tools/ab_build.sh) returns wrong IDs by design: only an explicit RQSID_LIB A/B
        # run may load one
        raise RuntimeError(f"{path} is a timing-probe build (rqsid_build_flags = {flags}); rebuild with "
                           "`python -c 'import __graft_entry__ as g; g.build()'`")
    _lib = lib
    return lib


def check(rc: int, what: str) -> None:
    if rc != 0:
        msg = load().rqsid_last_error().decode(errors="replace")
        if rc == -1:
            raise ValueError(f"{what}: {msg}")
        raise RuntimeError(f"{what} failed ({rc}): {msg}")
