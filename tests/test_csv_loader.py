"""Native CSV reader (librqsid_io.so, include/rqsid_io.h) against the Python-csv restatement of the
reference's loader (oracle/csv_oracle.py; simplified_semantic_id_generator.py:38-76,
train_semantic_ids.py:72-131).  Bit-exact: same kept ids in the same order, same float32 / float16
bits, same non-numeric count, same exceptions.  CPU only."""
import ctypes
import os
import re

import numpy as np
import pytest

from generative_ranking_recommender_amd import _lib
from generative_ranking_recommender_amd import io as rq_io
from oracle import csv_oracle


@pytest.fixture(scope="module", autouse=True)
def built():
    _lib.build_io()


def native(path, dim, lc=(), limit=None, threads=0):
    """(ids, x, nonnumeric, records) straight from the C ABI."""
    lib = _lib.load_io()
    h = ctypes.c_void_p()
    rc = lib.rqsid_csv_open(os.fsencode(str(path)), dim, int(limit or 0), threads, ctypes.byref(h))
    assert rc == 0, lib.rqsid_io_last_error()
    bad, recs = lib.rqsid_csv_nonnumeric(h), lib.rqsid_csv_records(h)
    lib.rqsid_csv_close(h)
    ids, x = rq_io.load_song_vectors(str(path), dim, lc, limit, n_threads=threads)
    return ids, x, bad, recs


def same(a, b):
    return a.dtype == b.dtype and a.shape == b.shape and np.array_equal(a.view(np.uint8), b.view(np.uint8))


def check(path, dim, lc=(), limit=None, threads=0):
    ids, x, bad, _ = native(path, dim, lc, limit, threads)
    rids, rx, rbad = csv_oracle.load_song_vectors(str(path), dim, lc, limit)
    assert ids == rids
    assert same(x, rx)
    assert bad == rbad
    return ids, x


def test_header_and_binding_agree():
    text = (_lib.REPO / "include" / "rqsid_io.h").read_text()
    declared = set(re.findall(r"^\s*(?:const\s+)?[a-z0-9_]+\*?\s+\*?(rqsid_[a-z0-9_]+)\s*\(", text, re.M))
    assert declared == set(_lib.IO_SIGNATURES)
    lib = _lib.load_io()
    for name in declared:
        assert hasattr(lib, name), name


VALUES = ["1.5", " 2.25 ", "-0.0", "+.5", "5.", "1e-3", "1E+3", "1_000.5", "1e1_0", "nan", "-Infinity", "INF",
          "1e400", "-1e-400", "1e-45", "3.4028235677973366e38", "0.1", "65519.99", "65520", "6e-8", "2.9802322387695312e-08",
          "123456789012345678901234567890", "0." + "0" * 140 + "1"]
BAD = ["0x1p3", "nan(1)", "1.5f", "", "1__0", "_1", "1_", "1._5", "e5", "1e", "--1", "1e+", ".", "1.2.3", "inf5", "1,5"]


@pytest.mark.parametrize("lc", [(), (128, 1280)])
def test_value_grammar_matches_python(tmp_path, lc):
    p = tmp_path / "v.csv"
    lines = [f"ok{i},{v},1,2" for i, v in enumerate(VALUES)]
    lines += [f"bad{i},1,{v},2" for i, v in enumerate(BAD) if "," not in v]
    lines.append('bad_q,1,"1,5",2')
    p.write_text("\n".join(lines) + "\n")
    ids, _ = check(p, 3, lc)
    assert ids == [f"ok{i}" for i in range(len(VALUES))]


def test_record_rules(tmp_path):
    p = tmp_path / "r.csv"
    body = ("a,1,2\r\n"          # CRLF (csv.writer's own terminator)
            "\n"                  # blank record
            "short\n"             # < 2 fields
            "b,1\rc,3,4\r"        # lone CR ends records (universal newlines)
            '"q,1",5,6\n'         # quoted id with a comma
            '"he said ""hi""",7,8\n'
            '"multi\nline",9,10\n'  # quoted line break
            'x"y,11,12\n'         # quote inside an unquoted field is literal
            '"p"tail,13,14\n'     # text after a closing quote joins the field
            "d,1,2,3\n"           # another dimension
            ",15,16\n"            # empty id is kept
            "e,\"17\",18")        # quoted number, no final newline
    p.write_bytes(body.encode())
    ids, x = check(p, 2)
    assert ids == ["a", "c", "q,1", 'he said "hi"', "multi\nline", 'x"y', "ptail", "", "e"]
    for lim in range(0, 14):
        check(p, 2, limit=lim or None)


def test_utf8_ids(tmp_path):
    p = tmp_path / "u.csv"
    p.write_text("歌曲一,1,2\nchanson-é,3,4\n", encoding="utf-8")
    ids, _ = check(p, 2)
    assert ids == ["歌曲一", "chanson-é"]


@pytest.mark.parametrize("threads", [1, 3, 8])
def test_threaded_ranges_match(tmp_path, threads):
    """A file big enough to be cut into several ranges (>= 2 MiB per worker) reads identically with any
    worker count, with dirty rows scattered through it; limit cuts inside the file too."""
    rng = np.random.default_rng(7)
    n, d = 9000, 64
    x = rng.standard_normal((n, d)).astype(np.float32) * np.float32(30)
    lines = []
    for i in range(n):
        r = i % 97
        vals = ",".join(repr(float(v)) for v in x[i])
        if r == 3:
            lines.append(f"s{i},{vals},x")       # non-numeric and too long
        elif r == 5:
            lines.append(f"s{i},{vals[: vals.rfind(',')]}")  # one short
        elif r == 7:
            lines.append("")
        else:
            lines.append(f"s{i},{vals}")
    p = tmp_path / "big.csv"
    p.write_text("\r\n".join(lines) + "\r\n")
    assert p.stat().st_size > 8 << 20
    ids, got = check(p, d, threads=threads)
    assert len(ids) == n - 3 * (n // 97 + 1) + (1 if n % 97 <= 3 else 0) + (1 if n % 97 <= 5 else 0) \
        + (1 if n % 97 <= 7 else 0)
    check(p, d, (128, 1280), threads=threads)
    check(p, d, limit=5000, threads=threads)


def test_f16_conversion_is_numpy_rne(tmp_path):
    """The fp16 output rounds each float32 like numpy's astype / torch .half(): ties, subnormals,
    overflow to inf, nan."""
    bits = np.concatenate([
        np.random.default_rng(1).integers(0, 2 ** 32, 20000, dtype=np.uint64).astype(np.uint32),
        np.array([0x477FEFFF, 0x477FF000, 0x477FE000, 0x38800000, 0x387FFFFF, 0x33000000, 0x33000001,
                  0x32FFFFFF, 0x7F800000, 0xFF800000, 0x00000001, 0x3F801000, 0x3F803000], dtype=np.uint32)])
    v = bits.view(np.float32)
    v = v[~np.isnan(v)]
    p = tmp_path / "h.csv"
    p.write_text("".join(f"r{i},{repr(float(t))}\n" for i, t in enumerate(v)))
    ids, x = check(p, 1, (1280,))
    assert x.dtype == np.float16 and len(ids) == len(v)


def test_errors(tmp_path):
    p = tmp_path / "e.csv"
    p.write_text("a,1,2\n")
    with pytest.raises(ValueError):
        rq_io.load_song_vectors(str(p), 5)
    with pytest.raises(FileNotFoundError):
        rq_io.load_song_vectors(str(tmp_path / "missing.csv"), 2)
    with pytest.raises(FileNotFoundError):
        rq_io.load_song_vectors(str(tmp_path), 2)  # a directory is not a file (osp.isfile)
    e = tmp_path / "empty.csv"
    e.write_text("")
    with pytest.raises(ValueError):
        rq_io.load_song_vectors(str(e), 2)


def test_integration_md_csv_stub_runs(tmp_path, monkeypatch):
    """The ctypes stub INTEGRATION.md shows for the reference's loaders returns what the reference's
    reader returns (ids, and the fp16 tensor for PROD layer_clusters)."""
    import torch
    text = (_lib.REPO / "INTEGRATION.md").read_text()
    code = re.search(r"```python\n(# semantic_id_generator/_rqsid_io.py.*?)```", text, re.S).group(1)
    monkeypatch.setenv("RQSID_IO_LIB", str(_lib.IO_LIB_PATH))
    ns = {}
    exec(compile(code, "INTEGRATION.md", "exec"), ns)
    p = tmp_path / "s.csv"
    x = np.random.default_rng(3).standard_normal((50, 8)).astype(np.float32)
    rq_io.write_song_vectors(str(p), [f"id{i}" for i in range(50)], x)
    ids, t = ns["load_data"](str(p), 8, [128, 1280, 1280])
    rids, rx, _ = csv_oracle.load_song_vectors(str(p), 8, [128, 1280, 1280])
    assert ids == rids and t.dtype == torch.float16 and np.array_equal(t.numpy(), rx)
    with pytest.raises(FileNotFoundError):
        ns["load_data"](str(tmp_path / "nope.csv"), 8, [128])


def _near_midpoint_strings(n=6000, seed=11):
    """Decimal strings of 15-19 significant digits at and around the midpoints between adjacent
    float32 values and between adjacent doubles: the inputs where a wrong str -> double rounding would
    change the float32 that numpy produces (the double is cast to float32 afterwards)."""
    from decimal import Decimal, getcontext
    getcontext().prec = 80
    rng = np.random.default_rng(seed)
    f = (rng.standard_normal(n) * 10.0 ** rng.integers(-9, 9, n)).astype(np.float32)
    out = []
    for i, a in enumerate(f[: n // 2]):
        b = np.nextafter(a, np.float32(np.inf))
        mid = (Decimal(float(a)) + Decimal(float(b))) / 2
        for digits in (15, 17, 19):
            out.append(format(mid, f".{digits - 1}e"))
        half_ulp = Decimal(float(np.spacing(float(mid)))) / 2
        for k in (-1, 1):
            out.append(format(mid + k * half_ulp, ".18e"))
    for a in f[n // 2:]:
        d = float(a) * (1 + 1e-9)
        e = np.nextafter(d, np.inf)
        mid = (Decimal(d) + Decimal(e)) / 2
        out += [format(mid, ".18e"), format(mid, ".16e"), repr(d), f"{d:.9g}", f"{d:.12f}"]
    return out


def test_float_fast_path_matches_numpy(tmp_path):
    vals = _near_midpoint_strings()
    p = tmp_path / "m.csv"
    p.write_text("".join(f"r{i},{v}\n" for i, v in enumerate(vals)))
    ids, x = check(p, 1)
    assert len(ids) == len(vals)
    check(p, 1, (1280,))


def test_random_grammar_matches_python(tmp_path):
    """Random short tokens over the literal alphabet: accepted / rejected and valued as numpy does."""
    rng = np.random.default_rng(5)
    alpha = list("0123456789") * 3 + list(".eE+-_ ")
    toks = ["".join(rng.choice(alpha, rng.integers(1, 9))) for _ in range(4000)]
    p = tmp_path / "g.csv"
    p.write_text("".join(f"t{i},{t}\n" for i, t in enumerate(toks)))
    check(p, 1)
