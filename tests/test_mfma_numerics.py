"""Pin the accumulation numerics of v_mfma_f32_32x32x16_bf16 that rqsid_assign's
screening bound depends on ("Screening bound").

Each case puts 16 exactly representable bf16 products whose fp32 partial sums would
lose bits if the hardware rounded after every addition, and records what comes out.
"""
import numpy as np
import pytest
import torch

from generative_ranking_recommender_amd import _lib

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def bf16_bits(x):
    u = np.asarray(x, dtype=np.float32).view(np.uint32)
    assert ((u & 0xFFFF) == 0).all(), "values must be exact in bf16"
    return (u >> 16).astype(np.uint16)


def probe(a, b, c):
    lib = _lib.load()
    ta = torch.from_numpy(bf16_bits(a).view(np.int16)).to(DEV)
    tb = torch.from_numpy(bf16_bits(b).view(np.int16)).to(DEV)
    tc = torch.from_numpy(np.asarray(c, np.float32)).to(DEV)
    td = torch.empty((32, 32), dtype=torch.float32, device=DEV)
    _lib.check(lib.rqsid_mfma_probe(ta.data_ptr(), tb.data_ptr(), tc.data_ptr(), td.data_ptr(),
                                    torch.cuda.current_stream().cuda_stream), "probe")
    torch.cuda.synchronize()
    return td.cpu().numpy()


def test_layout_matches_matmul():
    rng = np.random.default_rng(0)
    a = bf16_bits(rng.integers(-8, 8, (32, 16)).astype(np.float32)).view(np.uint16)
    a = (a.astype(np.uint32) << 16).view(np.float32)
    b = (bf16_bits(rng.integers(-8, 8, (16, 32)).astype(np.float32)).astype(np.uint32) << 16).view(np.float32)
    c = rng.integers(-100, 100, (32, 32)).astype(np.float32)
    assert np.array_equal(probe(a, b, c), a.astype(np.float64) @ b + c)


def test_block_sum_rounding_model():
    """Row 0: 2^25 + 14*1 - 2^25 (+ C) — sequential fp32 adds lose the ones."""
    a = np.zeros((32, 16), np.float32)
    b = np.zeros((16, 32), np.float32)
    b[:, 0] = 1.0
    a[0, 0], a[0, 15] = 2.0 ** 25, -(2.0 ** 25)
    a[0, 1:15] = 1.0
    a[1, :] = [2.0 ** 25, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1]  # 2^25 + 15
    a[2, :8] = 2.0 ** -20
    a[2, 8] = 1.0
    c = np.zeros((32, 32), np.float32)
    c[3, 0] = 2.0 ** 25
    a[3, :14] = 1.0  # C = 2^25, products 14 -> one rounding gives 2^25+16
    d = probe(a, b, c)
    res = {"cancel": float(d[0, 0]), "big_plus_ones": float(d[1, 0]), "tiny_plus_one": float(d[2, 0]),
           "c_plus_14": float(d[3, 0])}
    print("MFMA numerics:", res)
    # the screening bound (rqsid.hip screening_tau) assumes at most 17 fp32-rounding
    # additions per instruction; every model tried is at least that accurate:
    exact = {"cancel": 14.0, "big_plus_ones": 2.0 ** 25 + 15, "tiny_plus_one": 1.0 + 8 * 2.0 ** -20,
             "c_plus_14": 2.0 ** 25 + 16}
    for k, v in res.items():
        assert abs(v - exact[k]) <= 17 * 2.0 ** -24 * (2.0 ** 26), (k, v)
