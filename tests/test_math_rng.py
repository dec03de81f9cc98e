"""Deterministic math (c2d_math.h) and the lineage RNG (c2d_rng.h) on the CPU.

c2d_math restates fdlibm; it must stay within 1 ulp of glibc (2 for acos/pow)
so that the det-math oracle is a faithful stand-in for the reference's libm.
Philox4x32-10 is checked against the Random123 known-answer vectors.
"""
import ctypes as C

import numpy as np
import pytest

import oracle_lib as OL
from compton2d_amd import abi


def ulp_diff(a, b):
    ia = a.view(np.int64)
    ib = b.view(np.int64)
    ia = np.where(ia < 0, np.int64(-0x8000000000000000) - ia, ia)
    ib = np.where(ib < 0, np.int64(-0x8000000000000000) - ib, ib)
    return np.abs(ia - ib)


@pytest.mark.parametrize("fn,lo,hi,maxulp", [
    (0, 1e-300, 1e300, 1), (1, -700.0, 700.0, 1), (2, -7.0, 14.0, 1), (3, -1.0, 1.0, 2),
    (4, 1e-30, 1e30, 32)])  # pow = exp(y*log x): error grows with |y ln x| (<= 23 here)
def test_det_math_vs_glibc(fn, lo, hi, maxulp):
    rng = np.random.default_rng(100 + fn)
    if fn in (0, 4):
        x = np.exp(rng.uniform(np.log(lo), np.log(hi), 100000))
    else:
        x = rng.uniform(lo, hi, 100000)
    special = {0: [1.0, 2.0, 0.5, 1e-310, 5e-324, 1.0000001], 1: [0.0, 1e-20, -1e-20, 0.5, -0.34657359],
               2: [0.0, 1e-9, np.pi / 4, 3.1415926536, 6.283185307], 3: [0.0, 0.5, -0.5, 1.0, -1.0, 0.999999999],
               4: [1.0, 8.0, 27.0]}[fn]
    x[:len(special)] = special
    yd, yr = np.zeros_like(x), np.zeros_like(x)
    OL.load("det").c2o_unit_math(fn, x.ctypes.data_as(abi.PD), yd.ctypes.data_as(abi.PD), x.size)
    OL.load("ref").c2o_unit_math(fn, x.ctypes.data_as(abi.PD), yr.ctypes.data_as(abi.PD), x.size)
    assert ulp_diff(yd, yr).max() <= maxulp


def log_pos_inputs():
    """Positive finite doubles that reach every path of c2d_log: wide range,
    near 1 (|f| < 2^-20 and both sides of the sqrt(2) split), powers of two,
    subnormals, (0, 1) uniforms as the transport draws them."""
    rng = np.random.default_rng(77)
    parts = [np.exp(rng.uniform(np.log(1e-308), np.log(1e308), 200000)),
             1.0 + rng.uniform(-2.0 ** -19, 2.0 ** -19, 50000),
             np.ldexp(1.0 + rng.uniform(0.0, 1.0, 50000), rng.integers(-1000, 1000, 50000)),
             np.ldexp(1.0, np.arange(-1074, 1024)).astype(np.float64),
             rng.uniform(0.0, 1.0, 100000), 1.0 - rng.uniform(0.0, 1e-6, 50000),
             np.array([5e-324, 1e-310, 2.2250738585072014e-308, 1.0, 2.0, 0.5, 1.4142135623730951,
                       0.7071067811865476, 1.7976931348623157e308])]
    return np.concatenate(parts)


def test_branch_free_log_bitwise_equals_log():
    """c2d_log_pos (the bundle kernel's log, no branches) == c2d_log bit for bit."""
    x = log_pos_inputs()
    y0, y5 = np.zeros_like(x), np.zeros_like(x)
    lib = OL.load("det")
    lib.c2o_unit_math(0, x.ctypes.data_as(abi.PD), y0.ctypes.data_as(abi.PD), x.size)
    lib.c2o_unit_math(5, x.ctypes.data_as(abi.PD), y5.ctypes.data_as(abi.PD), x.size)
    np.testing.assert_array_equal(y5.view(np.uint64), y0.view(np.uint64))


def exp_inputs():
    rng = np.random.default_rng(6)
    parts = [rng.uniform(-750.0, 750.0, 200000), rng.uniform(-1.5, 1.5, 100000),
             rng.uniform(-1e-7, 1e-7, 50000), rng.uniform(-746.0, -700.0, 50000),
             rng.uniform(700.0, 710.0, 50000),
             np.ldexp(rng.uniform(-0.5, 0.5, 50000), rng.integers(-60, 20, 50000)),
             np.array([0.0, -0.0, 3.7252902984e-09, -3.7252902984e-09, 0.34657359027997264,
                       -0.3465735902799727, 1.0397207708399179, -1.0397207708399179,
                       709.782712893384, 709.79, -745.1332191019411, -745.2, 1000.0, -1000.0,
                       np.inf, -np.inf, np.nan, 5e-324, -5e-324])]
    return np.concatenate(parts)


def test_branch_free_exp_bitwise_equals_exp():
    """c2d_exp_bf (the FP and table kernels' exp, no branches) == c2d_exp bit
    for bit, NaN/inf/overflow/subnormal results included."""
    x = exp_inputs()
    y1, y6 = np.zeros_like(x), np.zeros_like(x)
    lib = OL.load("det")
    lib.c2o_unit_math(1, x.ctypes.data_as(abi.PD), y1.ctypes.data_as(abi.PD), x.size)
    lib.c2o_unit_math(6, x.ctypes.data_as(abi.PD), y6.ctypes.data_as(abi.PD), x.size)
    np.testing.assert_array_equal(y6.view(np.uint64), y1.view(np.uint64))


def test_rng_known_answers():
    lib = OL.load("det")
    # Random123 kat_vectors, philox4x32-10: (ctr, key) -> out
    kats = [((0, 0, 0, 0), (0, 0), (0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8)),
            ((0xffffffff,) * 4, (0xffffffff, 0xffffffff),
             (0x408f276d, 0x41c83b0e, 0xa20bc7c6, 0x6d5451fd)),
            ((0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344), (0xa4093822, 0x299f31d0),
             (0xd16cfe09, 0x94fdcceb, 0x5001e420, 0x24126ea1))]
    for ctr, key, out in kats:
        # c2o_unit_derive(key, tag, a, b) runs philox on ctr = (a, b, tag, DERIVE_C3)
        # -> test the raw permutation through the draw/derive wrappers is not
        # possible for arbitrary ctr[3]; use the python restatement instead
        got = philox_py(ctr, key)
        assert got == out
    # the C implementation agrees with the Python one on derive()/draw()
    for key in (0, 1, 0x5EEDC2D, (1 << 64) - 1):
        for (a, b, tag) in ((0, 0, 1), (7, 3, 9), (123456, 99, 11)):
            d = lib.c2o_unit_derive(key, tag, a, b)
            w = philox_py((a, b, tag, 0x9E3779B9), (key & 0xffffffff, key >> 32))
            assert d == (w[1] << 32) | w[0]
        for n in (0, 1, 2, 17, 1 << 20, (1 << 20) + 1):
            u = lib.c2o_unit_philox_draw(key, n)
            # draw n = 53 bits of SplitMix64 output n of the sequence seeded with key
            x = splitmix_py(key, n) >> 11
            assert u == (x + 0.5) * 2.0 ** -53
            assert 0.0 < u < 1.0
        # sub-streams (split1 copies) and sub-stream derivations
        for sub in (1, 7, 0xFFFFFF):
            for n in (0, 1, 5):
                u = lib.c2o_unit_philox_draw_s(key, sub, n)
                assert u == ((splitmix_py(key, (sub << 32) | n) >> 11) + 0.5) * 2.0 ** -53
            d = lib.c2o_unit_derive_s(key, 11, 5, 9, sub)
            w = philox_py((5, 9, 11 | (sub << 8), 0x9E3779B9), (key & 0xffffffff, key >> 32))
            assert d == (w[1] << 32) | w[0]


def splitmix_py(seed, i):
    """Output i (0-based) of SplitMix64 seeded with `seed` (Steele, Lea &
    Flood 2014; java.util.SplittableRandom): state seed + (i+1)*gamma, mixed."""
    m = (1 << 64) - 1
    z = (seed + (i + 1) * 0x9E3779B97F4A7C15) & m
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & m
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & m
    return z ^ (z >> 31)


def test_splitmix_known_answers():
    # the published SplitMix64 sequence for seed 0 (reference splitmix64.c)
    assert [splitmix_py(0, i) for i in range(3)] == [0xE220A8397B1DCDAF, 0x6E789E6AA1B965F4,
                                                     0x06C45D188009454F]


def philox_py(ctr, key):
    M0, M1, W0, W1 = 0xD2511F53, 0xCD9E8D57, 0x9E3779B9, 0xBB67AE85
    c0, c1, c2, c3 = ctr
    k0, k1 = key
    m = 0xffffffff
    for _ in range(10):
        p0 = M0 * c0
        p1 = M1 * c2
        hi0, lo0 = p0 >> 32, p0 & m
        hi1, lo1 = p1 >> 32, p1 & m
        c0, c1, c2, c3 = (hi1 ^ c1 ^ k0) & m, lo1, (hi0 ^ c3 ^ k1) & m, lo0
        k0 = (k0 + W0) & m
        k1 = (k1 + W1) & m
    return (c0, c1, c2, c3)


def test_lineage_streams_are_distinct():
    lib = OL.load("det")
    keys = set()
    base = 0x5EEDC2D
    for tag in range(1, 12):
        for a in range(200):
            keys.add(lib.c2o_unit_derive(base, tag, a, 0))
    assert len(keys) == 11 * 200
    u = np.array([lib.c2o_unit_philox_draw(base, n) for n in range(20000)])
    assert abs(u.mean() - 0.5) < 0.01 and abs(u.var() - 1 / 12) < 0.005
