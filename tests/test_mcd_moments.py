"""The fast FP kernel's McDonald moment table (compton2d_amd/csrc/fp_fast.hip
mcd_mtab), restated in numpy: the pair's series at z from the moments at the
nearest grid point z0 (7 per series, 1024 grid points per octave) with the
stopping index moved to z's term by term, against the term-by-term series
(src/volume2d.f:598-626 as the fast kernel sums it: same terms, same stopping
test).  CPU-only: the method, not the kernel (tests/test_gpu_fp.py checks the
kernel's table against its own series on the GPU)."""
import math

import numpy as np
import pytest

N = 16384
DT = 1.001
K = 7
Q = 1024


@pytest.fixture(scope="module")
def lattice():
    t = np.empty(N)
    t[0] = 1.0
    for n in range(1, N):
        t[n] = t[n - 1] * DT            # the reference's repeated product
    ts = t * 0.5 * (1.0 + DT)
    return t, ts, (ts * ts - 1.0) ** 1.5, (ts * ts - 1.0) ** 2.5


def series(z, t, ts, p):
    """sum of the terms up to and including the first stopping term"""
    y = z * ts
    v = p * np.exp(-np.minimum(y, 225.0)) * (y < 225.0)
    stop = ~((t * DT < 2.0) | (v > 1e-8))
    f = int(np.argmax(stop))
    assert stop[f]
    return math.fsum((DT - 1.0) * t[: f + 1] * v[: f + 1]), f


def table_value(z, t, ts, p):
    j = round((math.log2(z) + 17) * Q)
    z0 = 2.0 ** (j / Q - 17)
    y = z0 * ts
    v = p * np.exp(-y)
    stop = ~((t * DT < 2.0) | (v > 1e-8))
    f0 = int(np.argmax(stop))
    w = (DT - 1.0) * t[: f0 + 1] * v[: f0 + 1]
    mom = [math.fsum(w * y[: f0 + 1] ** k / math.factorial(k)) for k in range(K)]
    eta = z / z0 - 1.0
    s = 0.0
    for k in reversed(range(K)):
        s = s * (-eta) + mom[k]

    def term(n):
        vn = p[n] * math.exp(-z * ts[n])
        return (DT - 1.0) * t[n] * vn, not (t[n] * DT < 2.0 or vn > 1e-8)

    tm, st = term(f0)
    if st:                              # f(z) <= f0: drop the terms past it
        f = f0
        while f > 0:
            tp, sp = term(f - 1)
            if not sp:
                break
            s -= tm
            tm, f = tp, f - 1
        return s, f
    n = f0 + 1                          # f(z) > f0: add the terms up to it
    while True:
        tn, sn = term(n)
        s += tn
        if sn:
            return s, n
        n += 1


def test_moment_table_equals_the_series(lattice):
    t, ts, p2, p3 = lattice
    rng = np.random.default_rng(11)
    zs = list(2.0 ** rng.uniform(-15.0, math.log2(5.0), 40)) + [5.0, 0.2, 1.0, 2.0 ** -15]
    zs += [2.0 ** ((j + 0.5) / Q - 17) for j in (2000, 9000, 17000)]     # half-way between grid points
    worst = 0.0
    for z in zs:
        for p in (p2, p3):
            a, fa = series(z, t, ts, p)
            b, fb = table_value(z, t, ts, p)
            assert fa == fb
            worst = max(worst, abs(b / a - 1.0))
    assert worst < 1e-13, worst
