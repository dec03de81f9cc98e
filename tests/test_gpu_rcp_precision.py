"""Precision of the fast transport build's reciprocal and reciprocal-sqrt
sequences (transport.hip rcp_pos / the point loop's rsq, C2D_RSQ_NR): the
gfx950 estimates v_rcp_f64 / v_rsq_f64 alone and after ONE Newton step,
against the host's correctly rounded 1/x and 1/sqrt(x) over 12 decades
(c2d_selftest_math).  Printed; asserted: one Newton step is within a few
ulp (the estimate alone is ~2^-24): the fast build takes one step
(C2D_FAST_NR, C2D_RSQ_NR)."""
import numpy as np
import pytest

from compton2d_amd.engine import device_math as selftest_math

pytestmark = pytest.mark.gpu


def test_rcp_rsq_one_newton_step(capsys):
    rng = np.random.default_rng(11)
    x = 10.0 ** rng.uniform(-6, 6, 1 << 20)
    out = {}
    for fn, ref, name in ((10, 1.0 / x, "rcp"), (11, 1.0 / x, "rcp+1N"),
                          (12, 1.0 / np.sqrt(x), "rsq"), (13, 1.0 / np.sqrt(x), "rsq+1N")):
        y = selftest_math(fn, x)
        out[name] = float(np.max(np.abs(y - ref) / ref))
    with capsys.disabled():
        print("\nmax relative error over 1e-6..1e6:", {k: "%.2e" % v for k, v in out.items()})
    # measured on the box (r05k): estimates 4.6e-8 / 5.2e-8, one step 2.2e-15 / 4.1e-15
    assert out["rcp"] > 1e-9 and out["rsq"] > 1e-9
    assert out["rcp+1N"] < 1e-14 and out["rsq+1N"] < 1e-14


def test_tau_log_f32_relative_precision_in_the_tail(capsys):
    """The fast build's optical-depth log (c2d_device.hpp c2d_tau_log_f32,
    transport.hip TAU_LOG) over uniforms spread from 1e-16 to within 1e-16 of
    1: relative error ~1e-7 everywhere.  A collision in the optically thin C3
    medium needs u within ~1e-5 of 1, where v_log_f32 of (float)u kept only
    1 - u to 6e-8 absolute (1e-3 relative; 0 for u > 1 - 2^-25)."""
    rng = np.random.default_rng(12)
    tail = 1.0 - 10.0 ** rng.uniform(-16, -0.31, 1 << 19)
    u = np.concatenate([rng.random(1 << 19), tail, 10.0 ** rng.uniform(-16, -0.31, 1 << 16)])
    u = u[(u > 0) & (u < 1)]
    y = selftest_math(14, u)
    rel = np.abs(y - np.log(u)) / np.abs(np.log(u))
    with capsys.disabled():
        print("\ntau log f32: max relative error %.2e (tail u > 0.99999: %.2e)"
              % (rel.max(), rel[u > 0.99999].max()))
    assert rel.max() < 1e-6
