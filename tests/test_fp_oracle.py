"""The C oracle of the Fokker-Planck update (oracle/c2d_fp_oracle.c) against the
reference itself: tests/golden/fp_*.npz hold the inputs and outputs of the
reference's `update`/FP_calc (src/update2d.f:7-327, :337-1739) dumped by
oracle/ref/c2d_refdrv.f after real transport steps (tests/golden/make_golden.py).

* glibc build ('ref'): every zone output (f_nt, Pnt, Te_new, tea, n_e, gmin,
  gmax, amxwl, p_nth) is bit-identical to the reference; the E_add_up sums
  (E_tot_old, E_tot_new, hr_total, hr_st_total) agree to 1e-13 (the reference
  accumulates one running sum over zones, the oracle sums per-zone shares);
  dT_max is exact.
* det-math build ('det', c2d_math.h, what the GPU computes): same outputs to
  1e-10 relative (fdlibm exp/log/pow vs glibc over thousands of implicit
  sub-steps), Te_new/tea/gmin/gmax/p_nth identical.
"""
import numpy as np
import pytest

import oracle_lib as OL
from golden_io import FP_CASES, FpGoldenCase

ZONE_KEYS = ("Te_new", "tea", "n_e", "gmin", "gmax", "amxwl", "p_nth", "f_nt", "Pnt")
SUM_KEYS = ("E_tot_old", "E_tot_new", "hr_total", "hr_st_total")


def run(case: FpGoldenCase, n: int, flavor: str) -> dict:
    fi = case.fp_in(n)
    return OL.fp_step(case.grid(), case.constants(), fi["ncycle"], fi["time"], fi["dt"], fi, fi,
                      flavor=flavor)


@pytest.mark.parametrize("name", FP_CASES)
def test_fp_oracle_bitwise_equals_reference(name):
    case = FpGoldenCase(name)
    assert case.steps, "fixture has no FP step"
    for n in case.steps:
        r, ref = run(case, n, "ref"), case.fp_out(n)
        for k in ZONE_KEYS:
            np.testing.assert_array_equal(r[k], ref[k], err_msg="%s step %d %s" % (name, n, k))
        for k in SUM_KEYS:
            assert abs(r[k] - ref[k]) <= 1e-13 * abs(ref[k]), (name, n, k, r[k], ref[k])
        assert r["dT_max"] == ref["dT_max"]
        assert np.all(r["zone_diag"][..., 5] >= 1)     # implicit sub-steps taken


@pytest.mark.parametrize("name", FP_CASES)
def test_fp_oracle_detmath_close_to_reference(name):
    case = FpGoldenCase(name)
    for n in case.steps:
        r, ref = run(case, n, "det"), case.fp_out(n)
        for k in ("Te_new", "tea", "gmin", "gmax", "p_nth"):
            np.testing.assert_array_equal(r[k], ref[k], err_msg="%s step %d %s" % (name, n, k))
        for k in ("n_e", "amxwl", "f_nt", "Pnt"):
            a, b = r[k], ref[k]
            scale = np.maximum(np.abs(b), 1e-30 * np.max(np.abs(b)))
            assert np.max(np.abs(a - b) / scale) < 1e-10, (name, n, k)


def test_fp_zone_below_density_floor_is_left_untouched():
    """n_lept < 1e-11 returns before any update (update2d.f:478); Te_new = tea."""
    case = FpGoldenCase("fp_pick")
    n = case.steps[0]
    fi = case.fp_in(n)
    fi["n_e"] = fi["n_e"].copy()
    fi["n_e"][0, 1] = 1e-12
    r = OL.fp_step(case.grid(), case.constants(), fi["ncycle"], fi["time"], fi["dt"], fi, fi,
                   flavor="ref")
    np.testing.assert_array_equal(r["f_nt"][0, 1], fi["f_nt"][0, 1])
    np.testing.assert_array_equal(r["Pnt"][0, 1], fi["Pnt"][0, 1])
    assert r["Te_new"][0, 1] == fi["tea"][0, 1]
    assert r["zone_diag"][0, 1, 6] == 1.0
    assert r["n_e"][0, 1] == 1e-12


def test_gamma_bar_limits():
    """gamma_bar (volume2d.f:572-594): non-relativistic branch below Theta=0.2
    (single-precision literal), McDonald ratio above, floor 1."""
    lib = OL.load("ref")
    assert lib.c2o_gamma_bar(1e-6) == 1.0 or abs(lib.c2o_gamma_bar(1e-6) - 1.0) < 1e-5
    g_lo = lib.c2o_gamma_bar(np.float32(0.2) - 1e-9)
    g_hi = lib.c2o_gamma_bar(float(np.float32(0.2)))
    assert abs(g_lo - g_hi) / g_hi < 1e-3        # the two branches meet at Theta = 0.2
    for th in (0.5, 2.0, 10.0):                  # relativistic limit <gamma> ~ 3 Theta
        g = lib.c2o_gamma_bar(th)
        assert 1.0 < g and abs(g / (3 * th) - 1) < 0.6


def test_fp_pair_switch_branch_is_exercised():
    """fp_pair runs the reference with pair_switch = 1 (C3's setting) and the
    MPI build's inert positrons (H6, emulated in oracle/ref/c2d_refdrv.f by
    the master's n_ph staying 0): loop 460 (update2d.f:1187-1217) clips
    f_old below 1e-50 every sub-step, so the pair_switch = 0 solve differs
    from the reference on this fixture while pair_switch = 1 is bit-exact
    (test above)."""
    case = FpGoldenCase("fp_pair")
    c0 = case.constants()
    c0.pair_switch = 0
    differs = False
    for n in case.steps:
        fi = case.fp_in(n)
        assert np.all(fi["f_pair"] == 0.0)
        r = OL.fp_step(case.grid(), c0, fi["ncycle"], fi["time"], fi["dt"], fi, fi, flavor="ref")
        differs |= not np.array_equal(r["f_nt"], case.fp_out(n)["f_nt"])
    assert differs


def test_fp_pair_switch_rejects_positron_population():
    case = FpGoldenCase("fp_pair")
    fi = case.fp_in(case.steps[0])
    fi["f_pair"] = fi["f_pair"].copy()
    fi["f_pair"][0, 0] = 0.2
    with pytest.raises(RuntimeError):
        OL.fp_step(case.grid(), case.constants(), fi["ncycle"], fi["time"], fi["dt"], fi, fi,
                   flavor="ref")


def test_fp_gaussian_injection_branch_is_exercised():
    """fp_gauss runs the reference with inj_switch = 1, inj_dis = 1: the shock
    injects a Gaussian in gamma (src/update2d.f:1254-1258) into the zones the
    front crosses (:1249-1251).  Its outputs are bit-exact (tests above); here:
    the branch really ran on the fixture -- the same solve without injection,
    and the same solve with the power-law profile (inj_dis = 2), both differ
    from the reference's output."""
    case = FpGoldenCase("fp_gauss")
    assert case.constants().inj_dis == 1 and case.constants().inj_switch == 1
    for variant in ("off", "powerlaw"):
        differs = False
        for n in case.steps:
            fi = case.fp_in(n)
            c = case.constants()
            if variant == "off":
                c.inj_switch = 0
            else:
                c.inj_dis = 2
            r = OL.fp_step(case.grid(), c, fi["ncycle"], fi["time"], fi["dt"], fi, fi, flavor="ref")
            differs |= not np.array_equal(r["f_nt"], case.fp_out(n)["f_nt"])
        assert differs, variant
