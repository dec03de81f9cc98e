"""GPU Fokker-Planck update (c2d_fp_step, compton2d_amd/csrc/fp.hip) against the
oracle (oracle/c2d_fp_oracle.c, det-math build) on the reference's own FP inputs
(tests/golden/fp_*.npz): every zone output bit-identical; E_add_up sums equal
(both sum the per-zone shares in zone order).  The oracle's glibc build is
pinned bit-exactly to the reference in tests/test_fp_oracle.py."""
import numpy as np
import pytest

import oracle_lib as OL
from compton2d_amd import abi
from compton2d_amd.engine import Engine
from golden_io import FP_CASES, FpGoldenCase, GoldenCase

pytestmark = pytest.mark.gpu

ZONE_KEYS = ("Te_new", "tea", "n_e", "gmin", "gmax", "amxwl", "p_nth", "f_nt", "Pnt", "zone_diag")


@pytest.mark.parametrize("name", FP_CASES)
def test_gpu_fp_bitwise_equals_oracle(name):
    case = FpGoldenCase(name)
    eng = Engine(case.grid(device=0))
    eng.fp_set_config(case.constants())
    for n in case.steps:
        fi = case.fp_in(n)
        g = eng.fp_step(fi["ncycle"], fi["time"], fi["dt"], fi, fi)
        o = OL.fp_step(case.grid(), case.constants(), fi["ncycle"], fi["time"], fi["dt"], fi, fi,
                       flavor="det")
        for k in ZONE_KEYS:
            np.testing.assert_array_equal(g[k], o[k], err_msg="%s step %d %s" % (name, n, k))
        for k in ("E_tot_old", "E_tot_new", "hr_total", "hr_st_total", "dT_max"):
            assert g[k] == o[k], (name, n, k, g[k], o[k])
        ref = case.fp_out(n)       # and close to the reference itself
        np.testing.assert_array_equal(g["Te_new"], ref["Te_new"])
        assert np.max(np.abs(g["f_nt"] - ref["f_nt"])) <= 1e-10 * np.max(np.abs(ref["f_nt"]))
    assert eng.last_fp_ms() > 0
    eng.close()


def test_gpu_fp_reads_photon_field_from_device_tallies():
    """n_field / ecens = None: the kernel reads the fused tally buffer of the
    preceding transport step directly (no host round trip)."""
    tc = GoldenCase("ssc_tau")
    fc = FpGoldenCase("fp_pick")
    eng = Engine(tc.grid(comtot_mode=abi.COMTOT_EXACT, device=0))
    eng.fp_set_config(fc.constants())
    eng.transport_step(tc.step_inputs(0))
    eng.transport_step(tc.step_inputs(1))
    t = eng.tallies()
    fi = fc.fp_in(fc.steps[0])
    host = dict(fi, n_field=t["n_field"], ecens=t["ecens"])
    dev = dict(fi, n_field=None, ecens=None)
    a = eng.fp_step(2, fi["time"], fi["dt"], host, fi)
    b = eng.fp_step(2, fi["time"], fi["dt"], dev, fi)
    for k in ZONE_KEYS:
        np.testing.assert_array_equal(a[k], b[k], err_msg=k)
    assert a["E_tot_new"] == b["E_tot_new"]
    eng.close()


def test_gpu_fp_rejects_positrons_and_requires_config():
    """pair_switch = 1 runs with the MPI build's inert positrons (H6); a zone
    with f_pair != 0 (a positron population) and pair_switch = 2 are errors."""
    case = FpGoldenCase("fp_pair")
    eng = Engine(case.grid(device=0))
    fi = case.fp_in(case.steps[0])
    with pytest.raises(Exception, match="C2D_E_STATE"):
        eng.fp_step(fi["ncycle"], fi["time"], fi["dt"], fi, fi)
    c = case.constants()
    assert c.pair_switch == 1
    eng.fp_set_config(c)
    bad = dict(fi, f_pair=fi["f_pair"].copy())
    bad["f_pair"][1, 0] = 0.1
    with pytest.raises(Exception, match="C2D_E_ARG"):
        eng.fp_step(fi["ncycle"], fi["time"], fi["dt"], bad, fi)
    c.pair_switch = 2
    with pytest.raises(Exception, match="C2D_E_ARG"):
        eng.fp_set_config(c)
    eng.close()


# C2D_FP_FAST tolerance: the same per-bin and per-term
# arithmetic as the exact kernel, only the order of the additions and the
# tridiagonal algorithm (PCR) differ, so the zone outputs equal the det-math
# oracle's to rounding carried through the zone's implicit sub-steps
FAST_TOL = {"f_nt": 1e-10, "Pnt": 1e-10, "n_e": 1e-12, "amxwl": 1e-9}


def fast_vs_oracle(g, o, label):
    """Deviations of a C2D_FP_FAST result from the det oracle; asserts the
    stated tolerance and returns the measured figures."""
    dev = {}
    for k in ("Te_new", "tea", "gmin", "gmax", "p_nth"):
        np.testing.assert_array_equal(g[k], o[k], err_msg="%s %s" % (label, k))
    for k, tol in FAST_TOL.items():
        d = np.max(np.abs(np.asarray(g[k]) - np.asarray(o[k]))) / max(np.max(np.abs(o[k])), 1e-300)
        dev[k] = float(d)
        assert d <= tol, (label, k, d)
    np.testing.assert_array_equal(g["zone_diag"][..., 5], o["zone_diag"][..., 5])   # sub-steps
    for k in ("E_tot_old", "E_tot_new", "hr_total"):
        d = abs(g[k] - o[k]) / max(abs(o[k]), 1e-300)
        dev[k] = float(d)
        assert d <= 1e-10, (label, k, g[k], o[k])
    return dev


@pytest.mark.parametrize("name", FP_CASES)
def test_gpu_fp_fast_within_tolerance(name, capsys):
    """C2D_FP_FAST (fp_fast.hip) vs the det oracle on the reference's FP inputs:
    temperatures (Te_new, tea), gmin/gmax, p_nth and the sub-step count equal;
    f_nt, Pnt within 1e-10 of the spectrum's maximum; n_e 1e-12; energies 1e-10."""
    case = FpGoldenCase(name)
    eng = Engine(case.grid(device=0))
    eng.fp_set_config(case.constants())
    eng.fp_set_mode(abi.FP_FAST)
    for n in case.steps:
        fi = case.fp_in(n)
        g = eng.fp_step(fi["ncycle"], fi["time"], fi["dt"], fi, fi)
        o = OL.fp_step(case.grid(), case.constants(), fi["ncycle"], fi["time"], fi["dt"], fi, fi,
                       flavor="det")
        dev = fast_vs_oracle(g, o, "%s step %d" % (name, n))
        with capsys.disabled():
            print("\nC2D_FP_FAST %s step %d: %s" % (name, n, {k: "%.1e" % v for k, v in dev.items()}))
    # the same update again: now through the zone queue (costliest zones first,
    # one workgroup per CU, the gamma_bar memo warm): bit for bit the same
    g2 = eng.fp_step(fi["ncycle"], fi["time"], fi["dt"], fi, fi)
    for k in ("f_nt", "Pnt", "Te_new", "tea", "n_e", "gmin", "gmax", "amxwl", "p_nth"):
        np.testing.assert_array_equal(np.asarray(g2[k]), np.asarray(g[k]), err_msg="queue rerun %s" % k)
    with pytest.raises(Exception, match="C2D_E_ARG"):
        eng.fp_set_mode(7)
    eng.close()


def test_gpu_fp_fast_zero_field_zone(capsys):
    """A zone with B = 0: the fast kernel's scalar chain multiplies by hoisted
    reciprocals (fp_fast.hip rcp_nr_safe), whose 1/0 must be inf as the
    oracle's division has it (the Newton steps alone give NaN), so the zone's
    synchrotron terms vanish the same way.  Same tolerance as above."""
    case = FpGoldenCase("fp_pick")
    n = case.steps[0]
    fi = dict(case.fp_in(n))
    fi["B_field"] = fi["B_field"].copy()
    fi["B_field"][0, 1] = 0.0
    eng = Engine(case.grid(device=0))
    eng.fp_set_config(case.constants())
    eng.fp_set_mode(abi.FP_FAST)
    g = eng.fp_step(fi["ncycle"], fi["time"], fi["dt"], fi, fi)
    o = OL.fp_step(case.grid(), case.constants(), fi["ncycle"], fi["time"], fi["dt"], fi, fi,
                   flavor="det")
    assert np.all(np.isfinite(o["f_nt"]))
    dev = fast_vs_oracle(g, o, "fp_pick B=0 zone")
    with capsys.disabled():
        print("\nC2D_FP_FAST fp_pick, zone (0,1) at B = 0: %s" % {k: "%.1e" % v for k, v in dev.items()})
    eng.close()


def test_gpu_fp_fast_mcdonald_moment_table(capsys):
    """The fast kernel's McDonald pair from its moment table (fp_fast.hip
    mcd_mtab: 7 moments per series at 1024 grid points per octave of z, the
    stopping index moved to z's term by term) against the same kernel's
    term-by-term series, at random z over the table's range and on and half-way
    between its grid points: K2, K3 and gamma_bar = K3/K2 - 1/z (formed as the
    kernel does, (z/2) (S3/S2) Gamma(2.5)/Gamma(3.5) - 1/z) within 1e-13
    relative.  The table answers wherever the series stops inside the abscissa
    table (z >= 2^-16 here; below, both take the series)."""
    from compton2d_amd.engine import device_mcd_fast
    rng = np.random.default_rng(5)
    z = np.concatenate([2.0 ** rng.uniform(-17.0, np.log2(5.0), 3000),
                        2.0 ** (np.arange(-17 * 1024, 3 * 1024 + 1, 37) / 1024.0),
                        2.0 ** ((np.arange(-17 * 1024, 3 * 1024, 41) + 0.5) / 1024.0),
                        [5.0, 0.2, 1.0, 2.0 ** -16]])
    out = device_mcd_fast(z)
    ok = out[:, 4] == 1.0
    assert np.all(ok[z >= 2.0 ** -16]), z[(z >= 2.0 ** -16) & ~ok][:5]
    d2 = np.abs(out[ok, 0] / out[ok, 2] - 1.0)
    d3 = np.abs(out[ok, 1] / out[ok, 3] - 1.0)
    gs = out[ok, 3] / out[ok, 2] - 1.0 / z[ok]
    dg = np.abs(out[ok, 7] / gs - 1.0)
    with capsys.disabled():
        print("\nmoment table: %d of %d z answered; max rel dev K2 %.1e K3 %.1e gamma_bar %.1e; "
              "shader cycles table %.0f (median) vs series %.0f"
              % (ok.sum(), len(z), d2.max(), d3.max(), dg.max(), np.median(out[ok, 5]),
                 np.median(out[ok, 6])))
    assert d2.max() <= 1e-13 and d3.max() <= 1e-13 and dg.max() <= 1e-13
