"""Host-side surface budgets (compton2d_amd/surface.py) against the reference's own
tables: the golden EC case (tests/golden/ec_lower.npz) holds what the reference's
file_sp (src/imcsurf2d_para.f:544-685) and imcgen2d (src/imcgen2d.f:174-183, 442,
481-485) left in COMMON for three MC steps with disk/blackbody_20110929.in on both
lower rings."""
import os
from pathlib import Path

import numpy as np
import pytest

from compton2d_amd import abi, surface as S
from golden_io import GoldenCase

REF_DISK = Path(os.environ.get("C2D_REFERENCE", "/root/reference")) / "disk"


def test_file_sp_matches_reference_bit_for_bit():
    gc = GoldenCase("ec_lower")
    tab, int_file = S.file_sp(S.seed_spectrum("blackbody_20110929"), S.EcConstants())
    nfile = len(tab.E_file)
    for n in range(gc.nsteps):
        assert gc.meta["step%d" % n]["nfile"] == nfile
        for k in ("E_file", "F_file"):
            np.testing.assert_array_equal(getattr(tab, k), gc.out(n, k)[:nfile])
        for k in ("a1", "I_file", "P_file"):
            np.testing.assert_array_equal(getattr(tab, k), gc.out(n, k)[:nfile - 1])
    assert tab.P_file[-1] == 1.0 and np.all(np.diff(tab.P_file) >= 0)
    assert int_file > 0


def test_lower_surface_budget_matches_reference():
    gc = GoldenCase("ec_lower")
    _, int_file = S.file_sp(S.seed_spectrum("blackbody_20110929"), S.EcConstants())
    nst = gc.meta["case"]["nst"]
    for n in range(gc.nsteps):
        st = gc.meta["step%d" % n]
        si = gc.step_inputs(n)
        ns, ew = S.lower_surface_budget(gc.a["cfg_r"], gc.meta["rmin"], nst, st["dt"],
                                        np.asarray(si.tbbl, float), True, int_file)
        np.testing.assert_array_equal(ns, si.nsurfl)
        np.testing.assert_array_equal(ew, si.ewsurfl)


def test_budget_off_window_and_ring_counts():
    r = np.array([1.0, 2.0, 3.0, 4.0]) * 1e16
    ns, ew = S.lower_surface_budget(r, 0.0, 16000, 10.0, np.full(4, -1.0), False, 5.0)
    # packets are still allotted to EC rings outside the t0 gate, with the blackbody
    # energy of tbb = -1 (sigma * 1, sigma = 1.0267d24 in keV units, imcgen2d.f:13-14),
    # as imcgen2d.f:179 and :442 do
    # int() truncation of the f64 expression, as the Fortran assignment does (999, not 1000)
    assert list(ns) == [int(16000 * (r[k] ** 2 - (r[k - 1] if k else 0.0) ** 2) / r[-1] ** 2)
                        for k in range(4)]
    assert abs(int(ns.sum()) - 16000) <= 4
    A = S.ring_areas(r, 0.0)
    assert S.SIGMA_SB == 1.0267e24
    np.testing.assert_allclose(ew, 10.0 * A * 1.0267e24 / ns, rtol=1e-15)
    ns0, ew0 = S.lower_surface_budget(r, 0.0, 16000, 10.0, np.zeros(4), True, 5.0)
    assert ns0.sum() == 0 and ew0.sum() == 0.0


def test_time_window():
    t1 = [4.0e5, 1.0e30]
    assert S.time_window(0, 1e9, 1e3, t1) == 0            # ncycle 0: window 1
    assert S.time_window(3, 1.0e5, 1e3, t1) == 0
    assert S.time_window(3, 4.0e5, 1e3, t1) == 1          # time + dt/2 > t1(1)
    assert S.time_window(3, 1e31, 1e3, t1) == 2           # past every window


def test_bias_cap():
    si = GoldenCase("ec_lower").step_inputs(0)
    nsv0, ew0 = si.nsv.copy(), si.ewsv.copy()
    assert S.apply_bias(1000, si) == 1.0
    fb = S.apply_bias(100, si)                            # n_new = 1498 > 10 * 100
    assert fb == pytest.approx(1000.0 / 1498.0)
    np.testing.assert_array_equal(si.nsv, (nsv0 * fb).astype(np.int32))
    np.testing.assert_array_equal(si.ewsv, ew0 / fb)


@pytest.mark.skipif(not REF_DISK.is_dir(), reason="reference sources not present (GPU box)")
def test_shipped_seed_spectra_equal_reference_files():
    for name in ("blackbody_20110929", "blackbody_G25_4spectra"):
        np.testing.assert_array_equal(S.read_seed_columns(REF_DISK / (name + ".in")),
                                      S.seed_spectrum(name))


def test_g25_spectrum_is_usable():
    tab, int_file = S.file_sp(S.seed_spectrum("blackbody_G25_4spectra"), S.EcConstants(g_bulk=25.0))
    assert len(tab.E_file) == abi.NFMAX - 1
    assert np.isfinite(tab.P_file).all() and tab.P_file[-1] == 1.0 and int_file > 0


@pytest.mark.skipif(not (REF_DISK.parent / "postprocessing").is_dir(),
                    reason="reference sources not present (GPU box)")
def test_c5_binning_equals_ext25_deck():
    import importlib.util
    from compton2d_amd import observer as O
    root = Path(__file__).resolve().parents[1]
    spec = importlib.util.spec_from_file_location("c5_bench", root / "tools" / "c5_bench.py")
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    a = m.ext25_binning()
    b = O.parse_plcm_deck((REF_DISK.parent / "postprocessing" / "ext25_lc.input").read_text())
    for k in ("mode", "gam_bulk", "rmax", "t0", "t1", "mu0", "mu1", "E0", "E1", "dt",
              "t_offset", "t_stop"):
        np.testing.assert_array_equal(getattr(a, k), getattr(b, k))


def test_upper_surface_budget_matches_reference():
    """EC file spectrum on the upper rings (ec_upper: tbbu = -1)."""
    gc = GoldenCase("ec_upper")
    _, int_file = S.file_sp(S.seed_spectrum("blackbody_20110929"), S.EcConstants())
    nst = gc.meta["case"]["nst"]
    for n in range(gc.nsteps):
        st = gc.meta["step%d" % n]
        si = gc.step_inputs(n)
        assert si.nsurfu.sum() > 0
        ns, ew = S.upper_surface_budget(gc.a["cfg_r"], gc.meta["rmin"], nst, st["dt"],
                                        np.asarray(si.tbbu, float), True, int_file)
        np.testing.assert_array_equal(ns, si.nsurfu)
        np.testing.assert_array_equal(ew, si.ewsurfu)


def test_blackbody_ring_energy_matches_reference():
    """tbbu > 0: erinu = dt*A*sigma*tbbu^4 (imcgen2d.f:155-157) but no packets
    (imcgen2d.f:437); bb_upper's driver gave each such ring 200 packets of
    weight erinu/200 (oracle/ref/c2d_refdrv.f NFORCEU)."""
    gc = GoldenCase("bb_upper")
    nst = gc.meta["case"]["nst"]
    for n in range(gc.nsteps):
        st = gc.meta["step%d" % n]
        si = gc.step_inputs(n)
        tb = np.asarray(si.tbbu, float)
        assert (tb > 0).all()
        ns, ew, erin = S.ring_budget(gc.a["cfg_r"], gc.meta["rmin"], nst, st["dt"], tb, True, 0.0)
        assert ns.sum() == 0 and ew.sum() == 0.0
        np.testing.assert_array_equal(si.nsurfu, 200)
        np.testing.assert_array_equal(erin / 200.0, si.ewsurfu)


@pytest.mark.parametrize("name", ["ssc_tau", "ec_lower", "grid3x4", "c3_mrk421"])
def test_volume_budget_matches_reference(name):
    """nsv/ewsv from Eloss_tot (imcgen2d.f:406-413, :446-456), bit for bit."""
    gc = GoldenCase(name)
    nst = gc.meta["case"]["nst"]
    for n in range(gc.nsteps):
        si = gc.step_inputs(n)
        nsv, ewsv = S.volume_budget(nst, si.Eloss_tot)
        np.testing.assert_array_equal(nsv, si.nsv)
        np.testing.assert_array_equal(ewsv, si.ewsv)


@pytest.mark.parametrize("bad", [np.nan, np.inf, -np.inf])
def test_volume_budget_raises_on_non_finite_emission(bad):
    """A NaN emissivity (r08b: NaN tables after an n_field overflow) raises
    instead of casting NaN to a negative packet count, which the reference's
    `do i=1,nsv` would skip silently (src/imcgen2d.f:446-456)."""
    si = GoldenCase("c3_mrk421").step_inputs(1)
    fas = np.array(si.Eloss_tot, float)
    fas[3, 2] = bad
    with pytest.raises(FloatingPointError, match="non-finite"):
        S.volume_budget(20000, fas)
    fas[3, 2] = -1.0
    with pytest.raises(ValueError, match="negative"):
        S.volume_budget(20000, fas)
