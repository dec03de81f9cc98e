"""GPU parity of an external-Compton run whose boundary inputs come from the host
budget code (compton2d_amd/surface.py) rather than from a reference dump:
the Gamma = 25 seed spectrum `disk/blackbody_G25_4spectra.in` normalised by
`file_sp` on both lower rings while the first boundary window is open, then
switched off (src/imcgen2d.f:111-120, 174-183, 442, 481-485) — the C5 set-up
of tools/c5_bench.py on the 2x2 grid of the golden EC case.  The exact kernel
must reproduce the oracle's lineage-mode histories bit for bit (counters,
census, events) and its tallies to 1e-11 (atomic order)."""
import numpy as np
import pytest

import oracle_lib as OL
from compton2d_amd import abi, surface
from compton2d_amd.engine import Engine
from golden_io import GoldenCase
from test_gpu_parity import COUNTERS, TALLY_KEYS, sort_rows

pytestmark = pytest.mark.gpu

T1 = (2.0e5, 1.0e30)      # window 1 (EC on) ends after the second step of this case


def ec_steps(gc, nst):
    tab, int_file = surface.file_sp(surface.seed_spectrum("blackbody_G25_4spectra"),
                                    surface.EcConstants(g_bulk=25.0))
    r = np.asarray(gc.a["cfg_r"], float)
    out = []
    for n in range(4):
        base = gc.step_inputs(min(n, gc.nsteps - 1))
        st = gc.meta["step%d" % min(n, gc.nsteps - 1)]
        dt = st["dt"]
        ncycle, t = n, max(n - 1, 0) * dt
        w = surface.time_window(ncycle, t, dt, T1)
        tbbl = np.full(gc.nr, -1.0) if w == 0 else np.zeros(gc.nr)
        ns, ew = surface.lower_surface_budget(r, gc.meta["rmin"], nst, dt, tbbl, True, int_file)
        base.ncycle, base.time, base.dt = ncycle, t, dt
        base.nsurfl, base.ewsurfl, base.tbbl = ns, ew, tbbl
        base.spectra = [tab]
        surface.apply_bias(nst, base)
        out.append((w, base))
    return out


def test_ec_window_exact_parity():
    gc = GoldenCase("ec_lower")
    steps = ec_steps(gc, nst=1500)
    assert [w for w, _ in steps][:2] == [0, 0] and steps[-1][0] == 1
    eng = Engine(gc.grid(comtot_mode=abi.COMTOT_EXACT))
    orc = OL.Oracle(gc.grid(), OL.RNG_LINEAGE, "det")
    seen_events = 0
    for n, (w, si) in enumerate(steps):
        eng.transport_step(si)
        assert orc.step(si) == 0
        tg, to = eng.tallies(), orc.split()
        np.testing.assert_array_equal(tg["counters"][list(COUNTERS)], to["counters"][list(COUNTERS)],
                                      err_msg="step %d counters" % n)
        for k in TALLY_KEYS:
            ref = np.asarray(to[k])
            scale = max(np.max(np.abs(ref)), 1e-300)
            np.testing.assert_allclose(tg[k], ref, rtol=1e-11, atol=1e-13 * scale,
                                       err_msg="step %d %s" % (n, k))
        d6g, i5g, kg = eng.census()
        d6o, i5o, ko = orc.census()
        og, oo = np.argsort(kg), np.argsort(ko)
        np.testing.assert_array_equal(kg[og], ko[oo])
        np.testing.assert_array_equal(d6g[og], d6o[oo])
        np.testing.assert_array_equal(i5g[og], i5o[oo])
        eg, eo = eng.events(), orc.events()
        assert eg.shape == eo.shape
        np.testing.assert_array_equal(sort_rows(eg), sort_rows(eo))
        seen_events += len(eg)
        if w == 0:
            assert tg["counters"][abi.CNT_SOURCES] >= si.nsurfl.sum()
    assert seen_events > 0
    eng.close()
    orc.close()
