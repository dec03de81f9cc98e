"""Fail loudly on non-finite state (the r08b collapse: an f32 n_field overflow
made the FP state and tables NaN, the budget cast NaN to a negative count,
c2d_set_step clipped it to 0 and the run tracked nothing with exit 0).

The reference `stop`s on its own error paths (src/imctrk2d.f:573-577) but
carries a NaN on; the library refuses it instead:
* c2d_set_step: a negative nsv / surface count is C2D_E_ARG; NaN/Inf in a
  table, n_e, a budget weight or a seed spectrum (hazard H9) is
  C2D_E_NONFINITE, and no step is left to run (C2D_E_STATE after);
* c2d_run_step: a tally that overflows to Inf is C2D_E_NONFINITE;
* c2d_fp_step: NaN/Inf in the device n_field/ecens it reads (written here
  through a caller-owned tally tensor) or in the state it writes is C2D_E_FP;
* c2d_volume_em: NaN/Inf in its inputs or outputs is C2D_E_NONFINITE;
* surface.volume_budget (host) raises on a NaN emissivity
  (tests/test_surface.py, CPU).
"""
import numpy as np
import pytest

from compton2d_amd import abi, synth
from compton2d_amd.engine import C2DError, Engine
from golden_io import FpGoldenCase, GoldenCase

pytestmark = pytest.mark.gpu


def _expect(code, fn, *a, **k):
    with pytest.raises(C2DError) as e:
        fn(*a, **k)
    assert e.value.code == code, str(e.value)
    return e.value


def test_set_step_rejects_negative_counts_and_nan_tables():
    gc = GoldenCase("ec_lower")
    eng = Engine(gc.grid(comtot_mode=abi.COMTOT_TABLE, device=0))
    good = gc.step_inputs(1)
    eng.transport_step(good)
    si = gc.step_inputs(1)
    si.nsv = si.nsv.copy()
    si.nsv[0, 1] = -2147483648            # int(NaN) as the reference's budget makes it
    _expect(-1, eng.set_step, si)              # C2D_E_ARG
    _expect(-7, eng.run_step)             # C2D_E_STATE: the failed set_step left no step
    for key, val in (("kappa_tot", np.nan), ("eps_tot", np.inf), ("n_e", np.nan)):
        si = gc.step_inputs(1)
        arr = getattr(si, key).copy()
        arr.flat[arr.size - 1] = val
        setattr(si, key, arr)
        _expect(abi.C2D_E_NONFINITE, eng.set_step, si)
    si = gc.step_inputs(1)
    si.ewsv = si.ewsv.copy()
    si.ewsv[si.nsv > 0] = np.nan
    _expect(abi.C2D_E_NONFINITE, eng.set_step, si)
    si = gc.step_inputs(1)
    si.nsurfl = si.nsurfl.copy()
    si.nsurfl[0] = -1
    _expect(-1, eng.set_step, si)              # C2D_E_ARG
    si = gc.step_inputs(1)                 # hazard H9: disk/blackbody.in's NaN column
    assert si.spectra, "ec_lower steps carry the file_sp table"
    sp = si.spectra[0]
    sp.F_file = sp.F_file.copy()
    sp.F_file[3] = np.nan
    _expect(abi.C2D_E_NONFINITE, eng.set_step, si)
    eng.transport_step(good)               # the context recovers with good inputs
    assert eng.tallies()["counters"][abi.CNT_STEPS] > 0
    eng.close()


def test_run_step_rejects_an_overflowing_tally():
    """Finite inputs whose deposits overflow f64 (weights of 1e308): the step's
    tally check (capi.cpp c2d_check_finite over the fused buffer)."""
    gc = GoldenCase("ssc_tau")
    eng = Engine(gc.grid(comtot_mode=abi.COMTOT_TABLE, device=0))
    si = gc.step_inputs(1)
    si.ewsv = np.where(si.nsv > 0, 1.0e308, si.ewsv)
    err = _expect(abi.C2D_E_NONFINITE, eng.transport_step, si)
    assert "tallies" in str(err)
    eng.close()


def test_fp_step_rejects_inf_in_device_n_field():
    """An Inf written into n_field through the caller-owned tally tensor (as an
    f32 overflow did in r08b): c2d_fp_step reading the device tallies is
    C2D_E_FP; so is an Inf in host n_field."""
    import torch
    tc = GoldenCase("ssc_tau")
    fc = FpGoldenCase("fp_pick")
    eng = Engine(tc.grid(comtot_mode=abi.COMTOT_EXACT, device=0))
    T = torch.zeros(eng.layout.total, dtype=torch.float64, device="cuda:0")
    eng.use_tally_tensor(T)
    eng.fp_set_config(fc.constants())
    eng.transport_step(tc.step_inputs(0))
    eng.transport_step(tc.step_inputs(1))
    fi = fc.fp_in(fc.steps[0])
    dev = dict(fi, n_field=None, ecens=None)
    ok = eng.fp_step(2, fi["time"], fi["dt"], dev, fi)         # finite: runs
    assert np.isfinite(ok["f_nt"]).all()
    nf0 = int(eng.layout.n_field)
    T[nf0 + 17] = float("inf")
    torch.cuda.synchronize()
    err = _expect(abi.C2D_E_FP, eng.fp_step, 2, fi["time"], fi["dt"], dev, fi)
    assert "NaN/Inf" in str(err)
    T[nf0 + 17] = 0.0
    T[int(eng.layout.ecens)] = float("nan")
    torch.cuda.synchronize()
    _expect(abi.C2D_E_FP, eng.fp_step, 2, fi["time"], fi["dt"], dev, fi)
    host = dict(fi, n_field=fi["n_field"].copy())              # host arrays: the same guard
    host["n_field"][0, 0, 3] = np.inf
    _expect(abi.C2D_E_FP, eng.fp_step, 2, fi["time"], fi["dt"], host, fi)
    eng.close()


def test_volume_em_rejects_nan_inputs():
    wl = synth.c3_workload(sources=1000)
    st = dict(wl.fixed, tea=wl.state0["tea"], n_e=wl.state0["n_e"], f_nt=wl.state0["f_nt"])
    eng = Engine(wl.grid)
    res = eng.volume_em(wl.dt, st)
    assert np.isfinite(res["kappa_tot"]).all() and np.isfinite(res["Eloss_tot"]).all()
    bad = np.array(st["f_nt"], float)
    bad[0, 0, 50] = np.nan
    _expect(abi.C2D_E_NONFINITE, eng.volume_em, wl.dt, dict(st, f_nt=bad))
    tea = np.array(st["tea"], float)
    tea[1, 1] = np.inf
    _expect(abi.C2D_E_NONFINITE, eng.volume_em, wl.dt, dict(st, tea=tea))
    eng.volume_em(wl.dt, st)               # and recovers with good inputs
    eng.close()
