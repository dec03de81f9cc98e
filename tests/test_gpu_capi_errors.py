"""The C-ABI's argument and state checks on a live context
(include/compton2d.h: every entry returns C2D_E_ARG for a bad argument and
C2D_E_STATE for a call out of order, with the reason in c2d_last_error, the
way the reference stops on its own error paths, src/imctrk2d.f:573-577):
the tally readback's range, steps and FP updates out of order, NULL outputs.
A failed call leaves the context usable."""
import ctypes as C

import numpy as np
import pytest

from compton2d_amd import abi
from compton2d_amd.engine import Engine
from golden_io import GoldenCase

pytestmark = pytest.mark.gpu

E_ARG, E_STATE = -1, -7


def _engine():
    gc = GoldenCase("ssc_tau")
    return gc, Engine(gc.grid(comtot_mode=abi.COMTOT_EXACT))


def test_tally_range_bounds_and_contents():
    gc, eng = _engine()
    eng.transport_step(gc.step_inputs(0))
    full = eng.tallies_raw()
    total = eng.layout.total
    buf = np.zeros(8)
    p = buf.ctypes.data_as(abi.PD)
    for off, n in ((-1, 4), (0, -1), (total - 3, 4), (total, 1)):
        assert eng.lib.c2d_tally_download_range(eng.ctx, p, off, n) == E_ARG, (off, n)
    assert eng.lib.c2d_tally_download_range(eng.ctx, None, 0, 4) == E_ARG
    assert eng.lib.c2d_tally_download_range(eng.ctx, p, 5, 0) == 0
    for off, n in ((0, total), (eng.layout.counters, abi.NCOUNTERS), (total - 1, 1)):
        np.testing.assert_array_equal(eng.tally_range(off, n), full[off:off + n])
    eng.close()


def test_steps_and_updates_out_of_order():
    gc, eng = _engine()
    # no step inputs yet
    assert eng.lib.c2d_run_step(eng.ctx) == E_STATE
    assert b"c2d_set_step" in eng.lib.c2d_last_error(eng.ctx)
    # the FP update: NULL structs, then before its configuration
    assert eng.lib.c2d_fp_step(eng.ctx, None, None) == E_ARG
    sin, sout = abi.FpStepIn(), abi.FpStepOut()
    assert eng.lib.c2d_fp_step(eng.ctx, C.byref(sin), C.byref(sout)) == E_STATE
    assert b"c2d_fp_set_config" in eng.lib.c2d_last_error(eng.ctx)
    # a failed call leaves the context usable: the step runs afterwards
    eng.transport_step(gc.step_inputs(0))
    assert eng.tallies()["counters"][abi.CNT_SOURCES] > 0
    eng.close()


def test_null_outputs_are_rejected():
    gc, eng = _engine()
    eng.transport_step(gc.step_inputs(0))
    assert eng.lib.c2d_events(eng.ctx, None, 0, None) == E_ARG
    assert eng.lib.c2d_tally_download(eng.ctx, None, eng.layout.total) == E_ARG
    buf = np.zeros(eng.layout.total - 1)
    assert eng.lib.c2d_tally_download(eng.ctx, buf.ctypes.data_as(abi.PD), buf.size) == E_ARG
    n = C.c_int64()
    assert eng.lib.c2d_events(eng.ctx, None, 0, C.byref(n)) == 0
    assert n.value == eng.last_event_count() == int(eng.tallies()["counters"][abi.CNT_EVENTS])
    eng.close()
