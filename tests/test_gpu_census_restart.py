"""Checkpoint / restart through the reference's census record files
(write_record -> write_cens, read_record -> read_cens, src/census2d.f):
a context restarted from the file continues the same histories.  With the
key file the lineage keys are exact; the 6 doubles lose precision to e14.7
exactly as the reference's restart does, so the next step's tallies agree to
the level of that truncation (a few census decisions may flip)."""
import numpy as np
import pytest

from compton2d_amd import abi
from compton2d_amd.engine import Engine
from golden_io import GoldenCase

pytestmark = pytest.mark.gpu


def test_restart_from_census_file(tmp_path):
    gc = GoldenCase("ssc_tau")
    a = Engine(gc.grid(comtot_mode=abi.COMTOT_EXACT, kappa_lag=0))
    a.transport_step(gc.step_inputs(0))
    n = a.save_census(tmp_path / "p001_census.dat")
    assert n == a.census_count() > 0
    b = Engine(gc.grid(comtot_mode=abi.COMTOT_EXACT, kappa_lag=0))
    assert b.load_census(tmp_path / "p001_census.dat") == n
    si = gc.step_inputs(1)
    a.transport_step(si)
    b.transport_step(si)
    ta, tb = a.tallies(), b.tallies()
    for k in (abi.CNT_SOURCES, abi.CNT_STEPS, abi.CNT_CENSUS, abi.CNT_ESCAPES):
        x, y = ta["counters"][k], tb["counters"][k]
        assert abs(x - y) <= 1e-3 * x + 2, (k, x, y)
    for k in ("edep", "ecens", "fout"):
        x, y = np.sum(ta[k]), np.sum(tb[k])
        assert abs(x - y) <= 1e-3 * abs(x), (k, x, y)
    a.close()
    b.close()
