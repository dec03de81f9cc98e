"""Edge cases of the transport step on the GPU, exact build against the
oracle's lineage mode (as tests/test_gpu_parity.py): a step with no work at
all (no volume or surface sources, empty census), a ragged step with a single
volume source, and a step whose only sources sit on one z-surface.  The
reference's own drivers run such steps when a zone's emissivity or a
surface's flux rounds to no packets (src/imcvol2d_para.f:90-156,
src/imcsurf2d_para.f:228-253): nothing may be tallied, no record written,
and the step after it must be the oracle's again."""
import dataclasses

import numpy as np
import pytest

import oracle_lib as OL
from compton2d_amd import abi
from compton2d_amd.engine import Engine
from golden_io import GoldenCase

pytestmark = pytest.mark.gpu

COUNTERS = (abi.CNT_STEPS, abi.CNT_ESCAPES, abi.CNT_CENSUS, abi.CNT_COLLIDE, abi.CNT_KILLED,
            abi.CNT_SOURCES, abi.CNT_COMPB, abi.CNT_EVENTS, abi.CNT_ESC_SCAT)
TALLY_KEYS = ("edep", "prdep", "ecens", "npcen", "n_field", "E_IC", "nelectron", "fout", "edout",
              "erlki", "erlko", "erlku", "erlkl", "Ed_in")
SURF_N = ("nsurfi", "nsurfo", "nsurfu", "nsurfl")


def _no_sources(si, keep_surface=None):
    """si with every source count zero (one z-surface entry kept if asked)."""
    rep = {"nsv": np.zeros_like(si.nsv)}
    for k in SURF_N:
        a = getattr(si, k)
        rep[k] = np.zeros_like(a)
        if keep_surface == k:
            rep[k][0] = max(int(np.max(a)), 50)
    return dataclasses.replace(si, **rep)


def _same(eng, orc, tag):
    tg, to = eng.tallies(), orc.split()
    np.testing.assert_array_equal(tg["counters"][list(COUNTERS)], to["counters"][list(COUNTERS)],
                                  err_msg="%s counters" % tag)
    for k in TALLY_KEYS:
        ref = np.asarray(to[k])
        scale = max(np.max(np.abs(ref)), 1e-300)
        np.testing.assert_allclose(tg[k], ref, rtol=1e-11, atol=1e-13 * scale, err_msg="%s %s" % (tag, k))
    d6g, i5g, kg = eng.census()
    d6o, i5o, ko = orc.census()
    assert len(kg) == len(ko), tag
    og, oo = np.argsort(kg), np.argsort(ko)
    np.testing.assert_array_equal(kg[og], ko[oo])
    np.testing.assert_array_equal(d6g[og], d6o[oo])
    return tg


@pytest.mark.parametrize("inplace", [0, 1])
def test_empty_step_then_normal_step(inplace):
    gc = GoldenCase("ssc_tau")
    eng = Engine(gc.grid(comtot_mode=abi.COMTOT_EXACT, census_inplace=inplace))
    orc = OL.Oracle(gc.grid(), OL.RNG_LINEAGE, "det")
    si0 = gc.step_inputs(0)
    empty = _no_sources(si0)
    eng.transport_step(empty)
    assert orc.step(empty) == 0
    tg = _same(eng, orc, "empty step")
    assert not np.any(tg["counters"][list(COUNTERS)])
    for k in TALLY_KEYS:
        assert not np.any(tg[k]), k
    assert len(eng.census()[2]) == 0 and len(eng.events()) == 0
    # the next steps run as if the empty one had not been there
    for n in range(gc.nsteps):
        si = gc.step_inputs(n)
        eng.transport_step(si)
        assert orc.step(si) == 0
        tg = _same(eng, orc, "after empty, step %d" % n)
        assert tg["counters"][abi.CNT_SOURCES] > 0
    eng.close()
    orc.close()


def test_single_volume_source():
    """One volume packet in the last zone (a ragged launch: one lane of one wave)."""
    gc = GoldenCase("ssc_tau")
    eng = Engine(gc.grid(comtot_mode=abi.COMTOT_EXACT))
    orc = OL.Oracle(gc.grid(), OL.RNG_LINEAGE, "det")
    si = _no_sources(gc.step_inputs(0))
    nsv = np.zeros_like(si.nsv)
    nsv.flat[nsv.size - 1] = 1
    si = dataclasses.replace(si, nsv=nsv)
    eng.transport_step(si)
    assert orc.step(si) == 0
    tg = _same(eng, orc, "one source")
    assert tg["counters"][abi.CNT_SOURCES] == 1
    eng.close()
    orc.close()


@pytest.mark.parametrize("side", SURF_N)
def test_surface_sources_only(side):
    gc = GoldenCase("ssc_tau")
    si = _no_sources(gc.step_inputs(0), keep_surface=side)
    ew, tbb = "ew" + side[1:], "tbb" + side[-1]
    # ssc_tau has no surface photons: a 0.5 keV blackbody (planck2d.f) on that side
    si = dataclasses.replace(si, **{ew: np.full_like(getattr(si, ew), 1.0e30),
                                    tbb: np.full_like(getattr(si, tbb), 0.5)})
    eng = Engine(gc.grid(comtot_mode=abi.COMTOT_EXACT))
    orc = OL.Oracle(gc.grid(), OL.RNG_LINEAGE, "det")
    eng.transport_step(si)
    assert orc.step(si) == 0
    tg = _same(eng, orc, "surface %s only" % side)
    assert tg["counters"][abi.CNT_SOURCES] == int(np.sum(getattr(si, side)))
    eng.close()
    orc.close()
