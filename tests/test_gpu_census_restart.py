"""Checkpoint / restart through the reference's census record files
(write_record -> write_cens, read_record -> read_cens, src/census2d.f;
the record text format is pinned to the reference's own write_cens in
tests/test_census_io.py).

A run writes its census after step 0; a fresh GPU context and the oracle
both restart from that same file (e14.7 doubles + the exact lineage keys of
the .keys file) and run step 1 on the same inputs: the exact kernel's
histories equal the oracle's bit for bit (counters, census records sorted by
key, escape events); f64 tallies to the atomic summation order.  A second
check keeps the old property: the restarted run stays within the e14.7
truncation of the uninterrupted one."""
import numpy as np
import pytest

import oracle_lib as OL
from compton2d_amd import abi, census_io
from compton2d_amd.engine import Engine
from golden_io import GoldenCase

pytestmark = pytest.mark.gpu

TALLY_KEYS = ("edep", "prdep", "ecens", "npcen", "n_field", "E_IC", "nelectron", "fout", "edout",
              "erlki", "erlko", "erlku", "erlkl", "Ed_in")


def sort_rows(a):
    return a[np.lexsort(a.T[::-1])] if len(a) else a


@pytest.mark.parametrize("name", ["ssc_tau", "c3_mrk421"])
def test_restart_from_census_file_matches_oracle(tmp_path, name):
    gc = GoldenCase(name)
    a = Engine(gc.grid(comtot_mode=abi.COMTOT_EXACT, kappa_lag=0))
    a.transport_step(gc.step_inputs(0))
    path = tmp_path / "p001_census.dat"
    n = a.save_census(path)
    assert n == a.census_count() > 0
    b = Engine(gc.grid(comtot_mode=abi.COMTOT_EXACT, kappa_lag=0))
    assert b.load_census(path) == n
    o = OL.Oracle(gc.grid(kappa_lag=0), OL.RNG_LINEAGE, "det")
    assert o.import_census(*census_io.read_census(path)) == 0
    si = gc.step_inputs(1)
    b.transport_step(si)
    assert o.step(si) == 0
    tb, to = b.tallies(), o.split()
    np.testing.assert_array_equal(tb["counters"][:8], to["counters"][:8])   # GENS is GPU-only
    for k in TALLY_KEYS:
        ref = np.asarray(to[k])
        np.testing.assert_allclose(tb[k], ref, rtol=1e-11, atol=1e-13 * max(np.abs(ref).max(), 1e-300),
                                   err_msg=k)
    d6b, i5b, kb = b.census()
    d6o, i5o, ko = o.census()
    ob, oo = np.argsort(kb), np.argsort(ko)
    np.testing.assert_array_equal(kb[ob], ko[oo])
    np.testing.assert_array_equal(d6b[ob], d6o[oo])
    np.testing.assert_array_equal(i5b[ob], i5o[oo])
    np.testing.assert_array_equal(sort_rows(b.events()), sort_rows(o.events()))
    # the uninterrupted run differs only through the e14.7 truncation
    a.transport_step(si)
    ta = a.tallies()
    for k in (abi.CNT_SOURCES, abi.CNT_STEPS, abi.CNT_CENSUS, abi.CNT_ESCAPES):
        x, y = ta["counters"][k], tb["counters"][k]
        assert abs(x - y) <= 1e-3 * x + 2, (k, x, y)
    for e in (a, b):
        e.close()
    o.close()


def test_fast_census_azimuth_encoding():
    """Fast contexts keep the census azimuth encoded (c2d_device.hpp
    CensusSoA: cos(phi) in the phi column, the quadrant switch in a bins
    bit).  The exported phi is the decode of the raw device words with the
    kernel's own acos, bit for bit, and an import re-encodes it as the
    kernel's set_phi would (cos of the phi it is given)."""
    import torch
    gc = GoldenCase("c3_mrk421")
    a = Engine(gc.grid(comtot_mode=abi.COMTOT_TABLE))
    a.transport_step(gc.step_inputs(0))
    d6, i5, keys = a.census()
    n = len(keys)
    assert n > 1000
    raw = torch.zeros(n * abi.CENSUS_REC_WORDS, dtype=torch.int64, device="cuda:0")
    a.census_pack(0, n, raw.data_ptr())
    w = raw.view(n, abi.CENSUS_REC_WORDS).cpu().numpy().view(np.uint64)
    eta = w[:, 3].view(np.float64)
    bins = (w[:, 6] >> np.uint64(32)).astype(np.uint32)
    esw = (bins & np.uint32(1 << 24)) != 0
    assert np.all(np.abs(eta) <= 1.0) and esw.any() and (~esw).any()
    acos = np.zeros_like(eta)
    OL.load("det").c2o_unit_math(3, np.ascontiguousarray(eta).ctypes.data_as(abi.PD),
                                 acos.ctypes.data_as(abi.PD), n)
    phi = np.where(esw, 2.0 * 3.1415926536 - acos, acos)
    np.testing.assert_array_equal(d6[:, 3].view(np.uint64), phi.view(np.uint64))
    np.testing.assert_array_equal(i5[:, 0], (bins & np.uint32(0xff)).astype(np.int32))
    # import: cos(phi) and the switch, as set_phi forms them
    b = Engine(gc.grid(comtot_mode=abi.COMTOT_TABLE))
    b.import_census(d6, i5, keys)
    raw2 = torch.zeros_like(raw)
    b.census_pack(0, n, raw2.data_ptr())
    w2 = raw2.view(n, abi.CENSUS_REC_WORDS).cpu().numpy().view(np.uint64)
    cosv = np.zeros_like(eta)
    OL.load("det").c2o_unit_math(2, np.ascontiguousarray(d6[:, 3]).ctypes.data_as(abi.PD),
                                 cosv.ctypes.data_as(abi.PD), n)
    np.testing.assert_array_equal(w2[:, 3], cosv.view(np.uint64))
    np.testing.assert_array_equal(w2[:, 6] >> np.uint64(32), w[:, 6] >> np.uint64(32))
    a.close()
    b.close()


def test_fast_census_small_azimuth_round_trip():
    """phi < 1e-10 is the reference's eta_switch = -1 case (imctrk2d.f:228-232):
    the import encodes cos(phi) = 1.0 with the switch, which the kernel never
    writes itself (it clamps the cosine to 0.999999999), and the export
    decodes it to 0.0 — so an imported phi = 0 comes back as 0."""
    gc = GoldenCase("c3_mrk421")
    a = Engine(gc.grid(comtot_mode=abi.COMTOT_TABLE))
    a.transport_step(gc.step_inputs(0))
    d6, i5, keys = a.census()
    a.close()
    phis = np.array([0.0, 5.0e-11, 1.0e-10, 1.0e-6, 1.0, 3.0, 4.0, 6.0])
    m = len(phis)
    d6, i5, keys = d6[:m].copy(), i5[:m].copy(), keys[:m].copy()
    d6[:, 3] = phis
    b = Engine(gc.grid(comtot_mode=abi.COMTOT_TABLE))
    b.import_census(d6, i5, keys)
    e6, _, ekeys = b.census()
    b.close()
    back = dict(zip(ekeys.tolist(), e6[:, 3].tolist()))
    got = np.array([back[k] for k in keys.tolist()])
    assert got[0] == 0.0 and got[1] == 0.0, got
    np.testing.assert_allclose(got[2:], phis[2:], rtol=0, atol=1e-9)


@pytest.mark.parametrize("inplace", [0, 1])
@pytest.mark.parametrize("mode", [abi.COMTOT_EXACT, abi.COMTOT_TABLE])
def test_census_overflow_is_reported(mode, inplace):
    """A step whose census does not fit fails with C2D_E_CENSUS_OVERFLOW (the
    reference's `stop 'too many photons'`, src/imctrk2d.f:573-577) instead of
    writing past the buffer."""
    from compton2d_amd.engine import C2DError
    gc = GoldenCase("ssc_tau")
    full = Engine(gc.grid(comtot_mode=mode))
    full.transport_step(gc.step_inputs(0))
    need = full.census_count()
    full.close()
    assert need > 200
    small = Engine(gc.grid(comtot_mode=mode, census_capacity=need // 4, census_inplace=inplace))
    with pytest.raises(C2DError) as e:
        small.transport_step(gc.step_inputs(0))
    assert e.value.code == -3, str(e.value)
    small.close()


@pytest.mark.parametrize("inplace", [0, 1])
@pytest.mark.parametrize("mode", [abi.COMTOT_EXACT, abi.COMTOT_TABLE])
def test_census_at_capacity_fits(mode, inplace):
    """A run whose census reaches exactly the configured capacity succeeds
    and matches the oracle's records, double-buffered or in place
    (c2d_device.hpp C2D_CENS_DEAD): the append chunks' tails (and in place
    the dead census slots) are compacted away, so the usable capacity is
    census_capacity itself (chunk tails cost up to ~20 %)."""
    gc = GoldenCase("ssc_tau")
    probe = Engine(gc.grid(comtot_mode=mode, census_inplace=inplace))
    need = []
    for n in range(gc.nsteps):
        probe.transport_step(gc.step_inputs(n))
        need.append(probe.census_count())
    probe.close()
    cap = max(need)
    assert cap > 1000
    eng = Engine(gc.grid(comtot_mode=mode, census_capacity=cap, census_inplace=inplace))
    orc = OL.Oracle(gc.grid(), OL.RNG_LINEAGE, "det")
    for n in range(gc.nsteps):
        si = gc.step_inputs(n)
        eng.transport_step(si)
        assert orc.step(si) == 0
        assert eng.census_count() == need[n]
        if mode == abi.COMTOT_EXACT:
            kg, ko = eng.census()[2], orc.census()[2]
            np.testing.assert_array_equal(np.sort(kg), np.sort(ko))
    eng.close()
    orc.close()


@pytest.mark.parametrize("inplace", [0, 1])
def test_census_compaction_in_many_rounds(monkeypatch, inplace):
    """The census close in many rounds: double-buffered, the compaction's
    work lists hold C2D_COMPACT_LIST dead/live slot pairs per round; chunked,
    the packing of the partly filled chunks moves C2D_CHUNK_BATCH records per
    two-phase round.  With 7 / 100 every step needs many rounds, and the
    census (and so the next step's histories) stays the oracle's."""
    monkeypatch.setenv("C2D_COMPACT_LIST", "7")
    monkeypatch.setenv("C2D_CHUNK_BATCH", "100")
    gc = GoldenCase("ssc_tau")
    eng = Engine(gc.grid(comtot_mode=abi.COMTOT_EXACT, census_inplace=inplace))
    orc = OL.Oracle(gc.grid(), OL.RNG_LINEAGE, "det")
    rounds = []
    for n in range(gc.nsteps):
        si = gc.step_inputs(n)
        eng.transport_step(si)
        assert orc.step(si) == 0
        rounds.append(eng.last_compaction()[0])
        kg, ko = eng.census()[2], orc.census()[2]
        np.testing.assert_array_equal(np.sort(kg), np.sort(ko))
        tg, to = eng.tallies(), orc.split()
        sel = [abi.CNT_STEPS, abi.CNT_ESCAPES, abi.CNT_CENSUS, abi.CNT_COLLIDE, abi.CNT_KILLED,
               abi.CNT_SOURCES, abi.CNT_COMPB, abi.CNT_EVENTS, abi.CNT_ESC_SCAT]
        np.testing.assert_array_equal(tg["counters"][sel], to["counters"][sel])
        if inplace:
            chunks, _, _, held = eng.last_census_chunks()
            assert chunks == -(-eng.census_count() // 1024) and held > chunks
    assert max(rounds) > 10, rounds
    eng.close()
    orc.close()


def test_chunked_census_recycles_chunks():
    """Chunked census over several steps of a census-dominated run: the
    bundle kernel refills the chunks its finished census sources leave (most
    of the census chunks), the census stays the oracle's record for record,
    and a capacity just above the census suffices."""
    gc = GoldenCase("c3_mrk421")
    probe = Engine(gc.grid(comtot_mode=abi.COMTOT_EXACT, census_inplace=1))
    need = []
    for n in range(gc.nsteps):
        probe.transport_step(gc.step_inputs(n))
        need.append(probe.census_count())
    probe.close()
    eng = Engine(gc.grid(comtot_mode=abi.COMTOT_EXACT, census_inplace=1, census_capacity=max(need)))
    orc = OL.Oracle(gc.grid(), OL.RNG_LINEAGE, "det")
    reused = []
    for n in range(gc.nsteps):
        si = gc.step_inputs(n)
        eng.transport_step(si)
        assert orc.step(si) == 0
        d6g, i5g, kg = eng.census()
        d6o, i5o, ko = orc.census()
        og, oo = np.argsort(kg), np.argsort(ko)
        np.testing.assert_array_equal(kg[og], ko[oo])
        np.testing.assert_array_equal(d6g[og], d6o[oo])
        np.testing.assert_array_equal(i5g[og], i5o[oo])
        chunks, rec, lost, held = eng.last_census_chunks()
        reused.append((rec, lost, chunks))
    # the census of step n-1 is step n's first items: its chunks come back,
    # every one of them (the open-addressed count-down table tracks them all)
    assert any(r > 0 for r, _, _ in reused[1:]), reused
    assert all(lost == 0 for _, lost, _ in reused), reused
    for n in range(1, len(reused)):
        assert reused[n][0] == reused[n - 1][2], reused
    eng.close()
    orc.close()


def test_chunked_census_at_capacity_on_few_waves(monkeypatch):
    """the chunked census's usable capacity is census_capacity.
    Two workgroups (C2D_BUNDLE_GRID: every wave runs many census chunks) and
    the additive slack cut to 48 chunks (C2D_CHUNK_SLACK: ~6 per wave, for its
    partly filled chunk, the chunks whose sources are in flight and its free
    stack) beside capacity/16: a capacity equal to the census the run needs
    suffices, no census chunk goes untracked and every input chunk is
    recycled within its step; records stay the oracle's."""
    gc = GoldenCase("c3_mrk421")
    probe = Engine(gc.grid(comtot_mode=abi.COMTOT_EXACT, census_inplace=1))
    need = []
    for n in range(gc.nsteps):
        probe.transport_step(gc.step_inputs(n))
        need.append(probe.census_count())
    probe.close()
    monkeypatch.setenv("C2D_BUNDLE_GRID", "2")
    monkeypatch.setenv("C2D_CHUNK_SLACK", "48")
    eng = Engine(gc.grid(comtot_mode=abi.COMTOT_EXACT, census_inplace=1, census_capacity=max(need)))
    orc = OL.Oracle(gc.grid(), OL.RNG_LINEAGE, "det")
    prev = 0
    for n in range(gc.nsteps):
        si = gc.step_inputs(n)
        eng.transport_step(si)
        assert orc.step(si) == 0
        assert eng.census_count() == need[n]
        chunks, rec, lost, held = eng.last_census_chunks()
        assert lost == 0 and rec == prev, (n, chunks, rec, lost, held)
        prev = chunks
        kg, ko = eng.census()[2], orc.census()[2]
        np.testing.assert_array_equal(np.sort(kg), np.sort(ko))
    eng.close()
    orc.close()


def test_chunked_census_lost_after_failed_step():
    """a chunked step that fails after generation 0 has
    rewritten the census in place leaves no stale census behind: the count
    is 0 and census reads and the next step fail with C2D_E_STATE until a
    census is imported (include/compton2d.h c2d_run_step).  The failure here
    is a scatter-queue overflow found after generation 0 (ssc_tau collides;
    queue_capacity 1).  A double-buffered context keeps its census."""
    from compton2d_amd.engine import C2DError
    gc = GoldenCase("ssc_tau")
    for inplace in (1, 0):
        eng = Engine(gc.grid(comtot_mode=abi.COMTOT_EXACT, census_inplace=inplace))
        eng.transport_step(gc.step_inputs(0))
        d6, i5, keys = eng.census()
        n0 = eng.census_count()
        assert n0 > 0
        eng.close()
        eng = Engine(gc.grid(comtot_mode=abi.COMTOT_EXACT, census_inplace=inplace, queue_capacity=1))
        eng.import_census(d6, i5, keys)
        with pytest.raises(C2DError) as e:
            eng.transport_step(gc.step_inputs(1))
        assert e.value.code == -5                          # C2D_E_QUEUE_OVERFLOW
        if inplace:
            assert eng.census_count() == 0
            for call in (lambda: eng.census(), lambda: eng.run_step()):
                with pytest.raises(C2DError) as e:
                    call()
                assert e.value.code == -7                  # C2D_E_STATE
            eng.import_census(d6, i5, keys)                # a new census: the context runs again
        else:
            assert eng.census_count() == n0
            np.testing.assert_array_equal(np.sort(eng.census()[2]), np.sort(keys))
        assert eng.census_count() == n0
        eng.close()
