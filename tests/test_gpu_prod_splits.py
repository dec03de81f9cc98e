"""The C3 deck's production splits on the GPU (SURVEY.md §8(d) "parity run").

src_20121026/input.dat:113-116 sets split1/split2/split3/spl3_trg =
1000/1000/300/10.  Two goldens made by the reference itself at those splits
(tests/golden/make_golden.py `prod_c3`, `prod_dense`; the oracle's reference
mode is bit-identical to them in tests/test_oracle_golden.py):

* `prod_c3`: C3's 30x9 grid and inputm.dat medium (optically thin).  Every
  source and census packet is 1000 probes (src/imctrk2d.f:105-138, 690-704);
  the GPU tracks them as 32 successive probe bundles (g0 = 0, 32, ..., 992,
  the last of 8 probes; transport.hip bundle_begin / bundle_restart), the
  oracle's lineage mode the same way (oracle/c2d_oracle.c probe_bundle loop).
* `prod_dense`: n_e = 1e5, where probes collide and every collision fans out
  to 1000 split2 secondaries, split3 fires on the >1e7 gains of the
  gmax = 1e5 tail and resamples 300 copies (src/imctrk2d.f:584-704); the
  secondaries run as scatter generations.

The scatter kernels' cooperative paths are forced on prod_dense through the
test knobs C2D_KN_CAP_ITERS and C2D_SC_K1_ATTEMPTS.

Bar (as tests/test_gpu_parity.py): the exact build is bit-identical to the
oracle's lineage mode (counters, census records by key, escape events) with
tallies to 1e-11 (f64 atomic order), in both census layouts; the secondary
loop split into many packet-store chunks (capi.cpp run_step_body, knob
C2D_PK_CHUNK) tracks the same histories; the fast build is within 1e-3
(test_gpu_parity.test_fast_kernel_close_to_oracle runs both cases: they are
in golden_io.CASES).
"""
import numpy as np
import pytest

import oracle_lib as OL
from compton2d_amd import abi
from compton2d_amd.engine import Engine
from golden_io import GoldenCase

pytestmark = pytest.mark.gpu

PROD = ("prod_c3", "prod_dense")
TALLY_KEYS = ("edep", "prdep", "ecens", "npcen", "n_field", "E_IC", "nelectron", "fout", "edout",
              "erlki", "erlko", "erlku", "erlkl", "Ed_in")
COUNTERS = (abi.CNT_STEPS, abi.CNT_ESCAPES, abi.CNT_CENSUS, abi.CNT_COLLIDE, abi.CNT_KILLED,
            abi.CNT_SOURCES, abi.CNT_COMPB, abi.CNT_EVENTS, abi.CNT_ESC_SCAT)


def sort_rows(a):
    return a[np.lexsort(a.T[::-1])] if len(a) else a


def _assert_same_histories(eng, orc, tag):
    tg, to = eng.tallies(), orc.split()
    np.testing.assert_array_equal(tg["counters"][list(COUNTERS)], to["counters"][list(COUNTERS)],
                                  err_msg="%s counters" % tag)
    assert tg["counters"][abi.CNT_ABORTED] == 0, tag
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
    np.testing.assert_array_equal(i5g[og], i5o[oo])
    eg, eo = eng.events(), orc.events()
    assert eg.shape == eo.shape, tag
    np.testing.assert_array_equal(sort_rows(eg), sort_rows(eo))
    return tg, to


def test_production_split_goldens_are_the_decks():
    """Both fixtures carry the deck's splits and reach the branches they are for."""
    for name in PROD:
        m = GoldenCase(name).meta
        assert (m["split1"], m["split2"], m["split3"], m["spl3_trg"]) == (1000, 1000, 300, 10)
    c3 = GoldenCase("prod_c3")
    assert (c3.nz, c3.nr) == (30, 9) and c3.out(1, "census_d").shape[0] > 1000
    dn = GoldenCase("prod_dense")
    assert dn.out(1, "E_IC").sum() > 0 and len(dn.out(1, "events")) > 1000


@pytest.mark.parametrize("inplace", [0, 1])
@pytest.mark.parametrize("name", PROD)
def test_exact_kernel_bit_parity_production_splits(name, inplace):
    gc = GoldenCase(name)
    eng = Engine(gc.grid(comtot_mode=abi.COMTOT_EXACT, census_inplace=inplace))
    orc = OL.Oracle(gc.grid(), OL.RNG_LINEAGE, "det")
    for n in range(gc.nsteps):
        si = gc.step_inputs(n)
        eng.transport_step(si)
        assert orc.step(si) == 0
        tg, to = _assert_same_histories(eng, orc, "%s step %d inplace %d" % (name, n, inplace))
        # 32 bundles per source (31 of 32 probes + one of 8): the lane
        # path-steps are far fewer than the per-copy packet-steps
        g0p, allp = eng.last_path_steps()
        assert 0 < g0p <= allp < tg["counters"][abi.CNT_STEPS]
    if name == "prod_dense":
        # collisions among the probes, split2 fan-out and split3 resampling ran
        assert to["counters"][abi.CNT_COLLIDE] > 10 and to["counters"][abi.CNT_COMPB] > 1e5
    eng.close()
    orc.close()


@pytest.mark.parametrize("inplace", [0, 1])
def test_exact_kernel_bit_parity_chunked_secondaries(monkeypatch, inplace):
    """prod_dense with the secondary loop cut into packet-store chunks of 4096
    (the 1000-way split2 fan-out of one generation spans many chunks, as a
    full-size run's does past the 4M-entry store): same histories, more launches."""
    gc = GoldenCase("prod_dense")
    plain = Engine(gc.grid(comtot_mode=abi.COMTOT_EXACT, census_inplace=inplace))
    monkeypatch.setenv("C2D_PK_CHUNK", "4096")
    eng = Engine(gc.grid(comtot_mode=abi.COMTOT_EXACT, census_inplace=inplace))
    orc = OL.Oracle(gc.grid(), OL.RNG_LINEAGE, "det")
    for n in range(gc.nsteps):
        si = gc.step_inputs(n)
        monkeypatch.delenv("C2D_PK_CHUNK")
        plain.transport_step(si)
        monkeypatch.setenv("C2D_PK_CHUNK", "4096")
        eng.transport_step(si)
        assert orc.step(si) == 0
        _assert_same_histories(eng, orc, "chunked step %d" % n)
        nl_plain, nl = plain.last_kernel_ms()[2], eng.last_kernel_ms()[2]
        if n == 1:
            assert nl >= nl_plain + 20, (nl, nl_plain)
    plain.close()
    eng.close()
    orc.close()


def test_exact_kernel_bit_parity_production_splits_few_waves(monkeypatch):
    """Generation 0 on two workgroups: each wave restarts its bundles across
    many work chunks (C2D_BUNDLE_GRID), census items included."""
    monkeypatch.setenv("C2D_BUNDLE_GRID", "2")
    gc = GoldenCase("prod_c3")
    eng = Engine(gc.grid(comtot_mode=abi.COMTOT_EXACT, census_inplace=1))
    orc = OL.Oracle(gc.grid(), OL.RNG_LINEAGE, "det")
    for n in range(gc.nsteps):
        si = gc.step_inputs(n)
        eng.transport_step(si)
        assert orc.step(si) == 0
        _assert_same_histories(eng, orc, "few waves step %d" % n)
    eng.close()
    orc.close()


@pytest.mark.parametrize("kn,sc", [("0", "0"), ("1", "1"), ("0", "16"), ("32", "0")])
def test_exact_kernel_bit_parity_cooperative_scatter(monkeypatch, kn, sc):
    """The scatter kernels' wave-cooperative paths forced on prod_dense:
    C2D_KN_CAP_ITERS = 0 resolves every compb2d first loop (compb_2d.f:59-93)
    64 iterations per round across the wave (transport.hip kn_coop), and
    C2D_SC_K1_ATTEMPTS = 0 sends every split3 copy to the hard kernel (one
    wave per copy, 64 resamples per round, the ones past the first success
    rolled back).  Iteration j of the first loop draws counters c0 + 5j ..
    c0 + 5j + 4 and resample k sub-stream k in both the kernels and the
    oracle's lineage mode, so the histories stay the oracle's bit for bit."""
    monkeypatch.setenv("C2D_KN_CAP_ITERS", kn)
    monkeypatch.setenv("C2D_SC_K1_ATTEMPTS", sc)
    gc = GoldenCase("prod_dense")
    eng = Engine(gc.grid(comtot_mode=abi.COMTOT_EXACT))
    orc = OL.Oracle(gc.grid(), OL.RNG_LINEAGE, "det")
    for n in range(gc.nsteps):
        si = gc.step_inputs(n)
        eng.transport_step(si)
        assert orc.step(si) == 0
        _assert_same_histories(eng, orc, "kn %s sc %s step %d" % (kn, sc, n))
    eng.close()
    orc.close()
