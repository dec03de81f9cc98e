"""GPU parity: the HIP transport kernels against the oracle on the same inputs.

* exact build (C2D_COMTOT_EXACT, -ffp-contract=off) vs the oracle's lineage
  mode with the same deterministic math (liboracle_det): every packet history
  is the same, so counters, the census (sorted by lineage key) and the escape
  events are bit-identical; tallies agree to 1e-11 relative (only the order
  of the floating-point atomic additions differs).
* fast build (C2D_COMTOT_TABLE: cubic comtot table) vs the same oracle:
  the table changes comtot by < 1e-7 relative, so only packets whose
  collision/census decision lies within that margin can differ; tallies and
  counters agree to 1e-3 relative on these fixtures.
Inputs are the reference's own per-step tables (tests/golden/*.npz).
"""
import numpy as np
import pytest

import oracle_lib as OL
from compton2d_amd import abi
from compton2d_amd.engine import Engine, device_math
from golden_io import CASES, GoldenCase

pytestmark = pytest.mark.gpu

TALLY_KEYS = ("edep", "prdep", "ecens", "npcen", "n_field", "E_IC", "nelectron", "fout", "edout",
              "erlki", "erlko", "erlku", "erlkl", "Ed_in")
COUNTERS = (abi.CNT_STEPS, abi.CNT_ESCAPES, abi.CNT_CENSUS, abi.CNT_COLLIDE, abi.CNT_KILLED,
            abi.CNT_SOURCES, abi.CNT_COMPB, abi.CNT_EVENTS, abi.CNT_ESC_SCAT)


def sort_rows(a):
    return a[np.lexsort(a.T[::-1])] if len(a) else a


def _run_pair(name, mode, seed=0x5EEDC2D):
    gc = GoldenCase(name)
    grid = gc.grid(comtot_mode=mode, seed=seed)
    eng = Engine(grid)
    orc = OL.Oracle(gc.grid(seed=seed), OL.RNG_LINEAGE, "det")
    for n in range(gc.nsteps):
        si = gc.step_inputs(n)
        eng.transport_step(si)
        assert orc.step(si) == 0
        yield n, eng, orc
    eng.close()
    orc.close()


@pytest.mark.parametrize("name", CASES)
def test_exact_kernel_bit_parity_with_oracle(name):
    for n, eng, orc in _run_pair(name, abi.COMTOT_EXACT):
        tg, to = eng.tallies(), orc.split()
        np.testing.assert_array_equal(tg["counters"][list(COUNTERS)], to["counters"][list(COUNTERS)],
                                      err_msg="%s step %d counters" % (name, n))
        # lane path-steps (roofline unit): a bundle's shared step counts once
        g0p, allp = eng.last_path_steps()
        assert 0 < g0p <= allp <= tg["counters"][abi.CNT_STEPS], (name, n, g0p, allp)
        assert eng.last_gen0_steps() >= g0p
        for k in TALLY_KEYS:
            ref = np.asarray(to[k])
            scale = max(np.max(np.abs(ref)), 1e-300)
            np.testing.assert_allclose(tg[k], ref, rtol=1e-11, atol=1e-13 * scale,
                                       err_msg="%s step %d %s" % (name, n, k))
        d6g, i5g, kg = eng.census()
        d6o, i5o, ko = orc.census()
        assert len(kg) == len(ko)
        og, oo = np.argsort(kg), np.argsort(ko)
        np.testing.assert_array_equal(kg[og], ko[oo])
        np.testing.assert_array_equal(d6g[og], d6o[oo])
        np.testing.assert_array_equal(i5g[og], i5o[oo])
        eg, eo = eng.events(), orc.events()
        assert eg.shape == eo.shape
        np.testing.assert_array_equal(sort_rows(eg), sort_rows(eo))


@pytest.mark.parametrize("name", ["ssc_tau", "c3_mrk421", "c1_ec1x1", "ssc_tau_2012"])
def test_exact_kernel_bit_parity_in_place_census(name):
    """The in-place census mode (c2d_config.census_inplace) tracks the same
    histories: counters and census records (by key) equal the oracle's."""
    gc = GoldenCase(name)
    eng = Engine(gc.grid(comtot_mode=abi.COMTOT_EXACT, census_inplace=1))
    orc = OL.Oracle(gc.grid(), OL.RNG_LINEAGE, "det")
    for n in range(gc.nsteps):
        si = gc.step_inputs(n)
        eng.transport_step(si)
        assert orc.step(si) == 0
        tg, to = eng.tallies(), orc.split()
        np.testing.assert_array_equal(tg["counters"][list(COUNTERS)], to["counters"][list(COUNTERS)])
        d6g, i5g, kg = eng.census()
        d6o, i5o, ko = orc.census()
        og, oo = np.argsort(kg), np.argsort(ko)
        np.testing.assert_array_equal(kg[og], ko[oo])
        np.testing.assert_array_equal(d6g[og], d6o[oo])
        np.testing.assert_array_equal(i5g[og], i5o[oo])
    eng.close()
    orc.close()


@pytest.mark.parametrize("inplace", [0, 1])
@pytest.mark.parametrize("name", ["c3_mrk421", "c2_32x32"])
def test_exact_kernel_bit_parity_few_waves(monkeypatch, name, inplace):
    """Generation 0 on two workgroups (C2D_BUNDLE_GRID): every wave runs many
    work chunks and refills lanes across chunk boundaries, census chunks of
    later steps included; both census layouts still track the oracle's
    histories bit for bit."""
    monkeypatch.setenv("C2D_BUNDLE_GRID", "2")
    gc = GoldenCase(name)
    eng = Engine(gc.grid(comtot_mode=abi.COMTOT_EXACT, census_inplace=inplace))
    orc = OL.Oracle(gc.grid(), OL.RNG_LINEAGE, "det")
    for n in range(gc.nsteps):
        si = gc.step_inputs(n)
        eng.transport_step(si)
        assert orc.step(si) == 0
        tg, to = eng.tallies(), orc.split()
        np.testing.assert_array_equal(tg["counters"][list(COUNTERS)], to["counters"][list(COUNTERS)])
        for k in TALLY_KEYS:
            ref = np.asarray(to[k])
            scale = max(np.max(np.abs(ref)), 1e-300)
            np.testing.assert_allclose(tg[k], ref, rtol=1e-11, atol=1e-13 * scale, err_msg=k)
        d6g, i5g, kg = eng.census()
        d6o, i5o, ko = orc.census()
        og, oo = np.argsort(kg), np.argsort(ko)
        np.testing.assert_array_equal(kg[og], ko[oo])
        np.testing.assert_array_equal(d6g[og], d6o[oo])
        np.testing.assert_array_equal(i5g[og], i5o[oo])
    eng.close()
    orc.close()


@pytest.mark.parametrize("name", CASES)
def test_fast_kernel_close_to_oracle(name):
    _assert_fast_close(name)


def test_fast_kernel_close_to_oracle_cooperative_scatter(monkeypatch):
    """prod_dense's secondaries with every compb2d first loop resolved by the
    wave and every split3 copy in the hard kernel (test knobs; the exact
    build's bitwise runs are in test_gpu_prod_splits.py)."""
    monkeypatch.setenv("C2D_KN_CAP_ITERS", "0")
    monkeypatch.setenv("C2D_SC_K1_ATTEMPTS", "0")
    _assert_fast_close("prod_dense")


def _assert_fast_close(name):
    for n, eng, orc in _run_pair(name, abi.COMTOT_TABLE):
        tg, to = eng.tallies(), orc.split()
        for c in COUNTERS:
            a, b = tg["counters"][c], to["counters"][c]
            assert abs(a - b) <= 1e-3 * max(abs(b), 1.0) + 2, (name, n, c, a, b)
        for k in ("edep", "ecens", "npcen", "erlko", "erlku", "fout", "edout"):
            a, b = np.sum(tg[k]), np.sum(to[k])
            assert abs(a - b) <= 1e-3 * max(abs(b), 1e-300), (name, n, k, a, b)
        # radiation-pressure deposits (signed: compared against their magnitude);
        # the fast build's point loop uses a series for -log(1-x) and v_rsq_f64
        a, b = np.asarray(tg["prdep"]), np.asarray(to["prdep"])
        assert np.sum(np.abs(a - b)) <= 1e-3 * max(np.sum(np.abs(b)), 1e-300), (name, n, "prdep")
        # every other tally the FP solve and the host driver read: the photon
        # field, the Compton tallies and the boundary leaks, as totals and
        # per cell (relative L2 over the cells; n_field per cell over its 400 bins)
        for k in ("n_field", "E_IC", "nelectron", "erlki", "erlkl", "Ed_in", "erlko", "erlku"):
            a, b = np.sum(tg[k]), np.sum(to[k])
            assert abs(a - b) <= 1e-3 * max(abs(b), 1e-300) + (1e-300 if b == 0 else 0), (name, n, k, a, b)
        for k in ("edep", "ecens", "npcen", "n_field", "E_IC", "nelectron"):
            a, b = np.asarray(tg[k], float).ravel(), np.asarray(to[k], float).ravel()
            nb = np.linalg.norm(b)
            assert np.linalg.norm(a - b) <= 1e-3 * nb + (0.0 if nb > 0 else 1e-300), (name, n, k)
        nfg, nfo = np.asarray(tg["n_field"]), np.asarray(to["n_field"])
        for j in range(nfo.shape[0]):
            for kk in range(nfo.shape[1]):
                nb = np.linalg.norm(nfo[j, kk])
                assert np.linalg.norm(nfg[j, kk] - nfo[j, kk]) <= 1e-3 * nb + (0.0 if nb > 0 else 1e-300), \
                    (name, n, "n_field cell", j, kk)


@pytest.mark.parametrize("fn,lo,hi", [(0, 1e-300, 1e300), (1, -700.0, 700.0), (2, -7.0, 14.0),
                                      (3, -1.0, 1.0), (4, 1e-30, 1e30)])
def test_device_math_bitwise_equals_host(fn, lo, hi):
    rng = np.random.default_rng(fn)
    if fn in (0, 4):
        x = np.exp(rng.uniform(np.log(lo), np.log(hi), 200000))
    else:
        x = rng.uniform(lo, hi, 200000)
    x[:4] = [lo, hi, (lo + hi) / 2, x[4]]
    y = np.zeros_like(x)
    OL.load("det").c2o_unit_math(fn, x.ctypes.data_as(abi.PD), y.ctypes.data_as(abi.PD), x.size)
    yd = device_math(fn, x)
    np.testing.assert_array_equal(yd.view(np.uint64), y.view(np.uint64))


def test_device_branch_free_log_equals_host():
    from test_math_rng import log_pos_inputs
    x = log_pos_inputs()
    y = np.zeros_like(x)
    OL.load("det").c2o_unit_math(0, x.ctypes.data_as(abi.PD), y.ctypes.data_as(abi.PD), x.size)
    yd = device_math(8, x)
    np.testing.assert_array_equal(yd.view(np.uint64), y.view(np.uint64))


def test_device_branch_free_exp_equals_host():
    from test_math_rng import exp_inputs
    x = exp_inputs()
    y = np.zeros_like(x)
    OL.load("det").c2o_unit_math(1, x.ctypes.data_as(abi.PD), y.ctypes.data_as(abi.PD), x.size)
    yd = device_math(9, x)
    np.testing.assert_array_equal(yd.view(np.uint64), y.view(np.uint64))


def test_device_draws_equal_host():
    """Lineage draws (c2d_rng.h c2d_draw): device = host bit for bit."""
    keys = np.array([0, 1, 0x5EEDC2D, 2 ** 53 - 1], np.float64)
    x = np.repeat(keys, 1000)
    yd = device_math(7, x)
    lib = OL.load("det")
    yh = np.array([lib.c2o_unit_philox_draw(int(k), i) for i, k in enumerate(x)])
    np.testing.assert_array_equal(yd, yh)


def test_tridag_matches_reference_semantics():
    rng = np.random.default_rng(3)
    ncell, nt = 37, 200
    a = rng.uniform(-1, 0, (ncell, nt))
    c = rng.uniform(-1, 0, (ncell, nt))
    b = 2.5 + rng.uniform(0, 1, (ncell, nt))
    r = rng.uniform(-0.2, 1, (ncell, nt))
    b[5, 0] = 0.0                     # |b(1)| <= 1e-100: previous x kept
    x0 = np.full((ncell, nt), 7.0)
    from tridag_ref import tridag_ref
    eng = Engine(GoldenCase("ssc_tau").grid())
    x = eng.fp_tridag(a, b, c, r, x0)
    for i in range(ncell):
        np.testing.assert_array_equal(x[i], tridag_ref(a[i], b[i], c[i], r[i], x0[i]))
    eng.close()
