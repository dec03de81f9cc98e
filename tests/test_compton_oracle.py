"""The Compton fixtures (tests/golden/make_compton.py) pinned on the CPU, and
the Compton component of the RNG swap (tests/compton_case.py).

* compton_fib.npz's check run (the reference's algorithm with its own
  lagged-Fibonacci streams, glibc: bit-exact to the Fortran reference,
  tests/test_oracle_golden.py) and one shard of compton_ident.npz (the
  oracle's lineage mode, det math: what the GPU kernels reproduce) are
  recomputed bit for bit.
* The lineage streams, with probe bundles and with per-copy probes
  (compton_lin: 256 runs each), against the reference streams (compton_fib:
  5000 runs), all runs of 1e5 sources: a chi^2 over the Compton bins of F(E)
  and a z per Compton light-curve band from run-to-run variances, printed.
"""
from multiprocessing import get_context
from pathlib import Path

import numpy as np
import pytest

import compton_case as CC
import oracle_lib as OL
from compton2d_amd import abi

GOLD = Path(__file__).resolve().parent / "golden"


def _fib():
    p = GOLD / "compton_fib.npz"
    if not p.exists():
        pytest.skip("compton_fib.npz not generated yet (tests/golden/make_compton.py)")
    return np.load(p, allow_pickle=False)


def test_compton_fixtures_recompute_bitwise():
    OL.build()
    fx = np.load(GOLD / "compton_ident.npz", allow_pickle=False)
    fb = _fib()
    jobs = [("lineage", int(fx["seed"]), int(fx["sources"]), 3, int(fx["shards"]), "det"),
            ("fib", int(fb["check_seed"]), int(fb["check_sources"]))]
    with get_context("spawn").Pool(2) as pool:
        t_lin, t_fib = pool.map(CC.oracle_run, jobs)
    np.testing.assert_array_equal(t_lin, fx["shard_T"][3])
    np.testing.assert_array_equal(t_fib, fb["check_T"])
    np.testing.assert_array_equal(np.sum(fx["shard_T"], axis=0), fx["T"])


def test_lineage_streams_compton_component_vs_reference_streams(capsys):
    """The lineage streams with probe bundles (the GPU's algorithm), and with
    per-copy probes, against the reference's algorithm on its own streams:
    compton_lin.npz's 256 + 256 lineage runs and compton_fib.npz's 5000
    lagged-Fibonacci runs, all of FIB_SOURCES sources, every error from
    run-to-run scatter (CC.compare_runs).  Three pairs separate the RNG swap
    (per-copy vs fib) from the superposition (bundles vs per-copy).  Each:
    chi^2 p-value over the Compton bins of F(E) > 1e-3, rms z <= 1.2, no bin
    beyond its permutation null's 99.9 % (CC.perm_max_z: the top tail bins are
    too skewed for a normal bar at 256 runs), every Compton band within 4 sigma, rel L2 of F(E)
    within the 99.9 % quantile of its sampling distribution; collision rates
    within 4 sigma.  (Round 3 used 8 lineage shards for the lineage sigma:
    rms z 1.42 was that estimator's noise.)"""
    fb = _fib()
    L = np.load(GOLD / "compton_lin.npz", allow_pickle=False)
    assert int(L["sources"]) == int(fb["sources"])
    sides = {"bundles": (L["bundle_F"], L["bundle_edout"], L["bundle_counters"]),
             "per-copy": (L["copy_F"], L["copy_edout"], L["copy_counters"]),
             "fib": (fb["F"], fb["edout"], fb["counters"])}
    res = {}
    for a, b in (("bundles", "fib"), ("per-copy", "fib"), ("bundles", "per-copy")):
        res[a + " vs " + b] = CC.compare_runs(sides[a][0], sides[a][1], sides[b][0], sides[b][1])
    with capsys.disabled():
        for k, d in res.items():
            print("\nCompton component, %s (%d vs %d runs of %d sources): %s" % (
                k, len(sides[k.split(" vs ")[0]][0]), len(sides[k.split(" vs ")[1]][0]),
                int(fb["sources"]), {q: (np.round(v, 4).tolist() if isinstance(v, (float, list)) else v)
                                     for q, v in d.items()}))
    for k, d in res.items():
        assert d["p_value"] > 1e-3, (k, d)
        assert d["rms_z"] <= 1.2, (k, d)
        # the largest bin |z| against its permutation null (CC.perm_max_z):
        # runs of one size on both sides, so they are exchangeable
        a, b = k.split(" vs ")
        zmax, p_perm, q999 = CC.perm_max_z(sides[a][0], sides[b][0])
        with capsys.disabled():
            print("%s: max |z| %.2f, permutation p %.4f (99.9 %% quantile %.2f)" % (k, zmax, p_perm, q999))
        assert p_perm > 1e-3, (k, zmax, p_perm, q999)
        for i in CC.COMPTON_BANDS:
            assert abs(d["band_z"][i]) <= 4.0, (k, i, d)
        assert d["rel_l2"] <= d["rel_l2_bound_999"], (k, d)
    # collision rates per source agree to their run-to-run error
    for a, b in (("bundles", "fib"), ("per-copy", "fib")):
        ca, cb_ = sides[a][2][:, abi.CNT_COLLIDE], sides[b][2][:, abi.CNT_COLLIDE]
        se = np.sqrt(ca.var(ddof=1) / len(ca) + cb_.var(ddof=1) / len(cb_))
        assert abs(ca.mean() - cb_.mean()) <= 4.0 * se, (a, b, ca.mean(), cb_.mean(), se)


def test_compton_lin_fixture_recomputes_bitwise():
    """One run of each probe mode of compton_lin.npz recomputed by the oracle."""
    import os
    L = np.load(GOLD / "compton_lin.npz", allow_pickle=False)
    for bundles, tag in ((1, "bundle"), (0, "copy")):
        os.environ["C2O_PROBE_BUNDLES"] = str(bundles)
        try:
            with get_context("spawn").Pool(1) as pool:
                T = pool.map(CC.oracle_run, [("lineage", int(L["seeds"][3]), int(L["sources"]), 0, 1, "ref")])[0]
        finally:
            os.environ.pop("C2O_PROBE_BUNDLES", None)
        F, E, cnt = CC.summary(T)
        np.testing.assert_array_equal(F, L[tag + "_F"][3])
        np.testing.assert_array_equal(E, L[tag + "_edout"][3])
