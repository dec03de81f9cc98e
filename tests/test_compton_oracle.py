"""The Compton fixtures (tests/golden/make_compton.py) pinned on the CPU, and
the Compton component of the RNG swap (tests/compton_case.py).

* compton_fib.npz's check run (the reference's algorithm with its own
  lagged-Fibonacci streams, glibc: bit-exact to the Fortran reference,
  tests/test_oracle_golden.py) and one shard of compton_ident.npz (the
  oracle's lineage mode, det math: what the GPU kernels reproduce) are
  recomputed bit for bit.
* The lineage streams + probe bundles (compton_ident: 1e6 sources) against
  the reference streams (compton_fib: R x 1e5 sources): every Compton
  light-curve band and F(E) over the Compton bins agree within 4 sigma of
  the combined statistical error (the lineage side's shard scatter, the
  reference side's run-to-run scatter), printed with the deviations.
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
    fx = np.load(GOLD / "compton_ident.npz", allow_pickle=False)
    fb = _fib()
    R = len(fb["seeds"])
    shards = [CC.summary(t) for t in fx["shard_T"]]
    E_lin = np.sum([s[1] for s in shards], axis=0)
    F_lin = np.sum([s[0] for s in shards], axis=0)
    cnt = np.sum([s[2] for s in shards], axis=0)
    assert cnt[abi.CNT_COLLIDE] >= 1e5 and cnt[abi.CNT_ESC_SCAT] >= 1e6
    E_ref, F_ref = fb["edout"].mean(axis=0), fb["F"].mean(axis=0)
    ns = len(shards)
    sig_lin = np.std([s[1] for s in shards], axis=0, ddof=1) * np.sqrt(ns)
    sig_ref = fb["edout"].std(axis=0, ddof=1) / np.sqrt(R)
    sig = np.hypot(sig_lin, sig_ref) / E_ref
    dev = np.abs(E_lin - E_ref) / E_ref
    # F(E) per Compton bin, chi^2-like: deviations in units of their sigma
    cb = CC.compton_bins()
    sF_lin = np.std([s[0] for s in shards], axis=0, ddof=1) * np.sqrt(ns)
    sF_ref = fb["F"].std(axis=0, ddof=1) / np.sqrt(R)
    sF = np.hypot(sF_lin, sF_ref)
    live = cb[(F_ref[cb] > 0) & (sF[cb] > 0)]
    z = (F_lin[live] - F_ref[live]) / sF[live]
    with capsys.disabled():
        print("\nCompton component, lineage streams + bundles (%d sources, %d collisions) vs reference "
              "streams (%d x %d sources, %d collisions): bands |dev| %s, combined 1-sigma %s; F(E) "
              "Compton bins: rms z %.2f over %d bins, max |z| %.2f" % (
                  int(fx["sources"]), cnt[abi.CNT_COLLIDE], R, int(fb["sources"]),
                  fb["counters"][:, abi.CNT_COLLIDE].sum(), np.round(dev, 4).tolist(),
                  np.round(sig, 4).tolist(), float(np.sqrt(np.mean(z ** 2))), len(live),
                  float(np.abs(z).max())))
    for i in CC.COMPTON_BANDS:
        assert dev[i] <= 4.0 * sig[i], (i, dev[i], sig[i])
    assert np.sqrt(np.mean(z ** 2)) <= 1.5, z
    # collision rates per source agree to their Poisson error
    c_ref = fb["counters"][:, abi.CNT_COLLIDE].sum() / (R * float(fb["sources"]))
    c_lin = cnt[abi.CNT_COLLIDE] / float(fx["sources"])
    assert abs(c_lin - c_ref) <= 4.0 * np.sqrt(cnt[abi.CNT_COLLIDE]) / float(fx["sources"]) + 1e-12
