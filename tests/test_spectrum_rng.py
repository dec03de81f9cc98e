"""North-star spectrum criterion on the CPU: <= 1 % relative
L2 on F(E) of spb.dat between the reference's algorithm with the reference's
own lagged-Fibonacci streams (C oracle, glibc, rand_switch = 1: bit-exact to
the Fortran reference, tests/test_oracle_golden.py) and the same algorithm
with the engine's per-packet lineage streams (SplitMix64 draw streams whose
keys are derived with Philox, csrc/c2d_rng.h) — the RNG swap the GPU makes — with the reference's own seed-to-seed floor reported beside it.
Reference side: 3 seeds x ~1.9e6 escapes, averaged; lineage side: ~9.5e6
escapes (tests/spectrum_case.py).  Same for the light curves (edout).

The three fib runs are recomputed here and must equal the committed fixture
(tests/golden/spectrum_fib.npz, which the GPU test compares the fast kernel
against) bit for bit; the lineage run is sharded over processes by source
lineage (sums are the single-process run's to rounding).
"""
import itertools
from multiprocessing import get_context
from pathlib import Path

import numpy as np

import oracle_lib as OL
import spectrum_case as S

FIX = Path(__file__).resolve().parent / "golden" / "spectrum_fib.npz"
SHARDS = S.SHARDS


def test_lineage_rng_spectrum_within_1pct_of_reference_streams(capsys):
    OL.build()
    jobs = [("fib", s) for s in S.FIB_SEEDS] + [("lineage", S.LINEAGE_SEED, r, SHARDS)
                                                for r in range(SHARDS)]
    with get_context("spawn").Pool(8) as pool:
        res = pool.map(S.oracle_run, jobs)
    fib, lin = res[:3], res[3:]
    fx = np.load(FIX, allow_pickle=False)
    for i, r in enumerate(fib):                       # the fixture is this computation
        np.testing.assert_array_equal(r[0], fx["F"][i])
        np.testing.assert_array_equal(r[1], fx["edout"][i])
    for i, r in enumerate(lin):
        np.testing.assert_array_equal(r[1], fx["lineage_edout_shards"][i])
    # the lineage run: the per-packet streams scale the weights by 1/(sources)
    # through ewsv, so the sharded sum is F(E) of 1e7 packets at the same
    # normalisation as one 2e6-packet reference run
    F_lin = sum(r[0] for r in lin)
    E_lin = sum(r[1] for r in lin)
    esc_lin = sum(r[2] for r in lin)
    F_ref = np.mean([r[0] for r in fib], axis=0)
    E_ref = np.mean([r[1] for r in fib], axis=0)
    assert min(r[2] for r in fib) >= 1.0e6 and esc_lin >= 5.0e6
    cross = S.rel_l2(F_lin, F_ref)
    floor = [S.rel_l2(a[0], b[0]) for a, b in itertools.combinations(fib, 2)]
    # light curves per band (lcb_01.dat columns).  Each band's statistical
    # error is estimated from both sides: the reference's seed-to-seed
    # scatter (3 runs) and the lineage run's shard-to-shard scatter (8 shards
    # of 1.25e6 sources).  A band this sample resolves to the north-star
    # bound (4 sigma <= 1 %: the synchrotron band 0, carried by the
    # unscattered copies) must agree to 1 %.  The bands that rare Compton
    # events reach (~3 collisions per 1e6 packets in this thin medium, each
    # handing split2 x split3 secondaries a large gain; sigma 0.6-96 %) are
    # not asserted here: tests/test_gpu_compton.py pins every Compton band on
    # the Compton workload (n_e x 5e4, thousands of reference-stream runs)
    # to an explicit bound of at most 5 %.
    E_all = np.array([r[1] for r in fib])
    sig_b = S.band_errors(E_all, [r[1] for r in lin])
    bands = [i for i in range(E_all.shape[1]) if E_all[:, i].min() > 0]
    lc = []
    for i in bands:
        dev = abs(E_lin[i] - E_ref[i]) / E_ref[i]
        lc.append((i, dev, float(sig_b[i])))
    with capsys.disabled():
        print("\nF(E) rel L2, lineage (%.3g escapes) vs reference streams (3 x %.3g): %.4f; "
              "reference seed-to-seed floor (pairs of %.3g): %s" % (
                  esc_lin, fib[0][2], cross, fib[0][2], ["%.4f" % x for x in floor]))
        print("light curves per band (band, |dev|, combined 1-sigma error): %s" %
              ["(%d, %.4f, %.4f)" % x for x in lc])
    assert cross <= 1.0e-2, cross
    resolved = [(i, dev, sig) for i, dev, sig in lc if 4.0 * sig <= 1.0e-2]
    assert resolved and resolved[0][0] == 0              # the first synchrotron band
    for i, dev, sig in resolved:
        assert dev <= 1.0e-2, (i, dev, sig)
    # no bias beyond the noise: the larger-sample comparison is no further
    # apart than two reference runs of 2e6 packets are from each other
    assert cross <= max(floor), (cross, floor)
