"""North-star spectrum criterion: the escaping spectrum F(E)
of the production (fast) GPU kernel against the reference CPU path on identical
inputs and seeds, relative L2 over the spb.dat bins (src/graphics2d.f:140-160:
F(E) = fout / dE) <= 1 %.

"Reference CPU path on identical seeds" = the C oracle (oracle/c2d_oracle.c:
the reference's algorithm, glibc libm, pinned bit-exactly to the Fortran
reference in tests/test_oracle_golden.py) drawing the same per-packet counter-based
streams as the GPU.  The only differences left are the fast kernel's tabulated
comtot (< 1e-7 relative) and FMA-free vs libm rounding, which flip a handful of
collision/census decisions: the measured deviation is orders of magnitude
below the 1 % bound (and below the seed-to-seed noise; see
tests/test_spectrum_rng.py for the RNG swap against the reference's own
lagged-Fibonacci streams).
"""
import numpy as np
import pytest

import oracle_lib as OL
from compton2d_amd import abi, synth
from compton2d_amd.engine import Engine

pytestmark = pytest.mark.gpu


def f_of_e(fout):
    hu = synth.photon_grid()
    de = np.diff(hu)
    return np.asarray(fout)[..., :de.size].sum(axis=0) / de


def rel_l2(a, b):
    s = max(np.abs(a).max(), np.abs(b).max())
    m = (np.abs(a) > 1e-20 * s) | (np.abs(b) > 1e-20 * s)
    return float(np.linalg.norm(a[m] - b[m]) / np.linalg.norm(b[m]))


@pytest.mark.parametrize("kappa_lag", [0, 1])
def test_fast_kernel_spectrum_within_1pct_of_reference_cpu_path(kappa_lag):
    n = 200_000
    wl = synth.c2_workload(nz=3, nr=3, sources=n, comtot_mode=abi.COMTOT_TABLE,
                           census_capacity=4 * n, event_capacity=4 * n)
    wl.grid.kappa_lag = kappa_lag
    si = wl.step0
    si.ncycle = 1                     # escapes are tallied for ncycle > 0
    eng = Engine(wl.grid)
    eng.transport_step(si)
    tg = eng.tallies()
    eng.close()
    g = synth.c2_workload(nz=3, nr=3, sources=n, comtot_mode=abi.COMTOT_EXACT,
                          census_capacity=4 * n, event_capacity=4 * n).grid
    g.kappa_lag = kappa_lag
    o = OL.Oracle(g, OL.RNG_LINEAGE, "ref")
    assert o.step(si) == 0
    to = o.split()
    o.close()
    esc = to["counters"][abi.CNT_ESCAPES]
    assert esc > 20_000
    d = rel_l2(f_of_e(tg["fout"]), f_of_e(to["fout"]))
    print("kappa_lag=%d escapes=%d F(E) rel L2 GPU vs reference CPU path: %.3g" % (kappa_lag, esc, d))
    assert d <= 1e-2, d
    # light curves (lcb_NN.dat, src/graphics2d.f:170-200) and the census energy too
    assert rel_l2(tg["edout"].ravel(), to["edout"].ravel()) <= 1e-2
    assert abs(tg["ecens"].sum() - to["ecens"].sum()) <= 1e-2 * to["ecens"].sum()


def test_fast_kernel_spectrum_vs_reference_stream_fixture():
    """The production kernel (tabulated comtot, counter-based lineage streams) on the
    north-star spectrum workload (tests/spectrum_case.py, 1e7 packets: ~9.5e6
    escapes) against the reference algorithm WITH the reference's own
    lagged-Fibonacci streams (tests/golden/spectrum_fib.npz: 3 seeds x 1.9e6
    escapes, C oracle bit-exact to the Fortran, regenerated and checked in
    tests/test_spectrum_rng.py): F(E) relative L2 <= 1 %; each light-curve
    band the fixture resolves to 4 sigma <= 1 % of the combined statistical
    error (reference seed scatter and the lineage run's shard scatter) to 1 %:
    the synchrotron band 0.  The Compton bands, which 3 reference seeds of this
    thin medium leave at 0.6-96 % sigma, are pinned to <= 5 % bounds by
    tests/test_gpu_compton.py on the Compton workload."""
    from pathlib import Path
    import spectrum_case as S
    fx = np.load(Path(__file__).resolve().parent / "golden" / "spectrum_fib.npz", allow_pickle=False)
    grid, si = S.workload(mode=abi.COMTOT_TABLE, n=S.LINEAGE_SOURCES)
    eng = Engine(grid)
    eng.transport_step(si)
    t = eng.tallies()
    eng.close()
    assert t["counters"][abi.CNT_ESCAPES] >= 5e6 and t["counters"][abi.CNT_ABORTED] == 0
    F_ref = fx["F"].mean(axis=0)
    d = S.rel_l2(S.f_of_e(t["fout"]), F_ref)
    floor = [S.rel_l2(fx["F"][a], fx["F"][b]) for a, b in ((0, 1), (0, 2), (1, 2))]
    print("F(E) rel L2 fast kernel (%.3g escapes) vs reference streams: %.4f (reference floor %s)" % (
        t["counters"][abi.CNT_ESCAPES], d, floor))
    assert d <= 1e-2, d
    E = np.asarray(t["edout"]).ravel()
    E_ref = fx["edout"].mean(axis=0)
    sig = S.band_errors(fx["edout"], fx["lineage_edout_shards"])
    bands = [i for i in range(E_ref.size) if fx["edout"][:, i].min() > 0 and 4.0 * sig[i] <= 1e-2]
    assert bands and bands[0] == 0
    for i in bands:
        assert abs(E[i] - E_ref[i]) <= 1e-2 * E_ref[i], (i, E[i], E_ref[i], sig[i])
