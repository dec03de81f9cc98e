"""The Compton spectrum workload (SURVEY.md §8(d) parity metric on the
scattered component) — TEST INFRASTRUCTURE.

The north-star spectrum workload (tests/spectrum_case.py: the inputm.dat
medium of C3 on 2x2 zones, one MC step with ncycle = 1 and dt = 30 x the C2
step) with the electron density scaled by N_E_FACTOR = 5e4 (n_e = 4e6 cm^-3,
the `ssc_tau` golden case's density): the Thomson depth of the blob rises to
~0.02, so a source makes ~0.14 collisions (split1 = 10 probes), every
collision hands split2 = 10 secondaries a Klein-Nishina sample of the
power-law electrons (gmin 1e2 .. gmax 1e5, p = 2.3, src/compb_2d.f:1-318),
and gains above split1*split2*spl3_trg = 1000 trigger split3 resampling
(src/imctrk2d.f:580-684).  Above COMPTON_E_MIN = 1e-3 keV more than 87 % of
F(E) is carried by scattered packets (measured with n_e -> 0: tests/
golden/make_compton.py prints the unscattered share per bin), so the bins and
light-curve bands above it pin the scattered component:
LC bands 1..4 = (1e-3,1), (1,1e2), (1e2,1e5), (1e5,1e9) keV.

The band energies are heavy-tailed (a gain of up to ~gamma^2 = 1e10 per
scattering off the p = 2.3 tail): a run of 2e4 sources has a relative
seed-to-seed scatter of 6 %, 30 %, 40 % and 68 % in bands 1..4, so the
reference-stream side of a 1 % comparison needs ~1e8 sources
(tests/golden/compton_fib.npz); the identical-seed comparison (same lineage
streams on both sides) does not: it is per history.
"""
from __future__ import annotations

import numpy as np

import spectrum_case as S
from compton2d_amd import abi, synth

N_E_FACTOR = 5.0e4
COMPTON_E_MIN = 1.0e-3                # keV: lower edge of the first Compton bin/band
COMPTON_BANDS = (1, 2, 3, 4)          # lcb_01.dat columns carried by scattered packets
LINEAGE_SEED = 0x5EEDC2D
IDENT_SOURCES = 1_000_000             # identical-seed fixture (oracle lineage, det math)
IDENT_SHARDS = 8
FIB_SOURCES = 100_000                 # per reference-stream (fib) run
FIB_CHECK_SOURCES = 20_000            # the run the CPU test recomputes bit for bit
FIB_SEED0 = 10007


def fib_seed(k: int) -> int:
    """rseed of the k-th reference-stream run (distinct lagged-Fibonacci streams)."""
    return FIB_SEED0 + 7919 * k


def lin_seed(k: int) -> int:
    """Lineage seed of the k-th lineage-stream run (tests/golden/compton_lin.npz)."""
    return LINEAGE_SEED + 104729 * (k + 1)


def workload(mode=abi.COMTOT_EXACT, seed=LINEAGE_SEED, rank=0, world=1, n=IDENT_SOURCES, device=0,
             queue_capacity=None):
    grid, si = S.workload(mode=mode, seed=seed, rank=rank, world=world, n=n, device=device)
    si.n_e = si.n_e * N_E_FACTOR
    # collisions: ~0.15 per source; a generation can hold ~1.3 third-split records
    # per collision (split2 = 10 copies, gains above 1000 are common)
    per = int(np.ceil(n / world))
    grid.queue_capacity = queue_capacity or max(1 << 20, 4 * per)
    grid.census_capacity = max(grid.census_capacity, per // 2 + 4096)
    grid.event_capacity = max(grid.event_capacity, 8 * per + 4096)
    return grid, si


def compton_bins() -> np.ndarray:
    """Indices of the spb.dat bins whose lower edge is >= COMPTON_E_MIN."""
    hu = synth.photon_grid()
    return np.nonzero(hu[:-1] >= COMPTON_E_MIN * (1 - 1e-12))[0]


def oracle_run(args):
    """One oracle run of the Compton workload: ('fib', seed, n) with the
    reference's lagged-Fibonacci streams (glibc: bit-exact to the Fortran),
    or ('lineage', seed, n, rank, world, flavor) with the engine's lineage
    streams on a shard of the sources.  Returns the full tally vector."""
    import oracle_lib as OL
    kind, seed, n = args[0], args[1], args[2]
    if kind == "fib":
        grid, si = workload(seed=seed, n=n)
        o = OL.Oracle(grid, OL.RNG_FIB, "ref", rseed=seed)
    else:
        rank, world, flavor = args[3], args[4], args[5]
        grid, si = workload(seed=seed, rank=rank, world=world, n=n)
        o = OL.Oracle(grid, OL.RNG_LINEAGE, flavor)
    rc = o.step(si)
    t = o.tallies()
    o.close()
    if rc != 0:
        raise RuntimeError("oracle run %r failed: %d" % (args, rc))
    return t


def summary(tallies, nz=2, nr=2, nmu=1):
    """(F(E), edout, counters) of a tally vector."""
    t = abi.split_tallies(np.asarray(tallies), nz, nr, nmu)
    return S.f_of_e(t["fout"]), np.asarray(t["edout"]).ravel()[:5].copy(), np.asarray(t["counters"])


def perm_max_z(FA, FB, nperm=2000, seed=1):
    """Permutation null of the largest per-bin |z| of compare_runs over the
    Compton bins, for two sets of runs of the same size (so that, under the
    hypothesis that both draw from one distribution, the runs are
    exchangeable): the runs pooled and re-split nperm times.  The normal
    theory behind a fixed bar fails in the top tail bins, whose per-run values
    are rare large events (skewness 8-40 at 1e5 sources per run: a 256-run
    mean there is not normal).  Returns (observed max |z|, p-value, the
    99.9 % quantile of the permutation maxima)."""
    cb = compton_bins()
    FA, FB = np.asarray(FA, float)[:, cb], np.asarray(FB, float)[:, cb]
    live = FB.mean(axis=0) > 0
    FA, FB = FA[:, live], FB[:, live]

    def mz(a, b):
        s = np.sqrt(a.var(axis=0, ddof=1) / len(a) + b.var(axis=0, ddof=1) / len(b))
        return float(np.max(np.abs(a.mean(axis=0) - b.mean(axis=0)) / np.where(s > 0, s, np.inf)))

    obs = mz(FA, FB)
    X = np.vstack([FA, FB])
    rng = np.random.default_rng(seed)
    ms = np.empty(nperm)
    for k in range(nperm):
        pi = rng.permutation(len(X))
        ms[k] = mz(X[pi[:len(FA)]], X[pi[len(FA):]])
    return obs, float((1 + np.sum(ms >= obs)) / (1 + nperm)), float(np.quantile(ms, 0.999))


def compare_runs(FA, EA, FB, EB):
    """Two sets of independent runs of the Compton workload (per-run F(E)
    [runs, bins] and light-curve bands [runs, 5]; each side's runs i.i.d.),
    compared with run-to-run variances (not shard estimates): per Compton bin
    z = (mean_A - mean_B) / sqrt(s_A^2/n_A + s_B^2/n_B), its chi^2 and p-value,
    the bands' z, and the rel L2 of the mean F(E) over the Compton bins beside
    the rel L2 two unbiased estimates of these sizes are expected to show."""
    from scipy import stats
    FA, FB, EA, EB = (np.asarray(x, float) for x in (FA, FB, EA, EB))
    cb = compton_bins()
    mA, mB = FA.mean(axis=0), FB.mean(axis=0)
    vA = FA.var(axis=0, ddof=1) / len(FA)
    vB = FB.var(axis=0, ddof=1) / len(FB)
    s = np.sqrt(vA + vB)
    live = cb[(mB[cb] > 0) & (s[cb] > 0)]
    z = (mA[live] - mB[live]) / s[live]
    chi2 = float(np.sum(z ** 2))
    eA, eB = EA.mean(axis=0), EB.mean(axis=0)
    se = np.sqrt(EA.var(axis=0, ddof=1) / len(EA) + EB.var(axis=0, ddof=1) / len(EB))
    zb = np.where(se > 0, (eA - eB) / np.where(se > 0, se, 1.0), 0.0)
    rel = float(np.linalg.norm(mA[cb] - mB[cb]) / np.linalg.norm(mB[cb]))
    v = vA[cb] + vB[cb]
    rel_exp = float(np.sqrt(np.sum(v)) / np.linalg.norm(mB[cb]))
    # rel^2 is a variance-weighted sum of squared normals: ~ chi^2 with nu
    # effective degrees of freedom (a few bins carry most of the variance)
    nu = float(np.sum(v) ** 2 / np.sum(v ** 2))
    return {"rel_l2_bound_999": rel_exp * float(np.sqrt(stats.chi2.ppf(0.999, nu) / nu)), "nu": nu,
            "bins": int(len(live)), "rms_z": float(np.sqrt(np.mean(z ** 2))),
            "max_abs_z": float(np.abs(z).max()), "chi2": chi2,
            "p_value": float(stats.chi2.sf(chi2, len(live))),
            "bins_over_4sigma": [int(b) for b in live[np.abs(z) > 4.0]],
            "band_z": [float(x) for x in zb],
            "band_rel_dev": [float((a - b) / b) if b > 0 else 0.0 for a, b in zip(eA, eB)],
            "band_rel_sigma": [float(x / b) if b > 0 else 0.0 for x, b in zip(se, eB)],
            "rel_l2": rel, "rel_l2_expected": rel_exp}
