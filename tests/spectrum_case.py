"""The north-star spectrum workload (SURVEY.md §8(d) parity metric) —
TEST INFRASTRUCTURE.  The thin inputm.dat medium (compton2d_amd/synth.py) on
2x2 zones, one MC step with ncycle = 1 and dt = 30 x the C2 step, so that
nearly every packet escapes within the step: 2e6 volume packets give ~1.9e6
escape events.  F(E)'s L2 norm is carried by the self-absorbed low-energy
bins (70 % in the first), whose per-bin scatter is ~1.6 % at 2.5e5 packets
for either generator, so the reference side is 3 seeds x 2e6 packets and the
lineage side 1e7.  F(E) = fout / dE over the spb.dat bins
(src/graphics2d.f:140-160) and the light curves edout (lcb_NN.dat)."""
from __future__ import annotations

import numpy as np

from compton2d_amd import abi, synth

SOURCES = 2_000_000                  # per reference (fib) run: ~1.9e6 escapes
LINEAGE_SOURCES = 10_000_000         # the lineage-stream run: ~9.5e6 escapes
FIB_SEEDS = (9857, 24680, 13579)
LINEAGE_SEED = 0x5EEDC2D
SHARDS = 8                           # the lineage run in 8 lineage shards
DT_FACTOR = 30.0


def workload(mode=abi.COMTOT_EXACT, seed=LINEAGE_SEED, rank=0, world=1, n=SOURCES, device=0):
    wl = synth.c2_workload(nz=2, nr=2, sources=n, comtot_mode=mode, census_capacity=n // 4 + 4096,
                           event_capacity=2 * n + 4096, seed=seed, rank=rank, world=world,
                           device=device)
    wl.grid.kappa_lag = 0
    si = wl.step0
    si.ncycle = 1
    si.dt = si.dt * DT_FACTOR
    return wl.grid, si


def f_of_e(fout):
    de = np.diff(synth.photon_grid())
    return np.asarray(fout)[..., :de.size].sum(axis=0) / de


def band_errors(edout_fib, edout_shards):
    """Relative 1-sigma statistical error of each light-curve band of the
    fib mean (seed scatter / sqrt(seeds)) and of the lineage shard sum
    (shard scatter * sqrt(shards)), combined."""
    f, sh = np.asarray(edout_fib, float), np.asarray(edout_shards, float)
    m, tot = f.mean(axis=0), sh.sum(axis=0)
    with np.errstate(invalid="ignore", divide="ignore"):
        sd_f = f.std(axis=0, ddof=1) / np.sqrt(f.shape[0]) / m
        sd_l = sh.std(axis=0, ddof=1) * np.sqrt(sh.shape[0]) / tot
    return np.hypot(sd_f, sd_l)


def rel_l2(a, b):
    a, b = np.asarray(a, float).ravel(), np.asarray(b, float).ravel()
    s = max(np.abs(a).max(), np.abs(b).max())
    m = (np.abs(a) > 1e-20 * s) | (np.abs(b) > 1e-20 * s)
    return float(np.linalg.norm(a[m] - b[m]) / np.linalg.norm(b[m]))


def oracle_run(args):
    """(F(E), edout, escapes) of one oracle run: ('fib', seed) with the
    reference's lagged-Fibonacci zone streams, or ('lineage', seed, rank, world)
    with the engine's counter-based lineage streams on a shard of the sources."""
    import oracle_lib as OL
    kind, seed = args[0], args[1]
    rank, world = (args[2], args[3]) if kind == "lineage" else (0, 1)
    n = LINEAGE_SOURCES if kind == "lineage" else SOURCES
    grid, si = workload(seed=seed, rank=rank, world=world, n=n)
    o = OL.Oracle(grid, OL.RNG_FIB if kind == "fib" else OL.RNG_LINEAGE, "ref", rseed=seed)
    assert o.step(si) == 0
    t = o.split()
    o.close()
    return (f_of_e(t["fout"]), np.asarray(t["edout"]).ravel().copy(),
            float(t["counters"][abi.CNT_ESCAPES]))
