"""Probe bundles vs per-copy tracking of the split1 probes, in a
collision-rich medium (CPU, the C oracle).

The lineage mode of the oracle (and the GPU kernels, bit for bit) tracks the
split1 probe copies of a source as bundles: one shared path, the first
collision among the n probes drawn from an exponential of rate n*sigsc, the
collider chosen uniformly, the others continuing (memorylessness).  That is
the same stochastic process as the reference's per-copy tracking
(src/imctrk2d.f:106-123, a fresh colmfp per copy and packet-step), with other
random numbers.  The statistical reference is the oracle's lineage mode with
C2O_PROBE_BUNDLES=0: the reference's per-copy loop (flight_loop with s = -1, a
fresh colmfp per copy and packet-step) on the same lineage stream family, streams
(source key, 1 + probe).

Workload: the golden 'ssc_tau' step (2x2 zones, n_e = 4e6, ~4 collisions per
100 sources, split2/split3 secondaries, census, escapes) with 200x its packets
(2e5 sources per run, weights scaled by 1/200), 8 seeds per side.  Every
counter and tally total must agree within 4 sigma of the combined seed-to-seed
error of the two sides.
"""
import os
from multiprocessing import get_context

import numpy as np

import oracle_lib as OL
from compton2d_amd import abi
from golden_io import GoldenCase

SCALE = 200
SEEDS = (9857, 24680, 13579, 4242, 777, 31337, 1001, 55555)
COUNTERS = ("CNT_STEPS", "CNT_COLLIDE", "CNT_COMPB", "CNT_CENSUS", "CNT_ESCAPES", "CNT_KILLED")
SUMS = ("edep", "prdep", "ecens", "npcen", "E_IC", "fout", "edout", "erlki", "erlko", "erlku",
        "erlkl", "n_field")


def _run(args):
    kind, seed = args
    os.environ["C2O_PROBE_BUNDLES"] = "1" if kind == "bundles" else "0"
    gc = GoldenCase("ssc_tau")
    si = gc.step_inputs(0)
    si.nsv = np.asarray(si.nsv) * SCALE
    si.ewsv = np.asarray(si.ewsv) / SCALE
    g = gc.grid()
    g.seed = seed                       # the lineage streams' root key
    g.census_capacity = int(si.nsv.sum()) * 4 + 4096
    g.event_capacity = int(si.nsv.sum()) * 4 + 4096
    o = OL.Oracle(g, OL.RNG_FIB if kind == "fib" else OL.RNG_LINEAGE, "ref", rseed=seed)
    assert o.step(si) == 0
    t = o.split()
    o.close()
    c = t["counters"]
    out = {k: float(c[getattr(abi, k)]) for k in COUNTERS}
    out.update({k: float(np.sum(t[k])) for k in SUMS})
    return out


def _compare(A, B, label, capsys):
    rows = []
    for k in COUNTERS + SUMS:
        a = np.array([r[k] for r in A])
        b = np.array([r[k] for r in B])
        if a.mean() == 0.0 and b.mean() == 0.0:
            continue
        sig = np.hypot(a.std(ddof=1), b.std(ddof=1)) / np.sqrt(len(SEEDS))
        z = abs(b.mean() - a.mean()) / sig if sig > 0 else 0.0
        rows.append((k, a.mean(), b.mean(), (b.mean() - a.mean()) / a.mean(), z))
    with capsys.disabled():
        print("\n%s, %d seeds each:" % (label, len(SEEDS)))
        for k, ma, mb, rel, z in rows:
            print("  %-12s %.6e %.6e  rel %+.4f  z %.2f" % (k, ma, mb, rel, z))
    for k, ma, mb, rel, z in rows:
        assert z <= 4.0, (label, k, ma, mb, rel, z)


def test_probe_bundles_match_per_copy_tracking_statistically(capsys):
    """Bundles vs per-copy probes on the lineage streams, and vs the
    reference's own algorithm on its own lagged-Fibonacci streams (fib mode,
    rand_switch = 1)."""
    OL.build()
    jobs = [(k, s) for k in ("per_copy", "bundles", "fib") for s in SEEDS]
    with get_context("spawn").Pool(8) as pool:
        res = pool.map(_run, jobs)
    n = len(SEEDS)
    per_copy, bundles, fib = res[:n], res[n:2 * n], res[2 * n:]
    assert np.mean([r["CNT_COLLIDE"] for r in per_copy]) > 5000      # collision-rich
    # independent samples (different lineage roots / fib seeds)
    assert len({r["CNT_STEPS"] for r in bundles}) == n and len({r["CNT_STEPS"] for r in fib}) == n
    _compare(per_copy, bundles, "per-copy probes vs probe bundles (lineage streams)", capsys)
    _compare(fib, bundles, "reference algorithm + streams (fib) vs probe bundles (lineage)", capsys)
