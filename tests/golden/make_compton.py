"""tests/golden/compton_ident.npz and tests/golden/compton_fib.npz: the
Compton spectrum workload (tests/compton_case.py) on the CPU oracle.

* compton_ident.npz — the oracle's lineage mode with the engine's det math
  (the GPU's streams and probe bundles), IDENT_SOURCES sources in
  IDENT_SHARDS lineage shards, full tally vector summed over the shards: the
  identical-seed reference the production GPU kernel is compared with
  (tests/test_gpu_compton.py).  Also the unscattered share of F(E) per bin
  (the same run with n_e -> 0), which locates COMPTON_E_MIN.
* compton_fib.npz — the reference's algorithm with the reference's own
  lagged-Fibonacci streams (glibc: bit-exact to the Fortran reference,
  tests/test_oracle_golden.py), R runs of FIB_SOURCES sources with distinct
  rseeds: per-run F(E), light curves and counters.  Their mean is the
  reference-stream spectrum, their scatter its statistical error.  One extra
  run of FIB_CHECK_SOURCES (full tallies) is recomputed bit for bit by
  tests/test_compton_oracle.py.

Runs are cached per run under --work, so an interrupted generation resumes.

usage: python tests/golden/make_compton.py [--runs R] [--procs P] [--work DIR] [--only ident|fib]
"""
import argparse
import sys
import time
from multiprocessing import get_context
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
sys.path[:0] = [str(HERE.parents[1]), str(HERE.parent)]


def _fib_job(args):
    k, seed, n, work = args
    out = Path(work) / ("fib_%05d.npy" % k)
    if out.exists():
        return k, np.load(out)
    import compton_case as CC
    t0 = time.time()
    T = CC.oracle_run(("fib", seed, n))
    F, E, cnt = CC.summary(T)
    rec = np.concatenate([F, E, cnt, [time.time() - t0]])
    np.save(out, rec)
    return k, rec


def _lin_job(args):
    import compton_case as CC
    return CC.oracle_run(args)


def _nocomp_job(args):
    import compton_case as CC
    import oracle_lib as OL
    seed, n = args
    grid, si = CC.workload(seed=seed, n=n)
    si.n_e = si.n_e / CC.N_E_FACTOR * 1e-8        # n_e -> 0: no scattering
    o = OL.Oracle(grid, OL.RNG_LINEAGE, "ref")
    assert o.step(si) == 0
    t = o.tallies()
    o.close()
    return t


def make_ident(procs):
    import compton_case as CC
    import oracle_lib as OL
    OL.build()
    jobs = [("lineage", CC.LINEAGE_SEED, CC.IDENT_SOURCES, r, CC.IDENT_SHARDS, "det")
            for r in range(CC.IDENT_SHARDS)]
    with get_context("spawn").Pool(procs) as pool:
        shards = pool.map(_lin_job, jobs)
        T0 = pool.map(_nocomp_job, [(CC.LINEAGE_SEED, CC.IDENT_SOURCES // 4)])[0]
    T = np.sum(shards, axis=0)
    F, E, cnt = CC.summary(T)
    F0, _, _ = CC.summary(T0)     # ewsv = energy / packets: same normalisation at n/4
    with np.errstate(invalid="ignore", divide="ignore"):
        unscat = np.where(F > 0, F0 / F, 0.0)
    np.savez_compressed(HERE / "compton_ident.npz", T=T, shard_T=np.array(shards),
        unscattered_share=unscat,
        sources=CC.IDENT_SOURCES, shards=CC.IDENT_SHARDS, seed=CC.LINEAGE_SEED,
        n_e_factor=CC.N_E_FACTOR)
    print("ident: collisions %d, escapes %d (scattered %d), compb %d; unscattered share above "
          "%.0e keV <= %.3f" % (cnt[3], cnt[1], cnt[11], cnt[6], CC.COMPTON_E_MIN,
                                unscat[CC.compton_bins()].max()))


def make_fib(runs, procs, work):
    import compton_case as CC
    import oracle_lib as OL
    OL.build()
    work = Path(work)
    work.mkdir(parents=True, exist_ok=True)
    jobs = [(k, CC.fib_seed(k), CC.FIB_SOURCES, str(work)) for k in range(runs)]
    recs = [None] * runs
    t0 = time.time()
    with get_context("spawn").Pool(procs) as pool:
        for i, (k, rec) in enumerate(pool.imap_unordered(_fib_job, jobs)):
            recs[k] = rec
            if i % 20 == 0:
                print("fib run %d/%d (%.0f s)" % (i + 1, runs, time.time() - t0), flush=True)
        check = pool.map(_fib_check, [CC.FIB_SEED0 - 1])[0]
    R = np.array(recs)
    nb = 128
    F, E, cnt, secs = R[:, :nb], R[:, nb:nb + 5], R[:, nb + 5:nb + 5 + 16], R[:, -1]
    np.savez_compressed(HERE / "compton_fib.npz", seeds=np.array([CC.fib_seed(k) for k in range(runs)]),
                        F=F, edout=E, counters=cnt, sources=CC.FIB_SOURCES,
                        check_seed=CC.FIB_SEED0 - 1, check_sources=CC.FIB_CHECK_SOURCES,
                        check_T=check, n_e_factor=CC.N_E_FACTOR, cpu_seconds=secs)
    m, sd = E.mean(axis=0), E.std(axis=0, ddof=1) / np.sqrt(len(E))
    print("fib: %d runs x %d sources, %.3g collisions, %.3g scattered escapes; band means %s, "
          "rel 1-sigma of the mean %s" % (runs, CC.FIB_SOURCES, cnt[:, 3].sum(), cnt[:, 11].sum(),
                                          m, sd / np.where(m > 0, m, 1)))


def _lin_run_job(args):
    """One lineage-stream run of FIB_SOURCES sources (own seed), as a fib run:
    probe bundles (the GPU's algorithm) or per-copy probes (C2O_PROBE_BUNDLES=0)."""
    import os
    k, seed, n, bundles, work = args
    out = Path(work) / ("lin%d_%05d.npy" % (bundles, k))
    if out.exists():
        return k, np.load(out)
    os.environ["C2O_PROBE_BUNDLES"] = str(bundles)
    import compton_case as CC
    t0 = time.time()
    T = CC.oracle_run(("lineage", seed, n, 0, 1, "ref"))
    F, E, cnt = CC.summary(T)
    rec = np.concatenate([F, E, cnt, [time.time() - t0]])
    np.save(out, rec)
    return k, rec


def make_lin(runs, procs, work):
    """compton_lin.npz: `runs` lineage-stream runs per probe mode (bundles and
    per-copy), each FIB_SOURCES sources with seed lin_seed(k), per-run F(E),
    light curves and counters -- the lineage side of the Compton-component
    comparison with run-to-run (not shard) variances, and the bundles vs
    per-copy split on identical run sizes (tests/test_compton_oracle.py)."""
    import compton_case as CC
    import oracle_lib as OL
    OL.build()
    work = Path(work)
    work.mkdir(parents=True, exist_ok=True)
    out = {}
    t0 = time.time()
    with get_context("spawn").Pool(procs) as pool:
        for bundles in (1, 0):
            jobs = [(k, CC.lin_seed(k), CC.FIB_SOURCES, bundles, str(work)) for k in range(runs)]
            recs = [None] * runs
            for i, (k, rec) in enumerate(pool.imap_unordered(_lin_run_job, jobs)):
                recs[k] = rec
                if i % 20 == 0:
                    print("lin%d run %d/%d (%.0f s)" % (bundles, i + 1, runs, time.time() - t0), flush=True)
            R = np.array(recs)
            nb = 128
            tag = "bundle" if bundles else "copy"
            out[tag + "_F"] = R[:, :nb]
            out[tag + "_edout"] = R[:, nb:nb + 5]
            out[tag + "_counters"] = R[:, nb + 5:nb + 5 + 16]
            out[tag + "_cpu_seconds"] = R[:, -1]
    np.savez_compressed(HERE / "compton_lin.npz", seeds=np.array([CC.lin_seed(k) for k in range(runs)]),
                        sources=CC.FIB_SOURCES, n_e_factor=CC.N_E_FACTOR, **out)
    for tag in ("bundle", "copy"):
        c = out[tag + "_counters"]
        print("lin %s: %d runs, %.4g collisions per run" % (tag, runs, c[:, 3].mean()))


def _fib_check(seed):
    import compton_case as CC
    return CC.oracle_run(("fib", seed, CC.FIB_CHECK_SOURCES))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--runs", type=int, default=5000)
    ap.add_argument("--procs", type=int, default=8)
    ap.add_argument("--work", default="/tmp/c2d_compton_fib")
    ap.add_argument("--lin-runs", type=int, default=256)
    ap.add_argument("--only", choices=("ident", "fib", "lin"), default=None)
    a = ap.parse_args()
    if a.only in (None, "ident"):
        make_ident(a.procs)
    if a.only in (None, "fib"):
        make_fib(a.runs, a.procs, a.work)
    if a.only in (None, "lin"):
        make_lin(a.lin_runs, a.procs, a.work)


if __name__ == "__main__":
    main()
