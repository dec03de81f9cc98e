"""tests/golden/spectrum_fib.npz: F(E) and light curves of the reference's
algorithm with the reference's own lagged-Fibonacci streams (C oracle, glibc;
bit-exact to the Fortran reference, tests/test_oracle_golden.py) on the
north-star spectrum workload (tests/spectrum_case.py), 3 seeds, and the
light curves of the lineage-stream run's 8 shards (the oracle's lineage mode:
the GPU's SplitMix64 draw streams, Philox-derived keys, and probe bundles), whose shard-to-shard scatter sizes the
statistical error of a 1e7-packet run.  The GPU spectrum test compares the
fast kernel against it.

usage: python tests/golden/make_spectrum.py"""
import sys
from multiprocessing import get_context
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
sys.path[:0] = [str(HERE.parents[1]), str(HERE.parent)]


def main():
    import oracle_lib as OL
    import spectrum_case as S
    OL.build()
    jobs = [("fib", s) for s in S.FIB_SEEDS] + [("lineage", S.LINEAGE_SEED, r, S.SHARDS)
                                                for r in range(S.SHARDS)]
    with get_context("spawn").Pool(8) as pool:
        allres = pool.map(S.oracle_run, jobs)
    res, lin = allres[:len(S.FIB_SEEDS)], allres[len(S.FIB_SEEDS):]
    np.savez_compressed(HERE / "spectrum_fib.npz", seeds=np.array(S.FIB_SEEDS),
                        F=np.array([r[0] for r in res]), edout=np.array([r[1] for r in res]),
                        escapes=np.array([r[2] for r in res]), sources=S.SOURCES,
                        dt_factor=S.DT_FACTOR,
                        lineage_edout_shards=np.array([r[1] for r in lin]),
                        lineage_F=sum(r[0] for r in lin))
    print("escapes per seed:", [r[2] for r in res])


if __name__ == "__main__":
    main()
