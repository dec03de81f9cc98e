"""tests/golden/spectrum_fib.npz: F(E) and light curves of the reference's
algorithm with the reference's own lagged-Fibonacci streams (C oracle, glibc;
bit-exact to the Fortran reference, tests/test_oracle_golden.py) on the
north-star spectrum workload (tests/spectrum_case.py), 3 seeds.  The GPU
spectrum test compares the fast kernel against it.

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
    with get_context("spawn").Pool(len(S.FIB_SEEDS)) as pool:
        res = pool.map(S.oracle_run, [("fib", s) for s in S.FIB_SEEDS])
    np.savez_compressed(HERE / "spectrum_fib.npz", seeds=np.array(S.FIB_SEEDS),
                        F=np.array([r[0] for r in res]), edout=np.array([r[1] for r in res]),
                        escapes=np.array([r[2] for r in res]), sources=S.SOURCES,
                        dt_factor=S.DT_FACTOR)
    print("escapes per seed:", [r[2] for r in res])


if __name__ == "__main__":
    main()
