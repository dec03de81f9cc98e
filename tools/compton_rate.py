"""Time the Compton workload's runs on the GPU (tests/compton_case.py) at a
few run sizes: per-run wall time and the kernel milliseconds of the last
run (generation 0 vs all launches), to size tests/test_gpu_compton.py."""
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "tests")]

import compton_case as CC  # noqa: E402
from compton2d_amd import abi  # noqa: E402
from compton2d_amd.engine import Engine  # noqa: E402

for n in [int(x) for x in (sys.argv[1:] or ["100000", "1000000"])]:
    grid, si = CC.workload(mode=abi.COMTOT_TABLE, n=n)
    grid.event_capacity = max(16 * n, 32 * 8 * 100000)
    eng = Engine(grid)
    eng.set_step(si)
    reps = 5
    t0 = time.perf_counter()
    for r in range(reps):
        eng.census_truncate(0)
        eng.set_clock(r + 1, si.time, si.dt)
        eng.run_step()
        T = eng.tallies_raw()
    dt = (time.perf_counter() - t0) / reps
    g0, al, nl = eng.last_kernel_ms()
    c = T[eng.layout.counters:eng.layout.counters + abi.NCOUNTERS]
    print("n=%d: %.3f s per run; last run gen0 %.2f ms, all %.2f ms, %d launches, generations %d, "
          "collisions %d, compb %d, steps %.3g" % (n, dt, g0, al, nl, c[abi.CNT_GENS], c[abi.CNT_COLLIDE],
                                                   c[abi.CNT_COMPB], c[abi.CNT_STEPS]), flush=True)
    eng.close()
