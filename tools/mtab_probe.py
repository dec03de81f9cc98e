#!/usr/bin/env python3
"""Section cycles of the fast FP kernel's McDonald moment-table lookup
(c2d_selftest_mcd_fast of a -DC2D_MTAB_TIMERS build, C2D_LIBRARY=...):
entry load + Horner, the stopping-index fix of series 2, of series 3, the
ratio; medians over z spread across the table."""
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

from compton2d_amd.engine import device_mcd_fast

z = 2.0 ** np.random.default_rng(3).uniform(-12, np.log2(5.0), 2000)
out = device_mcd_fast(z)
ok = out[:, 4] == 1
print("answered %d of %d" % (ok.sum(), len(z)))
for i, name in enumerate(("load+exp+horner", "fixes", "-", "ratio")):
    print("%-12s median %8.0f  p90 %8.0f" % (name, np.median(out[ok, i]), np.percentile(out[ok, i], 90)))
print("%-12s median %8.0f" % ("total", np.median(out[ok, 5])))
print("%-12s median %8.0f" % ("series", np.median(out[ok, 6])))
