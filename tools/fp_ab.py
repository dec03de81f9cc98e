#!/usr/bin/env python3
"""A/B of FP kernel builds on the C3 golden FP inputs (all 270 zones, both FP
steps): kernel ms per library and, for -DC2D_FP_PROF builds, the per-zone
section cycles (zone_diag slots 0-3: search, tridag, loop, gamma_bar calls).

    python tools/fp_ab.py LIB.so [LIB2.so ...]
"""
import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "tests")]


def tiled(lib):
    """The steady regime: fp_pick tiled over 32x32 zones (thousands of
    sub-steps per zone, ~1.7 gamma_bar per sub-step)."""
    from compton2d_amd.engine import Engine
    from fp_bench import tiled_case
    c, g, tile = tiled_case(32, 32)
    g.device = 0
    eng = Engine(g, lib_path=Path(lib))
    eng.fp_set_config(c.constants())
    ms = []
    for _ in range(2):
        r = eng.fp_step(tile["ncycle"], tile["time"], tile["dt"], tile, tile)
        ms.append(eng.last_fp_ms())
    eng.close()
    return {"lib": Path(lib).name, "case": "fp_pick tiled 32x32", "kernel_ms": ms,
            "f_nt_sum": float(np.sum(r["f_nt"])), "Te_sum": float(np.sum(r["Te_new"]))}


def main():
    sys.path.insert(0, str(ROOT / "tools"))
    from compton2d_amd.engine import Engine
    from golden_io import CoupledGoldenCase
    gc = CoupledGoldenCase("c3_mrk421")
    ref = None
    for lib in sys.argv[1:]:
        print(json.dumps(tiled(lib)), flush=True)
        eng = Engine(gc.grid(device=0), lib_path=Path(lib))
        eng.fp_set_config(gc.constants())
        for n in gc.fp_steps:
            fi = gc.fp_in(n)
            ms = []
            for _ in range(3):
                r = eng.fp_step(fi["ncycle"], fi["time"], fi["dt"], fi, fi)
                ms.append(eng.last_fp_ms())
            d = np.asarray(r["zone_diag"]).reshape(-1, 8)
            out = {"lib": Path(lib).name, "step": n, "kernel_ms": ms, "substeps_mean": float(d[:, 5].mean()),
                   "substeps_max": float(d[:, 5].max())}
            if d[:, 2].max() > 0:
                loop = d[:, 2]
                out.update(loop_cycles_max=float(loop.max()), loop_cycles_mean=float(loop.mean()),
                           search_frac=float((d[:, 0] / np.maximum(loop, 1)).mean()),
                           tridag_frac=float((d[:, 1] / np.maximum(loop, 1)).mean()),
                           calls_per_substep=float((d[:, 3] / d[:, 5]).mean()),
                           search_cycles_per_call=float((d[:, 0] / np.maximum(d[:, 3], 1)).mean()))
            f = np.asarray(r["f_nt"])
            if ref is None:
                ref = {}
            if n in ref:
                out["f_nt_equal_first_lib"] = bool(np.array_equal(ref[n], f))
            else:
                ref[n] = f
            print(json.dumps(out), flush=True)
        eng.close()


if __name__ == "__main__":
    main()
