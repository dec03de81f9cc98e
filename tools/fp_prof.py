#!/usr/bin/env python3
"""FP kernel section timers (build with FP_FLAGS=-DC2D_FP_PROF; select it with
C2D_LIBRARY): shader cycles per zone in the temperature search (gamma_bar),
the tridiagonal solve and the whole sub-step loop, from zone_diag slots 0-2."""
import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "tests")]


def main():
    from compton2d_amd.engine import Engine
    from fp_bench import tiled_case
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--nz", type=int, default=8)
    ap.add_argument("--nr", type=int, default=8)
    ap.add_argument("--vary", action="store_true")
    ap.add_argument("--mode", choices=("exact", "fast"), default="exact")
    ap.add_argument("--sections", action="store_true",
                    help="the library was built with C2D_FP_PROF_SEC: slots 4/6/7 are the sub-step's "
                         "sections A (scalars..loop-350 sums), B (injection..tridiagonal coefficients), "
                         "C (after the solve..gbar sums)")
    ap.add_argument("--mcd", action="store_true",
                    help="built with C2D_FP_PROF_MCD: slot 7 is the McDonald stopping tests' cycles")
    ap.add_argument("--memo", action="store_true",
                    help="built with C2D_FP_PROF_MEMO: slots 4/6/7 are gamma_bar calls, LDS-memo hits, "
                         "global-memo hits")
    args = ap.parse_args()
    from compton2d_amd import abi
    c, g, tile = tiled_case(args.nz, args.nr, vary=args.vary)
    g.device = 0
    eng = Engine(g)
    eng.fp_set_config(c.constants())
    eng.fp_set_mode(abi.FP_FAST if args.mode == "fast" else abi.FP_EXACT)
    r = eng.fp_step(tile["ncycle"], tile["time"], tile["dt"], tile, tile)
    d = np.asarray(r["zone_diag"]).reshape(-1, 8)
    steps = d[:, 5]
    out = {"mode": args.mode, "zones": len(d), "substeps_mean": float(steps.mean()), "kernel_ms": eng.last_fp_ms(),
           "waves_per_zone": eng.last_fp_waves() if hasattr(eng, "last_fp_waves") else None}
    for i, k in enumerate(("search_cycles", "tridag_cycles", "loop_cycles", "search_calls")):
        out[k + "_per_substep"] = float((d[:, i] / steps).mean())
    # the zone that bounds the launch (largest loop cycles) and the spread
    zmax = int(np.argmax(d[:, 2]))
    out["critical_zone"] = {"zone": zmax, "substeps": float(steps[zmax]), "loop_cycles": float(d[zmax, 2]),
                            "search_cycles": float(d[zmax, 0]), "tridag_cycles": float(d[zmax, 1]),
                            "mcd_calls": float(d[zmax, 3])}
    out["loop_cycles_max_over_mean"] = float(d[:, 2].max() / d[:, 2].mean())
    out["substeps_max"] = float(steps.max())
    if args.memo:
        for name, q in (("memo_calls", 4), ("memo_lds_hits", 6), ("memo_global_hits", 7)):
            out[name + "_per_substep"] = float((d[:, q] / steps).mean())
            out["critical_zone"][name] = float(d[zmax, q])
    elif args.sections:
        for name, q in (("sec_a", 4), ("sec_b", 6), ("sec_c", 7)):
            out[name + "_cycles_per_substep"] = float((d[:, q] / steps).mean())
            out["critical_zone"][name + "_cycles"] = float(d[zmax, q])
    elif args.mcd:                    # built with C2D_FP_PROF_MCD: slot 7 = the stopping tests
        calls = np.maximum(d[:, 3], 1)
        out["mcd_passes_per_call"] = float((d[:, 4] / calls).mean())
        out["mcd_loop_cycles_per_call"] = float((d[:, 6] / calls).mean())
        out["mcd_firsts_cycles_per_call"] = float((d[:, 7] / calls).mean())
    elif args.mode == "fast":         # McDonald internals (fp_fast.hip, C2D_FP_PROF)
        calls = np.maximum(d[:, 3], 1)
        out["mcd_passes_per_call"] = float((d[:, 4] / calls).mean())
        out["mcd_loop_cycles_per_call"] = float((d[:, 6] / calls).mean())
        out["mcd_finish_cycles_per_call"] = float((d[:, 7] / calls).mean())
    print(json.dumps(out))
    eng.close()


if __name__ == "__main__":
    main()
