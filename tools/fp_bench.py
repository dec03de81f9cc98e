#!/usr/bin/env python3
"""Fokker-Planck update throughput (c2d_fp_step) on one MI355X.

Workload: an nz x nr grid whose zones carry the reference's own FP inputs
(tests/golden/fp_pick.npz, step 1: electron spectra after one transport step,
photon field n_field, Eloss_sy, ...) tiled over the grid; one `update` =
FP_calc for every zone (thousands of implicit sub-steps each).  Reports
zones/s on the GPU (HIP-event kernel time and wall time of c2d_fp_step), the
C oracle's zones/s on host cores for a bounded sample, and checks the GPU
result against the oracle on that sample (bit-identical).

    python tools/fp_bench.py [--grid 32] [--reps 3] [--cpu-zones 16]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "tests")]


def tiled_case(nz: int, nr: int, case: str = "fp_pick", vary: bool = False):
    from golden_io import FpGoldenCase
    c = FpGoldenCase(case)
    n = c.steps[0]
    fi = c.fp_in(n)
    src_nz, src_nr = c.nz, c.nr
    jj = np.arange(nz) % src_nz
    kk = np.arange(nr) % src_nr
    tile = {}
    for key, v in fi.items():
        if isinstance(v, np.ndarray):
            tile[key] = v[jj][:, kk].copy()
        else:
            tile[key] = v
    if vary:
        # every zone its own state: n_e and tea perturbed per zone, so no two
        # zones walk the same temperature-search chain (gamma_bar memo, fp.hip)
        cell = np.arange(nz * nr, dtype=np.float64).reshape(nz, nr)
        tile["n_e"] = tile["n_e"] * (1.0 + 0.013 * (cell % 53))
        tile["tea"] = tile["tea"] * (1.0 + 0.007 * (cell % 41))
    # same cylinder (z(nz), r(nr) fix t_esc/t_acc, update2d.f:460-461) cut into nz x nr
    # zones; with the fixture's switches (no flare, no shock injection) a zone's result
    # depends only on its own inputs, which are the fixture zone's
    g = c.grid()
    g.nz, g.nr = nz, nr
    zmax, rmax = c.a["cfg_z"][-1], c.a["cfg_r"][-1]
    g.z = zmax * np.arange(1, nz + 1, dtype=np.float64) / nz
    g.r = rmax * np.arange(1, nr + 1, dtype=np.float64) / nr
    return c, g, tile


def _cpu_zone(args):
    """Oracle `update` on a 1 x m strip of zones (one process)."""
    nz, nr, cols, case, vary = args
    sys.path[:0] = [str(ROOT), str(ROOT / "tests")]
    import oracle_lib as OL
    c, g, tile = tiled_case(nz, nr, case, vary)
    sub = {k: (v[:1, cols[0]:cols[1]].copy() if isinstance(v, np.ndarray) else v)
           for k, v in tile.items()}
    g.nz, g.nr = 1, cols[1] - cols[0]
    g.z = g.z[-1:]
    g.r = g.r[cols[0]:cols[1]]
    t0 = time.perf_counter()
    r = OL.fp_step(g, c.constants(), sub["ncycle"], sub["time"], sub["dt"], sub, sub, flavor="det")
    return time.perf_counter() - t0, r["f_nt"], r["Te_new"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--grid", type=int, default=32)
    ap.add_argument("--nz", type=int, default=None)
    ap.add_argument("--nr", type=int, default=None)
    ap.add_argument("--case", default="fp_pick")
    ap.add_argument("--vary", action="store_true", help="perturb n_e, tea per zone")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--cpu-zones", type=int, default=16)
    ap.add_argument("--mode", choices=("exact", "fast"), default="exact",
                    help="c2d_fp_set_mode: exact (bit for bit) or fast (block-parallel, fp_fast.hip)")
    args = ap.parse_args()
    from compton2d_amd.engine import Engine
    nz = args.nz or args.grid
    nr = args.nr or args.grid
    c, g, tile = tiled_case(nz, nr, args.case, args.vary)
    g.device = 0
    eng = Engine(g)
    eng.fp_set_config(c.constants())
    from compton2d_amd import abi
    eng.fp_set_mode(abi.FP_FAST if args.mode == "fast" else abi.FP_EXACT)
    r = eng.fp_step(tile["ncycle"], tile["time"], tile["dt"], tile, tile)   # warm-up
    first_ms = eng.last_fp_ms()    # cold gamma_bar memo, zones in index order
    walls, kms = [], []
    for _ in range(args.reps):
        t0 = time.perf_counter()
        r = eng.fp_step(tile["ncycle"], tile["time"], tile["dt"], tile, tile)
        walls.append(time.perf_counter() - t0)
        kms.append(eng.last_fp_ms())
    substeps = float(np.sum(r["zone_diag"][..., 5]))
    # CPU baseline: the oracle on a sample of zones (row 0, first cpu_zones columns)
    import multiprocessing as mp
    m = min(args.cpu_zones, nr)
    try:
        ncpu = len(os.sched_getaffinity(0))
    except AttributeError:
        ncpu = os.cpu_count() or 1
    cores = max(1, min(16, ncpu, m))
    bounds = np.linspace(0, m, cores + 1).astype(int)
    jobs = [(nz, nr, (int(bounds[i]), int(bounds[i + 1])), args.case, args.vary) for i in range(cores)
            if bounds[i + 1] > bounds[i]]
    t0 = time.perf_counter()
    with mp.get_context("spawn").Pool(len(jobs)) as pool:
        res = pool.map(_cpu_zone, jobs)
    cpu_wall = time.perf_counter() - t0
    cpu_t = max(x[0] for x in res)
    f_cpu = np.concatenate([x[1][0] for x in res], axis=0)
    te_cpu = np.concatenate([x[2][0] for x in res], axis=0)
    same = bool(np.array_equal(f_cpu, r["f_nt"][0, :m]) and np.array_equal(te_cpu, r["Te_new"][0, :m]))
    fg = r["f_nt"][0, :m]
    f_dev = float(np.max(np.abs(fg - f_cpu)) / max(np.max(np.abs(f_cpu)), 1e-300))
    te_same = bool(np.array_equal(te_cpu, r["Te_new"][0, :m]))
    ms = float(np.median(kms))
    out = {
        "kernel": ("c2d_fp_fast_kernel<256> (one 4-wave workgroup per zone, C2D_FP_FAST)"
                   if args.mode == "fast" else "c2d_fp_kernel (C2D_FP_EXACT)"),
        "mode": args.mode,
        "zones": nz * nr,
        "implicit_substeps": substeps,
        "kernel_ms": ms,
        "kernel_ms_first_call": first_ms,
        "wall_ms": float(np.median(walls)) * 1e3,
        "zones_per_s": nz * nr / (ms * 1e-3),
        "substeps_per_s": substeps / (ms * 1e-3),
        "cpu_baseline": {"zones_per_s": m / cpu_t, "cores": len(jobs), "kind": "port",
                         "sample": "%d zones of row 0 on %d processes (oracle, det math), "
                                   "%.1f s (pool wall %.1f s)" % (m, len(jobs), cpu_t, cpu_wall)},
        "gpu_equals_oracle_on_sample": same,
        "f_nt_max_dev_vs_oracle_on_sample": f_dev,
        "Te_new_equal_on_sample": te_same,
        "workload": "%s fixture zones (reference FP inputs after one transport step) "
                    "tiled over %dx%d%s" % (args.case, nz, nr, ", n_e/tea varied per zone" if args.vary else ""),
        "memo": os.environ.get("C2D_FP_MEMO", "1"),
        "Te_new_range": [float(r["Te_new"].min()), float(r["Te_new"].max())],
    }
    print(json.dumps(out))
    eng.close()


if __name__ == "__main__":
    main()
