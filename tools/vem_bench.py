#!/usr/bin/env python3
"""Emission/absorption tables (c2d_volume_em) throughput on one MI355X.

Workload: the C2 grid (32x32 = 1024 cells), cell states drawn over the
branches volume_em takes (tests/test_gpu_vem.py:_random_state, electron
spectra of the reference's fixtures); one call = imcgen2d's per-cell loop
for every cell (400 energies x 199 electron bins of two Bessel fits each).
Reports cells/s on the GPU (HIP-event kernel time and call wall time), the
C oracle (the reference's algorithm, glibc) on one host core for a bounded
sample of cells, and checks the GPU against the det oracle on that sample.

    python tools/vem_bench.py [--grid 32] [--reps 5] [--cpu-cells 8]
"""
from __future__ import annotations

import argparse
import json
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "tests")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--grid", type=int, default=32)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--cpu-cells", type=int, default=8)
    args = ap.parse_args()
    import oracle_lib as OL
    from compton2d_amd import synth
    from compton2d_amd.engine import Engine
    from test_gpu_vem import _random_state
    n = args.grid
    wl = synth.c2_workload(nz=n, nr=n, sources=1)
    st = _random_state(n, n, seed=9)
    eng = Engine(wl.grid)
    eng.volume_em(wl.dt, st)                          # warm-up
    ms, t0 = [], time.perf_counter()
    for _ in range(args.reps):
        r = eng.volume_em(wl.dt, st)
        ms.append(eng.last_vem_ms())
    wall = (time.perf_counter() - t0) / args.reps
    eng.close()
    cells = n * n
    m = max(1, min(args.cpu_cells, n))
    sub = {k: (v[:1, :m] if isinstance(v, np.ndarray) else v) for k, v in st.items()}
    g = synth.c2_workload(nz=n, nr=n, sources=1).grid
    g.nz, g.nr, g.z, g.r = 1, m, g.z[:1], g.r[:m]
    t0 = time.perf_counter()
    OL.vem_step(g, wl.dt, sub, flavor="ref")
    cpu = time.perf_counter() - t0
    o = OL.vem_step(g, wl.dt, sub, flavor="det")
    exact = all(np.array_equal(r[k][:1, :m], o[k]) for k in ("kappa_tot", "eps_tot", "eps_th", "Eloss_tot"))
    out = {"cells": cells, "kernel_ms": float(np.mean(ms)), "cells_per_s": cells / (np.mean(ms) * 1e-3),
           "wall_ms": wall * 1e3, "wall_cells_per_s": cells / wall,
           "cpu_baseline": {"value": m / cpu, "unit": "cells/s", "cores": 1, "kind": "port",
                            "sample": "%d cells of the same states, oracle (glibc)" % m},
           "sample_bit_exact_vs_det_oracle": bool(exact),
           "work_per_cell": "400 energies x 199 electron bins (expk13, expk43, exp) + cyclotron"}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
