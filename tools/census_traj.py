#!/usr/bin/env python3
"""Census population per MC step of the C2/C4 medium (32x32, FP off), to
size bench.py's spin-up and census capacity (the C3 deck: tools/c3_bench.py).

    python tools/census_traj.py [--sources 20000000] [--steps 120] [--grid 32]
"""
from __future__ import annotations

import argparse
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sources", type=int, default=20_000_000)
    ap.add_argument("--steps", type=int, default=120)
    ap.add_argument("--grid", type=int, default=32)
    ap.add_argument("--census-capacity", type=float, default=0.0)
    args = ap.parse_args()
    import torch
    from compton2d_amd import abi, synth
    from compton2d_amd.engine import Engine
    free, _ = torch.cuda.mem_get_info(0)
    ccap = int(args.census_capacity or min(60 * args.sources, 0.7 * free / 68))
    wl = synth.c2_workload(nz=args.grid, nr=args.grid, sources=args.sources, census_capacity=ccap,
                           event_capacity=2 * args.sources + (1 << 20))
    eng = Engine(wl.grid)
    eng.set_step(wl.step0)
    print(json.dumps({"workload": wl.description, "census_capacity": ccap}), flush=True)
    cnt0 = eng.layout.counters
    for n in range(args.steps):
        ncycle, t = wl.clock(n)
        eng.set_clock(ncycle, t, wl.dt)
        t0 = time.perf_counter()
        eng.run_step()
        wall = time.perf_counter() - t0
        c = eng.tallies_raw()[cnt0:cnt0 + abi.NCOUNTERS]
        g0, al, _ = eng.last_kernel_ms()
        print(json.dumps(dict(ncycle=ncycle, wall_s=wall, census_count=eng.census_count(),
                              packet_steps=float(c[abi.CNT_STEPS]), escapes=float(c[abi.CNT_ESCAPES]),
                              transport_gen0_ms=g0, transport_all_ms=al,
                              compaction=eng.last_compaction())), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
