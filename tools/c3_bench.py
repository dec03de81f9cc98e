#!/usr/bin/env python3
"""C3 coupled run, per step (compton2d_amd/coupled.py): tables, transport,
FP and the census population of every MC step, to size bench.py's census
capacity and to see where a coupled step's time goes.

    python tools/c3_bench.py [--sources 10000000] [--steps 25] [--host-tables]
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
    ap.add_argument("--sources", type=int, default=10_000_000)
    ap.add_argument("--steps", type=int, default=25)
    ap.add_argument("--host-tables", action="store_true")
    ap.add_argument("--census-capacity", type=float, default=0.0)
    args = ap.parse_args()
    import torch
    from compton2d_amd import abi, synth
    from compton2d_amd.coupled import CoupledRun
    from compton2d_amd.engine import Engine

    free, _ = torch.cuda.mem_get_info(0)
    ccap = int(args.census_capacity or min((args.steps + 1) * args.sources * 1.5 + (1 << 20),
                                           0.8 * free / 128))
    wl = synth.c3_workload(sources=args.sources, census_capacity=ccap,
                           event_capacity=2 * args.sources + (1 << 20))
    eng = Engine(wl.grid)
    run = CoupledRun(eng, wl, device_resident=not args.host_tables)
    print(json.dumps({"workload": wl.description, "census_capacity": ccap}), flush=True)
    for _ in range(args.steps):
        t0 = time.perf_counter()
        r = run.step()
        r["wall_s"] = time.perf_counter() - t0
        r["census_count"] = eng.census_count()
        print(json.dumps(r), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
