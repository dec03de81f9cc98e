#!/usr/bin/env python3
"""Where the transport kernel's time goes: wave-level section timers of a
-DC2D_TR_PROF build (tools/build_sweep.sh prof:4:off:-DC2D_TR_PROF, then
C2D_LIBRARY=compton2d_amd/sweep/prof/libcompton2d.so) on the C3 coupled run.

    python tools/tr_prof.py [--sources 100000000] [--steps 6]

Prints, for each step, the share of shader cycles per section of the lane
state machine (compton2d_amd/csrc/transport.hip TP_*), lanes in flight per
iteration, and how often per iteration (wave level) and per lane the rare
branches (new item, census write, escape, collision, probe restart) run.
"""
from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT)]

SECTIONS = ["refill", "start", "geom", "abs", "event", "post", "points", "write"]
COUNTS = {"got": 10, "census": 12, "leak": 14, "collide": 16, "restart": 18}


def summarize(v, steps):
    cyc = [float(v[i]) for i in range(len(SECTIONS))]
    tot = sum(cyc) or 1.0
    it = float(v[8]) or 1.0
    out = {"packet_steps": steps, "waves": int(v[20]), "iterations": int(v[8]),
           "cycles_per_iter": tot / it,
           "share": {k: round(c / tot, 4) for k, c in zip(SECTIONS, cyc)},
           "cycles_per_iter_by_section": {k: round(c / it, 1) for k, c in zip(SECTIONS, cyc)},
           "lanes_in_flight_per_iter": float(v[9]) / it,
           "steps_per_iter": steps / it}
    for k, i in COUNTS.items():
        out[k] = {"wave_frac": float(v[i]) / it, "lanes_per_exec": float(v[i + 1]) / max(1.0, float(v[i]))}
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sources", type=int, default=100_000_000)
    ap.add_argument("--steps", type=int, default=6)
    args = ap.parse_args()
    import torch
    from compton2d_amd import synth
    from compton2d_amd.coupled import CoupledRun
    from compton2d_amd.engine import Engine

    free, _ = torch.cuda.mem_get_info(0)
    ccap = int(min((args.steps + 1) * args.sources * 1.1 + (1 << 20), 0.8 * free / 128))
    wl = synth.c3_workload(sources=args.sources, census_capacity=ccap,
                           event_capacity=2 * args.sources + (1 << 20))
    eng = Engine(wl.grid)
    run = CoupledRun(eng, wl)
    for _ in range(args.steps):
        r = run.step()
        v = eng.transport_prof()
        row = summarize(v, r["packet_steps"])
        row.update(ncycle=r["ncycle"], transport_gen0_ms=r["transport_gen0_ms"])
        print(json.dumps(row), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
