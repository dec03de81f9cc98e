#!/usr/bin/env python3
"""Headline benchmark: photon packet-steps/s of the MI355X transport engine.

Workload (BASELINE.json configs[1]): 32x32 (r,z) grid,
1e7 volume packets per step per GPU (weak scaling), splits 10/10/3/10,
inputm.dat medium, FP solver off, census carried from step to step.  One
"step" = one Monte-Carlo time step of the hot path: census + volume
transport (all scatter generations) on every GPU + the RCCL all-reduce of
the fused tally buffer.  Inputs are resident in HBM before timing (the
per-step tables are constant for T_const=1, uploaded once).

    python bench.py [--gpus N --steps K --warmup W]
    torchrun --nproc-per-node N bench.py --gpus N ...   (one rank per GPU)

Rank 0 prints ONE JSON line.  `roofline` prices the dominant kernel
(generation-0 transport launch) at 160 algorithmic bytes per packet-step
(SURVEY.md §8(d)); `cpu_baseline` times the C oracle (a port of the
reference's algorithm, exact comtot, glibc libm) on the host cores on a
bounded sample of the same workload.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

METRIC = "photon-packet-steps/sec (whole node) at 1/2/4/8 GPUs; % HBM roofline"
BYTES_PER_STEP = 160.0          # 80 B packet record in + out
HBM_PEAK_GBS = 8000.0           # MI355X_MICROARCH.md: 8.0 TB/s


def _cpu_worker(args):
    """One host core: the C oracle (ref build: glibc, exact comtot, lineage RNG)."""
    rank, world, sources = args
    sys.path.insert(0, str(ROOT / "tests"))
    import oracle_lib as OL
    from compton2d_amd import abi, synth
    wl = synth.c2_workload(sources=sources, rank=rank, world=world,
                           comtot_mode=abi.COMTOT_EXACT,
                           census_capacity=int(2.5 * sources / world) + 4096,
                           event_capacity=1 << 16)
    o = OL.Oracle(wl.grid, OL.RNG_LINEAGE, "ref")
    si = wl.step0
    si.ncycle, si.time = 1, 0.0
    t0 = time.perf_counter()
    rc = o.step(si)
    dt = time.perf_counter() - t0
    steps = float(o.tallies()[abi.tally_layout(wl.grid.nz, wl.grid.nr, 1)["counters"][0]
                              + abi.CNT_STEPS])
    o.close()
    return rc, steps, dt


def cpu_baseline(target_s: float = 15.0) -> dict:
    import multiprocessing as mp
    sys.path.insert(0, str(ROOT / "tests"))
    import oracle_lib as OL
    OL.build()
    try:
        ncpu = len(os.sched_getaffinity(0))
    except AttributeError:
        ncpu = os.cpu_count() or 1
    cores = max(1, min(16, ncpu))
    # calibrate the per-core rate on a small sample, then size the real sample
    rc, steps, dt = _cpu_worker((0, 1, 400))
    per_core_src_s = 400.0 / max(dt, 1e-6)
    sources = int(max(cores * 400, per_core_src_s * cores * target_s))
    ctx = mp.get_context("spawn")
    t0 = time.perf_counter()
    with ctx.Pool(cores) as pool:
        res = pool.map(_cpu_worker, [(r, cores, sources) for r in range(cores)])
    wall = time.perf_counter() - t0
    if any(r[0] != 0 for r in res):
        raise RuntimeError("cpu baseline oracle failed: %s" % [r[0] for r in res])
    steps = sum(r[1] for r in res)
    t = max(r[2] for r in res)
    return {"value": steps / t, "unit": "packet-steps/s", "cores": cores, "kind": "port",
            "sample": ("C2 32x32 grid, one transport step of %d volume sources (from an empty "
                       "census) sharded over %d processes; C oracle = port of the reference "
                       "algorithm (exact 199-term comtot, glibc libm, lineage RNG); %.0f "
                       "packet-steps in %.1f s (pool wall %.1f s)" % (sources, cores, steps, t, wall))}


def load_pmc(workload_key: str):
    """HBM bytes per packet-step of the generation-0 transport launch, from the
    committed rocprofv3 PMC summary (tools/gpu_profile.sh + tools/pmc_summary.py:
    separate FETCH_SIZE and WRITE_SIZE passes, FETCH_SIZE doubled for gfx950)."""
    p = ROOT / "profiles" / "pmc_latest.json"
    if not p.exists():
        return None
    try:
        d = json.loads(p.read_text())
        if d.get("workload_key") == workload_key:
            return float(d["hbm_bytes_per_step"])
    except Exception:
        return None
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--sources", type=int, default=10_000_000, help="volume packets/step/GPU")
    ap.add_argument("--grid", type=int, default=32)
    ap.add_argument("--mode", choices=("fast", "exact"), default="fast")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    args = ap.parse_args()

    import torch
    from compton2d_amd import abi, distributed, synth
    from compton2d_amd.engine import Engine

    rank, world, local = distributed.init()
    if world != args.gpus and world > 1:
        raise SystemExit("bench: --gpus %d but WORLD_SIZE=%d" % (args.gpus, world))
    if not torch.cuda.is_available():
        raise SystemExit("bench: no GPU visible")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    total_steps = args.warmup + args.steps
    mode = abi.COMTOT_TABLE if args.mode == "fast" else abi.COMTOT_EXACT
    wl = synth.c2_workload(nz=args.grid, nr=args.grid, sources=args.sources * world,
                           comtot_mode=mode, rank=rank, world=world, device=local,
                           census_capacity=int((total_steps + 1) * args.sources * 1.2) + (1 << 20),
                           event_capacity=int(2 * args.sources) + (1 << 20))
    eng = Engine(wl.grid)
    T = torch.zeros(eng.layout.total, dtype=torch.float64, device=dev)
    eng.use_tally_tensor(T)
    eng.set_step(wl.step0)
    cnt0 = eng.layout.counters

    def one_step(n):
        ncycle, t = wl.clock(n)
        eng.set_clock(ncycle, t, wl.dt)
        eng.run_step()
        distributed.allreduce_tallies(T)

    n = 0
    for _ in range(args.warmup):
        one_step(n)
        n += 1
    distributed.barrier(dev)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    steps_global = 0.0
    g0_ms, g0_steps, aborted = 0.0, 0, 0.0
    per_step = {k: 0.0 for k in ("sources", "escapes", "census", "collisions", "events", "generations")}
    cidx = {"sources": abi.CNT_SOURCES, "escapes": abi.CNT_ESCAPES, "census": abi.CNT_CENSUS,
            "collisions": abi.CNT_COLLIDE, "events": abi.CNT_EVENTS, "generations": abi.CNT_GENS}
    for _ in range(args.steps):
        one_step(n)
        n += 1
        c = T[cnt0:cnt0 + abi.NCOUNTERS].cpu().numpy()
        steps_global += float(c[abi.CNT_STEPS])
        aborted += float(c[abi.CNT_ABORTED])
        for k, i in cidx.items():
            per_step[k] += float(c[i]) / args.steps
        ms, _, _ = eng.last_kernel_ms()
        g0_ms += ms
        g0_steps += eng.last_gen0_steps()
    torch.cuda.synchronize()
    distributed.barrier(dev)
    elapsed = time.perf_counter() - t0
    elapsed = distributed.allreduce_max(elapsed, dev)
    if rank != 0:
        return
    value = steps_global / elapsed
    achieved = g0_steps * BYTES_PER_STEP / (g0_ms * 1e-3) / 1e9 if g0_ms > 0 else 0.0
    workload_key = "c2_%dx%d_%d_%s" % (args.grid, args.grid, args.sources, args.mode)
    bps = load_pmc(workload_key)
    # HBM bytes of one generation-0 launch: measured bytes/packet-step x this run's steps/launch
    traffic = bps * (g0_steps / args.steps) if bps is not None else None
    out = {
        "metric": METRIC,
        "value": value,
        "unit": "packet-steps/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic: reference volume_em/P_nontherm tables of the inputm.dat medium tiled "
                "over the grid; volume packets sampled on device",
        "config": {
            "workload": wl.description,
            "grid": "%dx%d" % (args.grid, args.grid),
            "sources_per_gpu_per_step": args.sources,
            "comtot": "table (cubic, 2048 pts)" if mode == abi.COMTOT_TABLE else "exact",
            "parallelism": "lineage-sharded sources, %d rank(s), RCCL all-reduce of tallies" % world,
            "packet_steps_timed": steps_global,
            "aborted_packets": aborted,
            "per_step_counts": per_step,
        },
        "roofline": {
            "bound": "hbm",
            "achieved": achieved,
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS,
            "traffic": traffic,
            "kernel": "c2d_transport_kernel_%s (generation 0)" % args.mode,
            "per_unit_bytes": BYTES_PER_STEP,
            "kernel_ms_avg": g0_ms / args.steps,
            "traffic_unit": "bytes per launch (PMC FETCH_SIZEx2 + WRITE_SIZE)",
            "traffic_bytes_per_step": bps,
            "steps_per_launch_avg": g0_steps / args.steps,
        },
        "cpu_baseline": None,
    }
    if world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(args.cpu_seconds)
    print(json.dumps(out))
    eng.close()


if __name__ == "__main__":
    main()
