#!/usr/bin/env python3
"""Headline benchmark: photon packet-steps/s of the MI355X Compton engine.

Workload (default `--workload c3`, BASELINE.json configs[2], SURVEY.md §8(d)
C3, the largest single-GPU configuration): the Mrk 421 SSC deck
(src_20121026/input.dat + inputm.dat; compton2d_amd/synth.py C3_DECK), 30x9
(z,r) zones, 1e8 volume packets per step per GPU, FP on.  One "step" = one
whole coupled Monte-Carlo time step on the GPU (compton2d_amd/coupled.py,
src/xec2d.f:67-87):

    c2d_volume_em       emission/absorption tables from the electron state
    budgets             nsv/ewsv (imcgen2d) from the zone emissivities
    c2d_run_step        census + volume transport, all scatter generations
    all-reduce          the fused tally buffer over RCCL (N > 1)
    c2d_fp_step         FP_calc for every zone, photon field read on the device

with tables and electron spectra resident in HBM across steps and the census
carried from step to step.  `--workload c2` is the 32x32 FP-off transport
workload of round 1; `--workload c4` is C2's medium at C4's 1.25e8
sources per GPU (1e9 per step on 8 GPUs).

    python bench.py [--gpus N --steps K --warmup W] [--workload c3|c2|c4]
    torchrun --nproc-per-node N bench.py --gpus N ...   (one rank per GPU)

Rank 0 prints ONE JSON line.  `value` = packet-steps of all ranks / the max
over ranks of the wall time of the K timed steps.  `roofline` prices the
dominant kernel (generation-0 transport launch) at 160 algorithmic bytes
(an 80-B packet record in + out) per lane path-step, the
pass through the geometry block that a probe bundle shares among its copies,
and carries its measured HBM bytes and VALU-issue fraction from the committed
PMC profile of the same command; `kernels` reports the FP and table kernels beside it;
`cpu_baseline` times the C oracle (a port of the reference's algorithm) on
the host's CPU share, on a strided sample of the GPU's own final census plus
the same fraction of the step's volume sources, and the FP_calc of sampled
zones, extrapolated to one whole coupled step.
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
N_SIMD = 1024                   # 256 CUs x 4 SIMDs
CLOCK_HZ = 2.4e9                # MI355X peak engine clock
CENSUS_BYTES = 2 * 64           # in + out census SoA record (c2d_device.hpp CensusSoA)
DEFAULT_SOURCES = {"c3": 100_000_000, "c2": 10_000_000, "c4": 125_000_000}


def cpu_share() -> tuple[int, int]:
    """(threads this job may use, nproc of the host).  On the GPU box the
    job's CPU share is OMP_NUM_THREADS (16 per GPU); nproc shows the host."""
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = os.cpu_count() or 1
    share = int(os.environ.get("OMP_NUM_THREADS", aff) or aff)
    return max(1, min(aff, share)), os.cpu_count() or aff


def _cpu_transport(args):
    """One host core: the C oracle (glibc, exact comtot, lineage RNG) on its
    shard of the sampled step (census records + volume sources)."""
    rank, world, grid_kw, si, cens = args
    sys.path.insert(0, str(ROOT / "tests"))
    import oracle_lib as OL
    from compton2d_amd import abi
    g = abi.GridConfig(**grid_kw)
    g.rank, g.world, g.comtot_mode = rank, world, abi.COMTOT_EXACT
    o = OL.Oracle(g, OL.RNG_LINEAGE, "ref")
    d6, i5, keys = cens
    o.import_census(d6[rank::world], i5[rank::world], keys[rank::world])
    t0 = time.perf_counter()
    rc = o.step(si)
    dt = time.perf_counter() - t0
    L = abi.tally_layout(g.nz, g.nr, int(np.asarray(g.mu).size))
    steps = float(o.tallies()[L["counters"][0] + abi.CNT_STEPS])
    o.close()
    return rc, steps, dt


def _cpu_fp(args):
    grid_kw, const, call, cells = args
    sys.path.insert(0, str(ROOT / "tests"))
    import oracle_lib as OL
    from compton2d_amd import abi
    t0 = time.perf_counter()
    OL.fp_step(abi.GridConfig(**grid_kw), const, *call, flavor="ref", cells=cells)
    return time.perf_counter() - t0


def cpu_baseline(eng, run, target_s: float = 12.0) -> dict:
    """The reference algorithm on the host (oracle, `kind: port`) over a
    bounded sample of the next coupled step of this run: a strided sample of
    the GPU's census and the same fraction of the step's volume sources,
    plus FP_calc of sampled zones."""
    import multiprocessing as mp
    from dataclasses import asdict
    sys.path.insert(0, str(ROOT / "tests"))
    import oracle_lib as OL
    OL.build()
    cores, nproc = cpu_share()
    wl = run.wl
    si_full = run.next_step_inputs()
    fp_call = run.fp_call_host() if run.fp_on else None
    n_cens = eng.census_count()
    grid_kw = {k: v for k, v in asdict(wl.grid).items()}
    # calibrate on a small sample, then size the sample for ~target_s per core
    def sample(frac):
        stride = max(1, int(round(1.0 / frac)))
        cens = eng.census_sample(0, stride, 1 << 62)
        si = run.sample_step(si_full, 1.0 / stride)
        return stride, cens, si
    stride, cens, si = sample(min(1.0, 2000.0 / max(n_cens, 1)))
    rc, st, dt = _cpu_transport((0, 1, grid_kw, si, cens))
    per_core_s = dt / max(1.0, len(cens[2]) + si.nsv.sum())
    items = n_cens + float(si_full.nsv.sum())
    frac = min(1.0, target_s * cores / max(per_core_s * items, 1e-9))
    stride, cens, si = sample(frac)
    ctx = mp.get_context("spawn")
    with ctx.Pool(cores) as pool:
        t0 = time.perf_counter()
        res = pool.map(_cpu_transport, [(r, cores, grid_kw, si, cens) for r in range(cores)])
        wall = time.perf_counter() - t0
        if any(r[0] != 0 for r in res):
            raise RuntimeError("cpu baseline oracle failed: %s" % [r[0] for r in res])
        tr_steps = sum(r[1] for r in res)
        tr_s = max(r[2] for r in res)
        fp_s_zone = 0.0
        nfp = 0
        if fp_call is not None:
            ncell = wl.grid.nz * wl.grid.nr
            cells = list(range(0, ncell, max(1, ncell // cores)))[:cores]
            fp_t = pool.map(_cpu_fp, [(grid_kw, wl.fp_const, fp_call, [c]) for c in cells])
            fp_s_zone = float(np.mean(fp_t))
            nfp = len(cells)
    ncell = wl.grid.nz * wl.grid.nr
    step_s = tr_s * stride + fp_s_zone * ncell / cores
    cpu_steps = tr_steps * stride                # the whole step's packet-steps on the CPU
    return {"value": cpu_steps / step_s, "unit": "packet-steps/s", "cores": cores, "kind": "port",
            "sample": ("the C3 step after this run's last timed step: every %d-th census record "
                       "the GPU left (%d of %d) + 1/%d of the step's volume sources, lineage-sharded "
                       "over %d processes (host nproc %d, CPU share %d); C oracle = port of the "
                       "reference algorithm (exact 199-term comtot, glibc libm, lineage RNG): %.0f "
                       "packet-steps in %.2f s; FP_calc of %d zones at %.2f s/zone; whole coupled "
                       "step extrapolated = %.2f s x %d + %.2f s/zone x %d zones / %d cores = %.1f s "
                       "for %.3g packet-steps (pool wall %.1f s)"
                       % (stride, len(cens[2]), n_cens, stride, cores, nproc, cores, tr_steps,
                          tr_s, nfp, fp_s_zone, tr_s, stride, fp_s_zone, ncell, cores, step_s,
                          cpu_steps, wall))}


def load_pmc(workload_key: str):
    """Per-packet-step counters of the generation-0 transport launch and the
    FP kernel's issue figures, from the committed rocprofv3 PMC summary
    (tools/gpu_profile.sh + tools/pmc_summary.py: separate FETCH_SIZE,
    WRITE_SIZE and SQ passes; FETCH_SIZE doubled for gfx950)."""
    p = ROOT / "profiles" / "pmc_latest.json"
    if not p.exists():
        return {}
    try:
        d = json.loads(p.read_text())
        return d if d.get("workload_key") == workload_key else {}
    except Exception:
        return {}


def build_c2(args, rank, world, local, total_steps, sources, grid_n, ccap, ecap):
    from compton2d_amd import abi, synth
    mode = abi.COMTOT_TABLE if args.mode == "fast" else abi.COMTOT_EXACT
    return synth.c2_workload(nz=grid_n, nr=grid_n, sources=sources * world, comtot_mode=mode,
                             rank=rank, world=world, device=local, census_capacity=ccap,
                             event_capacity=ecap)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--workload", choices=("c3", "c2", "c4"), default="c3")
    ap.add_argument("--sources", type=int, default=None, help="volume packets/step/GPU")
    ap.add_argument("--grid", type=int, default=32, help="c2/c4 grid (NxN)")
    ap.add_argument("--mode", choices=("fast", "exact"), default="fast")
    ap.add_argument("--host-tables", action="store_true",
                    help="c3: move tables/electrons through host arrays every step")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    args = ap.parse_args()

    import torch
    from compton2d_amd import abi, distributed, synth
    from compton2d_amd.coupled import CoupledRun
    from compton2d_amd.engine import Engine

    rank, world, local = distributed.init()
    if world != args.gpus and world > 1:
        raise SystemExit("bench: --gpus %d but WORLD_SIZE=%d" % (args.gpus, world))
    if not torch.cuda.is_available():
        raise SystemExit("bench: no GPU visible")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    wk = args.workload
    sources = args.sources or DEFAULT_SOURCES[wk]
    total_steps = args.warmup + args.steps
    # census SoA in + out: as many records as the run can create, within ~70 %
    # of the free HBM (288 GB per MI355X); events and the packet store beside it
    free, _ = torch.cuda.mem_get_info(dev)
    ecap = int(2 * sources) + (1 << 20)
    side = ecap * 56 + sources * 80 + (4 << 30)
    ccap = int(min((total_steps + 1) * sources * 1.1 + (1 << 20),
                   max(1 << 20, (0.85 * free - side) / CENSUS_BYTES)))
    mode = abi.COMTOT_TABLE if args.mode == "fast" else abi.COMTOT_EXACT
    T = None
    if wk == "c3":
        wl = synth.c3_workload(sources=sources * world, comtot_mode=mode, rank=rank, world=world,
                               device=local, census_capacity=ccap, event_capacity=ecap)
        eng = Engine(wl.grid)
        T = torch.zeros(eng.layout.total, dtype=torch.float64, device=dev)
        eng.use_tally_tensor(T)
        run = CoupledRun(eng, wl, device_resident=not args.host_tables,
                         allreduce=(lambda: distributed.allreduce_tallies(T)) if world > 1 else None)
        one_step = run.step
        desc = wl.description
    else:
        grid_n = args.grid
        wl = build_c2(args, rank, world, local, total_steps, sources, grid_n, ccap, ecap)
        eng = Engine(wl.grid)
        T = torch.zeros(eng.layout.total, dtype=torch.float64, device=dev)
        eng.use_tally_tensor(T)
        eng.set_step(wl.step0)
        state = {"n": 0}
        cnt0 = eng.layout.counters

        def one_step():
            ncycle, t = wl.clock(state["n"])
            eng.set_clock(ncycle, t, wl.dt)
            eng.run_step()
            distributed.allreduce_tallies(T)
            state["n"] += 1
            c = T[cnt0:cnt0 + abi.NCOUNTERS].cpu().numpy()
            g0, al, _ = eng.last_kernel_ms()
            return dict(packet_steps=float(c[abi.CNT_STEPS]), sources=float(c[abi.CNT_SOURCES]),
                        census=float(c[abi.CNT_CENSUS]), escapes=float(c[abi.CNT_ESCAPES]),
                        aborted=float(c[abi.CNT_ABORTED]), transport_gen0_ms=g0,
                        transport_all_ms=al, gen0_steps=float(eng.last_gen0_steps()),
                        gen0_paths=float(eng.last_path_steps()[0]),
                        all_paths=float(eng.last_path_steps()[1]))
        desc = wl.description.replace("C2:", "C4 (C2 medium, per GPU):") if wk == "c4" else wl.description

    for _ in range(args.warmup):
        one_step()
    distributed.barrier(dev)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    rows = []
    for _ in range(args.steps):
        rows.append(dict(one_step()))
    torch.cuda.synchronize()
    distributed.barrier(dev)
    elapsed = time.perf_counter() - t0
    elapsed = distributed.allreduce_max(elapsed, dev)
    # packet-steps of all ranks: the counters were all-reduced with the tallies
    steps_global = sum(r["packet_steps"] for r in rows)
    if world > 1 and wk == "c3":
        pass   # CoupledRun reads the counters after its all-reduce hook: already global
    if rank != 0:
        eng.close()
        return
    g0_ms = sum(r["transport_gen0_ms"] for r in rows)
    g0_steps = sum(r["gen0_steps"] for r in rows)
    g0_paths = sum(r["gen0_paths"] for r in rows)
    value = steps_global / elapsed
    # algorithmic bytes: SURVEY.md §8(d)'s 80-B packet record in + out per
    # pass of a packet through the geometry block.  A probe bundle carries all
    # the copies on its path through ONE pass, so the bytes a
    # streamed design would move for this launch are 160 B per lane
    # path-step; the per-copy count (the metric's unit) would exceed the
    # chip's peak and is reported beside it only as `survey_formula_frac`.
    g0_s = g0_ms * 1e-3
    achieved = g0_paths * BYTES_PER_STEP / g0_s / 1e9 if g0_ms > 0 else 0.0
    survey_frac = (g0_steps * BYTES_PER_STEP / g0_s / 1e9 / HBM_PEAK_GBS) if g0_ms > 0 else 0.0
    grid_txt = "30x9" if wk == "c3" else "%dx%d" % (args.grid, args.grid)
    workload_key = "%s_%s_%d_%s" % (wk, grid_txt, sources, args.mode)
    pmc = load_pmc(workload_key)
    bpp = pmc.get("hbm_bytes_per_path")
    steps_per_launch = g0_steps / args.steps
    paths_per_launch = g0_paths / args.steps
    traffic = bpp * paths_per_launch if bpp is not None else None
    # VALU issue: wave-instructions per path-step (PMC SQ_INSTS_VALU) at the
    # achieved rate vs 1024 SIMDs x one wave64 VALU instruction per 4 cycles
    vpp = pmc.get("valu_wave_insts_per_path")
    g0_rate = g0_steps / g0_s if g0_ms > 0 else 0.0
    g0_prate = g0_paths / g0_s if g0_ms > 0 else 0.0
    valu_frac = (g0_prate * vpp / (N_SIMD * CLOCK_HZ / 4.0)) if vpp else None
    per_step = {k: float(np.mean([r[k] for r in rows])) for k in rows[0]
                if isinstance(rows[0][k], (int, float))}
    kernels = {
        "transport_gen0": {"ms_avg": g0_ms / args.steps, "packet_steps_per_launch": steps_per_launch,
                           "path_steps_per_launch": paths_per_launch,
                           "packet_steps_per_path": (g0_steps / g0_paths) if g0_paths else None,
                           "packet_steps_per_s": g0_rate, "path_steps_per_s": g0_prate,
                           "bound": "issue/latency (packet state in VGPRs); reported against HBM",
                           "hbm_frac_algorithmic": achieved / HBM_PEAK_GBS,
                           "hbm_frac_measured": (bpp * g0_prate / 1e9 / HBM_PEAK_GBS) if bpp else None,
                           "valu_issue_frac": valu_frac},
        "transport_all_generations": {"ms_avg": per_step.get("transport_all_ms")},
    }
    if wk == "c3":
        fp_ms = per_step.get("fp_kernel_ms", 0.0)
        ncell = wl.grid.nz * wl.grid.nr
        kernels["fp"] = {"ms_avg": fp_ms, "zones": ncell,
                         "bound": "latency: in-order recurrences per zone (SURVEY a15)",
                         "simd_occupancy": pmc.get("fp_simd_occupancy"),
                         "valu_issue_frac": pmc.get("fp_valu_issue_frac"),
                         "wait_frac": pmc.get("fp_wait_frac")}
        kernels["volume_em"] = {"ms_avg": per_step.get("vem_kernel_ms", 0.0), "zones": ncell}
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
        "data": ("synthetic: the reference's P_nontherm electrons of the inputm.dat medium in every "
                 "zone, tables recomputed on the device every step from the evolving electrons; "
                 "volume packets sampled on device" if wk == "c3" else
                 "synthetic: reference volume_em/P_nontherm tables of the inputm.dat medium tiled "
                 "over the grid; volume packets sampled on device"),
        "config": {
            "workload": desc,
            "grid": grid_txt,
            "sources_per_gpu_per_step": sources,
            "fp": wk == "c3",
            "comtot": ("table (cubic in ln E, 2048 pts per cell, f64)" if mode == abi.COMTOT_TABLE
                       else "exact 199-term sum"),
            "arithmetic": "f64 throughout (comtot table stored in f64)",
            "tables": ("device-resident (C2D_DEV_EMISSION | C2D_DEV_ELECTRONS)"
                       if wk == "c3" and not args.host_tables else "host arrays"),
            "parallelism": "lineage-sharded sources, %d rank(s), RCCL all-reduce of tallies" % world,
            "census_capacity_per_gpu": ccap,
            "packet_steps_timed": steps_global,
            "per_step": per_step,
        },
        "roofline": {
            "bound": "hbm",
            "achieved": achieved,
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS,
            "traffic": traffic,
            "kernel": "c2d_bundle_kernel_%s (generation 0)" % args.mode,
            "per_unit_bytes": BYTES_PER_STEP,
            "unit_of_work": "lane path-step (one pass through imctrk2d.f:228-379 shared by the copies "
                            "on the path; c2d_last_path_steps)",
            "kernel_ms_avg": g0_ms / args.steps,
            "traffic_unit": "bytes per launch (PMC FETCH_SIZEx2 + WRITE_SIZE), from %s" %
                            (pmc.get("source") or "no PMC profile of this workload"),
            "traffic_bytes_per_path": bpp,
            "valu_issue_frac": valu_frac,
            "steps_per_launch_avg": steps_per_launch,
            "paths_per_launch_avg": paths_per_launch,
            "survey_formula_frac": survey_frac,
        },
        "kernels": kernels,
        "cpu_baseline": None,
    }
    if world == 1 and not args.no_cpu_baseline and wk == "c3":
        out["cpu_baseline"] = cpu_baseline(eng, run, args.cpu_seconds)
    print(json.dumps(out))
    eng.close()


if __name__ == "__main__":
    main()
