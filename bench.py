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
carried from step to step.  `--gpus N` runs the same per-GPU workload on every
rank (weak scaling: 1e8 sources per GPU per step, lineage-sharded, one RCCL
all-reduce of the tally buffer per step), so the per-N lines compare.
`--workload c2` is the 32x32 FP-off transport workload of round 1;
`--workload c4` is C2's medium at C4's 1.25e8 sources per GPU (1e9 per step
on 8 GPUs, BASELINE configs[3]).

    python bench.py [--gpus N --steps K --warmup W] [--workload c3|c2|c4]
    torchrun --nproc-per-node N bench.py --gpus N ...   (one rank per GPU)

Rank 0 prints ONE JSON line.  `value` = packet-steps of all ranks / the max
over ranks of the wall time of the K timed steps.  `roofline` prices the
dominant kernel (generation-0 transport launch) at 160 algorithmic bytes
(an 80-B packet record in + out) per lane path-step, the
pass through the geometry block that a probe bundle shares among its copies,
and carries its measured HBM bytes and VALU-issue fraction from the committed
PMC profile of the same command; `kernels` reports the FP and table kernels beside it;
`cpu_baseline` times the reference's algorithm (the C oracle in its
reference mode: per-copy probes, lagged-Fibonacci streams with the
per-census-packet reseed, bit-exact to the Fortran) on the host's CPU share,
on a strided sample of the GPU's own final census plus the same fraction of
the step's volume sources, and the FP_calc of sampled zones, extrapolated to
one whole coupled step.
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
# census bytes per record of capacity (c2d_device.hpp CensusSoA, capi.cpp cens_phys):
# double-buffered in + out, or in place + 1/16 append slack
CENSUS_BYTES = {0: 2 * 64, 1: 64 * (1 + 1 / 16)}
DEFAULT_SOURCES = {"c3": 100_000_000, "c2": 10_000_000, "c4": 125_000_000, "c5": 20_000_000}
# untimed census spin-up (steps before the warm-up): a C3 source stays in the
# census ~16 steps (tools/c3_bench.py: the census saturates at 15.8 records
# per source of a step after ~40 steps, profiles/r03a), so the timed steps
# see the steady-state census of a long run instead of its growth
SPINUP = {"c3": 40, "c4": 60, "c2": 0, "c5": 0}
# in-place census by default where the double buffer cannot hold the run: C4's
# 1.25e8 sources per GPU on the 32x32 C2 medium saturate at 22.6 census
# records per source of a step (2.8e9, tools/census_traj.py, profiles/r03e)
INPLACE = {"c3": 0, "c4": 1, "c2": 0, "c5": 0}
# census records per source of a step the capacity is sized for
CENSUS_PER_SOURCE = {"c3": 20.0, "c4": 26.0, "c2": 40.0, "c5": 8.0}


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
    """One host core = one reference worker: the C oracle in its reference
    mode (glibc libm, exact comtot, per-copy split1 probes, the reference's
    lagged-Fibonacci streams with the per-census-packet reseed of
    src/imcfield2d.f:115-116) on its share of the sampled step: every
    world-th census record and the volume zones j*nr+k = rank (mod world),
    as the reference's master hands zone jobs to its workers."""
    import dataclasses
    rank, world, grid_kw, si, cens = args
    sys.path.insert(0, str(ROOT / "tests"))
    import oracle_lib as OL
    from compton2d_amd import abi
    g = abi.GridConfig(**grid_kw)
    g.rank, g.world, g.comtot_mode = 0, 1, abi.COMTOT_EXACT
    o = OL.Oracle(g, OL.RNG_FIB, "ref", rseed=9857 + 7919 * rank)
    d6, i5, keys = cens
    # census seeds: the reference stores int(fibran()*1e5) (imctrk2d.f:571, hazard H5)
    o.import_census(d6[rank::world], i5[rank::world], (keys[rank::world] % 100000).astype(np.uint64))
    nsv = np.asarray(si.nsv).copy()
    cells = np.arange(nsv.size).reshape(nsv.shape)
    nsv[cells % world != rank] = 0
    t0 = time.perf_counter()
    rc = o.step(dataclasses.replace(si, nsv=nsv))
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
    """The reference algorithm on the host (the C oracle in its reference
    mode, `kind: port`) over a bounded sample of the next coupled step of
    this run: a strided sample of the GPU's census and the same fraction of
    the step's volume sources, plus FP_calc of sampled zones."""
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
    # the port's speed against the reference's own Fortran on the same C3
    # transport work (bitwise-identical histories, one process each; measured
    # in the build container by tools/fortran_vs_port.py: the Fortran does not
    # travel to this box)
    fvp = None
    fp_path = ROOT / "profiles" / "r06c" / "fortran_vs_port.json"
    if fp_path.exists():
        fvp = json.loads(fp_path.read_text())
    return {"value": cpu_steps / step_s, "unit": "packet-steps/s", "cores": cores, "kind": "port",
            "algorithm": "the reference's algorithm restated in C (oracle/c2d_oracle.c reference mode: "
                         "per-copy split1 probes, lagged-Fibonacci streams reseeded per census packet, "
                         "exact comtot, glibc libm); bit-exact results, not the Fortran's code or speed",
            "port_speed_vs_fortran": None if fvp is None else round(fvp["port_speed_vs_fortran"], 3),
            "port_speed_source": None if fvp is None else (
                "profiles/r06c/fortran_vs_port.json: the C3 deck (nst %d, %d steps, %.3g packet-steps), "
                "Fortran %.3g vs port %.3g packet-steps/s on one core each, bitwise-identical tallies and "
                "census" % (fvp["nst"], fvp["steps"], fvp["packet_steps"], fvp["fortran_packet_steps_per_s"],
                            fvp["port_packet_steps_per_s"])),
            "sample": ("the C3 step after this run's last timed step: every %d-th census record "
                       "the GPU left (%d of %d) + 1/%d of the step's volume sources, over %d "
                       "processes = reference workers (census records strided, volume zones "
                       "j*nr+k mod %d; host nproc %d, CPU share %d); C oracle in its reference mode "
                       "= the reference's algorithm restated in C (per-copy split1 probes, "
                       "no bundles; rand_switch=1 lagged-Fibonacci zone streams and the 10000-number "
                       "reseed per census packet, src/imcfield2d.f:115-116; exact 199-term comtot; "
                       "glibc libm; bit-exact to the Fortran in tests/test_oracle_golden.py; see "
                       "port_speed_vs_fortran for its speed against the Fortran): %.0f "
                       "packet-steps in %.2f s; FP_calc of %d zones at %.2f s/zone; whole coupled "
                       "step extrapolated = %.2f s x %d + %.2f s/zone x %d zones / %d cores = %.1f s "
                       "for %.3g packet-steps (pool wall %.1f s)"
                       % (stride, len(cens[2]), n_cens, stride, cores, cores, nproc, cores, tr_steps,
                          tr_s, nfp, fp_s_zone, tr_s, stride, fp_s_zone, ncell, cores, step_s,
                          cpu_steps, wall))}


def fp_offclamp(device: int, cpu: bool) -> dict:
    """One FP update off the temperature clamp, outside the timed steps (C3's
    zones all sit on the reference's 1000 keV clamp, so the coupled step's FP
    is the cheap case).  The workload of tools/fp_bench.py --vary: the
    reference's fp_pick FP inputs tiled over 30x9 with n_e and tea varied per
    zone, so no two zones share a temperature-search chain (2 391 implicit
    sub-steps per zone).  On fresh contexts, i.e. with an empty gamma_bar
    memo: the fast mode's first update (zones costliest first by the cost
    probe; the same update in index order without it on a second context), a
    second with the memo emptied again (zones in the measured, costliest-first
    order) and a third with the memo warm; the exact mode's first update.  The fast mode
    takes McDonald pairs from its moment table (fp_fast.hip mcd_mtab, built in
    c2d_fp_set_config: config_wall_ms), so a cold memo costs it little.  cpu: the C
    oracle's FP_calc on 8 zones of the same tile, one process each (the
    bench's cpu_baseline leg)."""
    sys.path.insert(0, str(ROOT / "tools"))
    import fp_bench
    from compton2d_amd import abi
    from compton2d_amd.engine import Engine
    c, g, tile = fp_bench.tiled_case(30, 9, "fp_pick", vary=True)
    g.device = device
    out = {"workload": "tools/fp_bench.py --nz 30 --nr 9 --vary: the reference's fp_pick FP inputs "
                       "(tests/golden/fp_pick.npz) tiled over 30x9, n_e and tea varied per zone",
           "zones": 30 * 9, "timed_in_value": False}
    call = (tile["ncycle"], tile["time"], tile["dt"], tile, tile)
    for mode in ("fast", "exact"):
        eng = Engine(g)
        try:
            t0 = time.perf_counter()
            eng.fp_set_config(c.constants())
            setup_ms = 1e3 * (time.perf_counter() - t0)
            eng.fp_set_mode(abi.FP_FAST if mode == "fast" else abi.FP_EXACT)
            r = eng.fp_step(*call)
            leg = {"ms_first_update": eng.last_fp_ms(),
                   "config_wall_ms": setup_ms,
                   "implicit_substeps": float(np.sum(r["zone_diag"][..., 5])),
                   "Te_new_range": [float(r["Te_new"].min()), float(r["Te_new"].max())]}
            if mode == "fast":
                leg["first_update_order"] = ("costliest first by the cost probe (every zone's first "
                                             "implicit sub-step, 1/f_t_implicit)")
                # the same first update without the probe: one workgroup per zone in index order
                e2 = Engine(g)
                try:
                    os.environ["C2D_FPF_PROBE"] = "0"
                    e2.fp_set_config(c.constants())
                    e2.fp_set_mode(abi.FP_FAST)
                    e2.fp_step(*call)
                    leg["ms_first_update_index_order"] = e2.last_fp_ms()
                finally:
                    del os.environ["C2D_FPF_PROBE"]
                    e2.close()
                os.environ["C2D_FPF_MEMO_RESET"] = "1"
                try:
                    eng.fp_step(*call)
                    leg["ms_cold_measured_order"] = eng.last_fp_ms()
                finally:
                    del os.environ["C2D_FPF_MEMO_RESET"]
                eng.fp_step(*call)
                leg["ms_warm"] = eng.last_fp_ms()
                leg["kernel"] = "c2d_fp_fast_kernel<256> (C2D_FP_FAST; stated tolerance)"
            else:
                leg["kernel"] = "c2d_fp_kernel (C2D_FP_EXACT; bit for bit)"
            out[mode] = leg
        finally:
            eng.close()
    if cpu:
        import multiprocessing as mp
        cores = min(8, cpu_share()[0])
        jobs = [(30, 9, (i, i + 1), "fp_pick", True) for i in range(cores)]
        t0 = time.perf_counter()
        with mp.get_context("spawn").Pool(cores) as pool:
            res = pool.map(fp_bench._cpu_zone, jobs)
        wall = time.perf_counter() - t0
        per_zone = float(np.mean([x[0] for x in res]))
        out["cpu_baseline"] = {"s_per_zone": per_zone, "zones_per_s_per_core": 1.0 / per_zone,
                               "cores": cores, "kind": "port",
                               "sample": "FP_calc of zones (0, 0..%d) of the tile, one process each "
                                         "(C oracle, det math), pool wall %.1f s" % (cores - 1, wall)}
    return out


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


def census_capacity(sources: int, per_source: float, free: float, side: float, inplace: int) -> int:
    """Census records the run may hold: per_source x sources, within 85 % of
    the free HBM beside the event and packet buffers."""
    return int(min(per_source * sources + (1 << 20),
                   max(1 << 20, (0.85 * free - side) / CENSUS_BYTES[inplace])))


def tally_exchange(eng, T, rank, world, dev):
    """The per-step tally all-reduce of an N-rank run (xec_add / cens_add_up):
    by default RCCL inside the C-ABI (c2d_comm_init + c2d_allreduce_tallies on
    the library's stream, the Fortran host's path); `C2D_TALLY_EXCHANGE=torch`
    or a gloo process group (the one-GPU rehearsal) use torch.distributed."""
    from compton2d_amd import abi, distributed
    if world == 1:
        return None, "none (1 rank)"
    import torch.distributed as dist
    if dist.get_backend() == "nccl" and os.environ.get("C2D_TALLY_EXCHANGE", "cabi") == "cabi":
        obj = [eng.comm_unique_id() if rank == 0 else bytes(abi.COMM_ID_BYTES)]
        dist.broadcast_object_list(obj, src=0, device=dev)
        eng.comm_init(obj[0], rank, world)
        return eng.allreduce_tallies, "RCCL all-reduce inside the C-ABI (c2d_allreduce_tallies)"
    return (lambda: distributed.allreduce_tallies(T)), \
        "torch.distributed all-reduce (%s)" % dist.get_backend()


def transport_row(eng, T, cnt0):
    """Per-step counters and kernel times of a transport-only step (after the
    tally exchange: the counters are global)."""
    from compton2d_amd import abi
    c = T[cnt0:cnt0 + abi.NCOUNTERS].cpu().numpy()
    g0, al, _ = eng.last_kernel_ms()
    g0p, allp = eng.last_path_steps()
    return dict(packet_steps=float(c[abi.CNT_STEPS]), sources=float(c[abi.CNT_SOURCES]),
                census=float(c[abi.CNT_CENSUS]), escapes=float(c[abi.CNT_ESCAPES]),
                aborted=float(c[abi.CNT_ABORTED]), transport_gen0_ms=g0, transport_all_ms=al,
                gen0_steps=float(eng.last_gen0_steps()), gen0_paths=float(g0p),
                all_paths=float(allp), census_records=float(eng.census_count()))


def build_c3(args, rank, world, local, dev, sources, ccap, ecap, mode):
    import torch
    from compton2d_amd import synth
    from compton2d_amd.coupled import CoupledRun
    from compton2d_amd.engine import Engine
    wl = synth.c3_workload(sources=sources * world, comtot_mode=mode, rank=rank, world=world,
                           device=local, census_capacity=ccap, event_capacity=ecap)
    wl.grid.census_inplace = args.inplace
    eng = Engine(wl.grid)
    T = torch.zeros(eng.layout.total, dtype=torch.float64, device=dev)
    eng.use_tally_tensor(T)
    ex, ex_desc = tally_exchange(eng, T, rank, world, dev)
    from compton2d_amd import abi
    fpm = {"auto": abi.FP_AUTO, "exact": abi.FP_EXACT, "fast": abi.FP_FAST}[args.fp_mode]
    # C3's named output: the step's escapes binned into the observer-frame SED
    # of postprocessing/mrk421_sed.input (pspt.c:245-294) on the device, from
    # the event buffer the transport just wrote (no event text, no download),
    # on a second stream beside the census close, the FP update and the next
    # step's tables
    from compton2d_amd import observer
    eng.obs_begin(observer.mrk421_sed_binning())
    run = CoupledRun(eng, wl, device_resident=not args.host_tables, allreduce=ex, fp_mode=fpm,
                     after_transport=lambda: eng.obs_accumulate(None))

    def one_step():
        r = dict(run.step())
        r["census_records"] = float(eng.census_count())
        r["escape_events"] = float(eng.last_event_count())
        return r
    return eng, run, one_step, wl, wl.description + "; every step's escapes binned on the device " \
        "into the mrk421_sed.input SED (pspt.c)", ex_desc


def build_c2(args, rank, world, local, dev, sources, ccap, ecap, mode):
    """C2 (32x32, 1e7/step, FP off) and C4 (C2's medium at 1.25e8 per GPU)."""
    import torch
    from compton2d_amd import synth
    from compton2d_amd.engine import Engine
    wl = synth.c2_workload(nz=args.grid, nr=args.grid, sources=sources * world, comtot_mode=mode,
                           rank=rank, world=world, device=local, census_capacity=ccap,
                           event_capacity=ecap)
    wl.grid.census_inplace = args.inplace
    eng = Engine(wl.grid)
    T = torch.zeros(eng.layout.total, dtype=torch.float64, device=dev)
    eng.use_tally_tensor(T)
    ex, ex_desc = tally_exchange(eng, T, rank, world, dev)
    eng.set_step(wl.step0)
    state = {"n": 0}
    cnt0 = eng.layout.counters

    def one_step():
        ncycle, t = wl.clock(state["n"])
        eng.set_clock(ncycle, t, wl.dt)
        eng.run_step()
        if ex is not None:
            ex()
        state["n"] += 1
        return transport_row(eng, T, cnt0)
    desc = wl.description
    if args.workload == "c4":
        desc = ("C4: C2's medium (%dx%d, inputm.dat, FP off) at %d volume packets/step per GPU, "
                "lineage-sharded over %d rank(s) (%d per step in all; BASELINE configs[3] is 1e9 "
                "on 8 GPUs), tallies all-reduced every step" % (args.grid, args.grid, sources, world,
                                                              sources * world))
    return eng, None, one_step, wl, desc, ex_desc


def build_c5(args, rank, world, local, dev, sources, ccap, ecap, mode):
    """C5 (BASELINE configs[4]): the external-Compton BLR light-curve run of
    tools/c5_bench.py as a bench workload.  Every step: host budgets (file_sp
    + the lower-ring EC budget, imcsurf2d_para.f:544-685, imcgen2d.f:111-120,
    174-183), census + volume + surface transport on the GPU, the tally
    exchange, and the observer-frame light curves of the step's escapes
    binned on the device (postprocessing/plcm.c:382-456, ext25_lc.input)."""
    import torch
    from compton2d_amd import surface, synth
    from compton2d_amd.engine import Engine
    sys.path.insert(0, str(ROOT / "tools"))
    import c5_bench as C5
    nz = nr = args.grid_c5
    nst = sources * world
    g_bulk, zmax, rmax, rmin = 25.0, 1.0e17, 1.0e17, 0.0
    wl = synth.c2_workload(nz=nz, nr=nr, sources=nst, comtot_mode=mode, rank=rank, world=world,
                           device=local, census_capacity=ccap, event_capacity=ecap)
    wl.grid.census_inplace = args.inplace
    z, r, vol, zs = synth.zone_geometry(nz, nr, zmax, rmin, rmax)
    wl.grid.z, wl.grid.r = z, r
    dt = min(r[-1] / nr, z[-1] / nz) / (np.sqrt(1.0 - 1.0 / g_bulk ** 2) * synth.C_LIGHT)
    med = np.load(synth.DATA, allow_pickle=False)
    fas = med["emiss_per_vol_per_s"] * vol * dt
    nsv = (0.5 * nst * fas / fas.sum()).astype(np.int64)            # imcgen2d.f:446
    ewsv = np.where(nsv > 0, fas / np.maximum(nsv, 1), 0.0)
    tab, int_file = surface.file_sp(surface.seed_spectrum("blackbody_G25_4spectra"),
                                    surface.EcConstants(g_bulk=g_bulk))
    eng = Engine(wl.grid)
    T = torch.zeros(eng.layout.total, dtype=torch.float64, device=dev)
    eng.use_tally_tensor(T)
    ex, ex_desc = tally_exchange(eng, T, rank, world, dev)
    eng.obs_begin(C5.ext25_binning())
    cnt0 = eng.layout.counters
    state = {"n": 0}

    def one_step():
        n = state["n"]
        ncycle, t = n, max(n - 1, 0) * dt
        w = surface.time_window(ncycle, t, dt, C5.T1)
        ec_on = w < len(C5.T0) and (t + 0.5 * dt) >= C5.T0[w]
        tbbl = np.full(nr, -1.0) if w == 0 else np.zeros(nr)
        nsurfl, ewsurfl = surface.lower_surface_budget(r, rmin, nst, dt, tbbl, ec_on, int_file)
        si = wl.step0
        si.ncycle, si.time, si.dt = ncycle, t, dt
        si.zsurf, si.Eloss_tot, si.Eloss_th = zs, fas, fas * float(med["Eloss_th_frac"])
        si.nsv, si.ewsv = nsv.astype(np.int32), ewsv
        si.nsurfl, si.ewsurfl, si.tbbl = nsurfl, ewsurfl, tbbl
        si.spectra = [tab]
        surface.apply_bias(nst, si)
        eng.transport_step(si)
        if ex is not None:
            ex()
        eng.obs_accumulate(None)
        state["n"] += 1
        row = transport_row(eng, T, cnt0)
        row["surface_sources"] = float(nsurfl.sum())
        return row
    desc = ("C5: EC/BLR light curve, %dx%d grid, z_max=r_max=1e17 cm, Gamma 25, "
            "disk/blackbody_G25_4spectra.in on all %d lower rings (EC window t < 4e5 s), nst=%d per "
            "GPU (nst surface + nst/2 volume packets), %d rank(s), ext25_lc light curves binned on "
            "the device every step" % (nz, nr, nr, sources, world))
    return eng, None, one_step, wl, desc, ex_desc


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--workload", choices=("c3", "c2", "c4", "c5"), default=None,
                    help="default: c3 at every N (weak scaling: the same per-GPU workload, so the "
                         "driver's per-N values compare); c4 = BASELINE configs[3]'s 1.25e8 per GPU "
                         "on the 32x32 medium")
    ap.add_argument("--sources", type=int, default=None, help="volume packets/step/GPU (c5: nst/GPU)")
    ap.add_argument("--spinup", type=int, default=None,
                    help="untimed steps before the warm-up that bring the census to its steady "
                         "state (default: c3 %d, c4 %d, else 0)" % (SPINUP["c3"], SPINUP["c4"]))
    ap.add_argument("--census-inplace", type=int, choices=(0, 1), default=None,
                    help="1: one in-place census SoA (half the memory), 0: in + out buffers "
                         "(default: 1 for c4, else 0)")
    ap.add_argument("--grid", type=int, default=32, help="c2/c4 grid (NxN)")
    ap.add_argument("--grid-c5", type=int, default=16, help="c5 grid (NxN)")
    ap.add_argument("--mode", choices=("fast", "exact"), default="fast")
    ap.add_argument("--fp-mode", choices=("auto", "exact", "fast"), default="auto",
                    help="C3: the coupled step's FP update (auto: C2D_FP_AUTO, exact while every "
                         "zone sits on the tea clamp -- C3's steady state -- fast off it; exact: "
                         "bit-identical to the oracle)")
    ap.add_argument("--host-tables", action="store_true",
                    help="c3: move tables/electrons through host arrays every step")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-fp-offclamp", action="store_true",
                    help="c3: skip the untimed off-clamp FP update (kernels.fp_offclamp)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--dump", default=None,
                    help="directory: each rank writes rank<r>.npz with the last timed step's tally "
                         "buffer, and for c3 the timed steps' SED sums and the electron state "
                         "(the N-rank rehearsal compares them, tests/test_gpu_bench_ranks.py)")
    args = ap.parse_args()

    import torch
    from compton2d_amd import abi, distributed

    rank, world, local = distributed.init()
    if world != args.gpus and world > 1:
        raise SystemExit("bench: --gpus %d but WORLD_SIZE=%d" % (args.gpus, world))
    if not torch.cuda.is_available():
        raise SystemExit("bench: no GPU visible")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    wk = args.workload or "c3"
    args.workload = wk
    sources = args.sources or DEFAULT_SOURCES[wk]
    spinup = SPINUP.get(wk, 0) if args.spinup is None else args.spinup
    inplace = INPLACE[wk] if args.census_inplace is None else args.census_inplace
    total_steps = spinup + args.warmup + args.steps
    free, _ = torch.cuda.mem_get_info(dev)
    mode = abi.COMTOT_TABLE if args.mode == "fast" else abi.COMTOT_EXACT
    per_gpu_items = sources * (1.5 if wk == "c5" else 1.0)
    ecap = int(2 * per_gpu_items) + (1 << 20)
    side = ecap * 56 + per_gpu_items * 80 + (4 << 30)
    ccap = census_capacity(int(per_gpu_items), min(CENSUS_PER_SOURCE[wk], total_steps + 1), free, side,
                           inplace)
    args.inplace = inplace
    build = {"c3": build_c3, "c2": build_c2, "c4": build_c2, "c5": build_c5}[wk]
    eng, run, one_step, wl, desc, ex_desc = build(args, rank, world, local, dev, sources, ccap, ecap,
                                                  mode)

    t_spin = time.perf_counter()
    for _ in range(spinup):
        one_step()
    t_spin = time.perf_counter() - t_spin
    census_start = eng.census_count()
    for _ in range(args.warmup):
        one_step()
    distributed.barrier(dev)
    torch.cuda.synchronize()
    if wk == "c3":
        eng.obs_begin(eng._obs)            # the timed steps' SED alone (zeroes sums and kernel ms)
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
    census_timed_start = rows[0]["census_records"] if rows else census_start
    all_paths = distributed.allreduce_sum(float(sum(r["all_paths"] for r in rows)), dev)
    # fail loudly: a run that tracked nothing, or whose last step left NaN/Inf
    # in a tally, is no measurement (the library already refuses non-finite
    # tables and tallies with C2D_E_NONFINITE; this guards the line itself)
    last_tallies = eng.tallies_raw()
    if not (steps_global > 0 and elapsed > 0 and np.isfinite(last_tallies).all()):
        raise SystemExit("bench: invalid run on rank %d: %g packet-steps in %g s, %d non-finite tallies"
                         % (rank, steps_global, elapsed, int((~np.isfinite(last_tallies)).sum())))
    if args.dump:
        d = Path(args.dump)
        d.mkdir(parents=True, exist_ok=True)
        blob = {"tallies": last_tallies}
        if wk == "c3":
            F, F2, cnt, _ = eng.obs_result()
            f_nt, Pnt = run.electrons()
            blob.update(sed_F=F, sed_F2=F2, sed_count=cnt, f_nt=f_nt, Pnt=Pnt,
                        tea=np.asarray(run.state["tea"]), Te_new=np.asarray(run.state["Te_new"]))
        np.savez(d / ("rank%d.npz" % rank), **blob)
    if rank != 0:
        eng.close()
        return
    g0_ms = sum(r["transport_gen0_ms"] for r in rows)
    # this rank's own generation-0 work (its kernel time is this rank's)
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
    grid_txt = {"c3": "30x9", "c5": "%dx%d" % (args.grid_c5, args.grid_c5)}.get(
        wk, "%dx%d" % (args.grid, args.grid))
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
        modes = [r.get("fp_mode") for r in rows if r.get("fp_mode")]
        kernels["fp"] = {"ms_avg": fp_ms, "zones": ncell,
                         "mode": args.fp_mode,
                         "modes_run": {m: modes.count(m) for m in sorted(set(modes))},
                         "bound": "latency: in-order recurrences per zone (SURVEY a15)",
                         "simd_occupancy": pmc.get("fp_simd_occupancy"),
                         "valu_issue_frac": pmc.get("fp_valu_issue_frac"),
                         "wait_frac": pmc.get("fp_wait_frac")}
        kernels["volume_em"] = {"ms_avg": per_step.get("vem_kernel_ms", 0.0), "zones": ncell}
        _, _, sed_cnt, sed_ms = eng.obs_result()
        kernels["sed_binning"] = {
            "ms_avg": sed_ms / args.steps, "events_per_step": per_step.get("escape_events"),
            "binned_per_step": float(sed_cnt.sum()) / args.steps,
            "deck": "postprocessing/mrk421_sed.input (30 time bins 1.6e4-6e4 s, mu 0.99944-0.99964, "
                    "100 log channels 1e-7-1e10 keV)",
            "bound": "hbm: 56 B per escape event read once"}
    rounds, moved, phys = eng.last_compaction()
    chunks, recycled, unrecycled, held = eng.last_census_chunks()
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
        # the hardware rate beside the metric: lane path-steps (one pass of a
        # GPU lane through the geometry block, whatever the copies on it) of
        # all ranks and generations per second, and the copies a path carries
        "path_steps_per_s": all_paths / elapsed,
        "packet_steps_per_path": steps_global / all_paths if all_paths else None,
        "dtype": "f64",
        "data": {"c3": "synthetic: the reference's P_nontherm electrons of the inputm.dat medium in "
                       "every zone, tables recomputed on the device every step from the evolving "
                       "electrons; volume packets sampled on device",
                 "c5": "synthetic: reference volume_em/P_nontherm tables of the inputm.dat medium "
                       "tiled over the grid, the reference's blackbody_G25_4spectra.in seed file on "
                       "the lower rings; volume and surface packets sampled on device"}.get(
            wk, "synthetic: reference volume_em/P_nontherm tables of the inputm.dat medium tiled "
                "over the grid; volume packets sampled on device"),
        "config": {
            "workload": desc,
            "grid": grid_txt,
            "sources_per_gpu_per_step": sources,
            "fp": wk == "c3",
            "comtot": ("table (cubic in ln E, 2048 pts per cell, f64)" if mode == abi.COMTOT_TABLE
                       else "exact 199-term sum"),
            "arithmetic": ("f64 (geometry, positions, weights, tallies, the comtot table and its cubic "
                           "interpolation); three statistics-only quantities of the fast build in f32, each to "
                           "~1e-7 relative, inside the stated tolerance (tallies 1e-3, spectra <= 1 % L2 per "
                           "north_star): the probes' absorption points, which weight only prdep "
                           "(C2D_PT_F32), the bundle's optical depth -log(u)/n (C2D_TAU_F32) and the comtot "
                           "table coordinate ln xnu (C2D_LNX_F32); DESIGN.md section 2" if mode == abi.COMTOT_TABLE
                           else "f64 throughout (exact build, bit for bit with the oracle)"),
            "tables": ("device-resident (C2D_DEV_EMISSION | C2D_DEV_ELECTRONS)"
                       if wk == "c3" and not args.host_tables else "host arrays"),
            "parallelism": "lineage-sharded sources, %d rank(s), no data-path collective" % world,
            "tally_exchange": ex_desc,
            "census": {"spinup_steps": spinup, "spinup_s": t_spin,
                       "records_after_spinup": census_start,
                       "records_at_timed_start": census_timed_start,
                       "records_at_end": eng.census_count(),
                       "capacity_per_gpu": ccap, "physical_slots": phys,
                       "bytes_per_record_of_capacity": CENSUS_BYTES[inplace],
                       "layout": ("chunked: one SoA in 1024-record chunks, chunks of finished "
                                  "census sources refilled within the step (c2d_device.hpp C2D_CCHUNK)"
                                  if inplace else
                                  "double-buffered SoA (in + out), chunk tails compacted"),
                       "last_close_rounds": rounds, "last_close_moved": moved,
                       **({"chunks": chunks, "chunks_recycled_last_step": recycled,
                           "chunks_not_counted_down_last_step": unrecycled, "chunks_held": held}
                          if inplace else {})},
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
            # what binds the kernel: VALU issue (PMC SQ_INSTS_VALU per path-step
            # at the achieved rate) against one wave64 VALU op / 4 cycles / SIMD
            "issue_roof": {"bound": "valu_issue", "frac": valu_frac,
                           "valu_wave_insts_per_path": vpp,
                           "peak": "1024 SIMDs x 2.4 GHz / 4 cycles per wave64 VALU op",
                           "source": pmc.get("source")},
        },
        "kernels": kernels,
        "cpu_baseline": None,
    }
    if world == 1 and not args.no_cpu_baseline and wk == "c3":
        out["cpu_baseline"] = cpu_baseline(eng, run, args.cpu_seconds)
    if world == 1 and wk == "c3" and not args.no_fp_offclamp:
        kernels["fp_offclamp"] = fp_offclamp(local, cpu=not args.no_cpu_baseline)
    print(json.dumps(out))
    eng.close()


if __name__ == "__main__":
    main()
