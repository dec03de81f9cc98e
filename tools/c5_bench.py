#!/usr/bin/env python3
"""External-Compton light-curve run on the GPU (BASELINE.json configs[4]).

Every MC step, through the C-ABI:

    host   file_sp + lower-ring budgets (compton2d_amd/surface.py: imcsurf2d_para.f:544-685,
           imcgen2d.f:111-120,174-183,442,481-485), volume budgets (imcgen2d.f:446-456)
    GPU    c2d_transport_step: census + volume + surface transport (imcfield2d, imcvol2d,
           imcsurf2d -> r_surf_calc + file_sample on every lower ring)
    GPU    c2d_obs_accumulate: observer-frame light curves of the step's escapes
           (postprocessing/plcm.c:382-456), binned from the device event buffer

Set-up (synthetic, no network): Gamma = 25 with the reference's
`disk/blackbody_G25_4spectra.in` seed spectrum on every lower-boundary ring
(compton2d_amd/data/ec_seed_spectra.npz); two boundary windows, EC on for
t in [1, 4e5] s and off after (imcgen2d.f:174 gate `time + dt/2 >= t0`);
z_max = r_max = 1e17 cm; the inputm.dat medium in every zone (volume SSC
sources, compton2d_amd/data/medium_inputm.npz); the EC normalisation constants
of the golden EC case (surface.EcConstants); light curves binned as
`postprocessing/ext25_lc.input` (Gamma 25, r_max 1e17, mu in [0.9991, 0.9993),
2e4 s bins to 1.5e6 s, its 7 bands).  Multi-rank (torchrun): sources are
lineage-sharded by the library, tallies and light curves are summed over ranks.

    python tools/c5_bench.py [--sources 20000000] [--steps 6] [--warmup 1] [--grid 16]
"""
from __future__ import annotations

import argparse
import json
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT)]

# postprocessing/ext25_lc.input: (E_lower, E_upper) keV per band, one bin each, log spacing
EXT25_BANDS = ((1e-6, 3e-6), (1.25e-3, 1.9e-3), (1.9e-3, 7.5e-3), (1.5e-2, 2e-2), (1.0, 5.0),
               (1e3, 1e4), (1e5, 1e6))
EXT25 = dict(gam_bulk=25.0, rmax=1e17, mu_bins=((0.9991, 0.9993),), dt=2e4, t_offset=0.0,
             t_max=1.5e6)
T0, T1 = (1.0, 1.0e30), (4.0e5, 1.0e30)        # boundary windows: EC on, then off


def ext25_binning():
    from compton2d_amd import observer as O
    return O.lc_binning(regions=tuple((lo, hi, 1, False) for lo, hi in EXT25_BANDS), **EXT25)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sources", type=int, default=20_000_000, help="nst: packets/step (all ranks)")
    ap.add_argument("--census-per-source", type=int, default=8)
    ap.add_argument("--steps", type=int, default=6)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--grid", type=int, default=16)
    ap.add_argument("--lc-out", default="", help="directory for plcm-format light-curve files")
    args = ap.parse_args()
    import torch
    from compton2d_amd import abi, distributed, observer, surface, synth
    from compton2d_amd.engine import Engine

    rank, world, local = distributed.init()
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    nz = nr = args.grid
    nst = args.sources
    total = args.warmup + args.steps
    g_bulk, zmax, rmax, rmin = 25.0, 1.0e17, 1.0e17, 0.0
    per_rank = (2 * nst) // world + 1         # nst surface + nst/2 volume sources, sharded
    # census records per step: up to split1 per source plus the carried census
    wl = synth.c2_workload(nz=nz, nr=nr, sources=nst, comtot_mode=abi.COMTOT_TABLE, rank=rank,
                           world=world, device=local,
                           census_capacity=args.census_per_source * per_rank + (1 << 20),
                           event_capacity=per_rank + (1 << 20))
    # the C5 geometry and time step (setup2d.f:60-100; xec2d dt = mcdt*min(dr,dz)/v_bulk)
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
    binning = ext25_binning()
    eng.obs_begin(binning)
    cnt0 = eng.layout.counters
    rows = []
    for n in range(total):
        ncycle, t = n, max(n - 1, 0) * dt
        w = surface.time_window(ncycle, t, dt, T1)
        ec_on = w < len(T0) and (t + 0.5 * dt) >= T0[w]
        tbbl = np.full(nr, -1.0) if w == 0 else np.zeros(nr)
        nsurfl, ewsurfl = surface.lower_surface_budget(r, rmin, nst, dt, tbbl, ec_on, int_file)
        si = wl.step0
        si.ncycle, si.time, si.dt = ncycle, t, dt
        si.zsurf, si.Eloss_tot, si.Eloss_th = zs, fas, fas * float(med["Eloss_th_frac"])
        si.nsv, si.ewsv = nsv.astype(np.int32), ewsv
        si.nsurfl, si.ewsurfl, si.tbbl = nsurfl, ewsurfl, tbbl
        si.spectra = [tab]
        fb = surface.apply_bias(nst, si)
        distributed.barrier(dev)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        eng.transport_step(si)
        distributed.allreduce_tallies(T)
        t_tr = time.perf_counter() - t0
        t0 = time.perf_counter()
        eng.obs_accumulate(None)
        torch.cuda.synchronize()
        t_obs = time.perf_counter() - t0
        c = T[cnt0:cnt0 + abi.NCOUNTERS].cpu().numpy()
        rows.append(dict(ncycle=ncycle, time=t, ec_on=bool(ec_on and nsurfl.sum() > 0),
                         surface_sources=int(nsurfl.sum()), volume_sources=int(si.nsv.sum()),
                         fbias=fb, packet_steps=float(c[abi.CNT_STEPS]),
                         escapes=float(c[abi.CNT_ESCAPES]), events=float(c[abi.CNT_EVENTS]),
                         census=float(c[abi.CNT_CENSUS]), collisions=float(c[abi.CNT_COLLIDE]),
                         step_s=distributed.allreduce_max(t_tr + t_obs, dev), obs_s=t_obs))
    F, F2, cnt, obs_ms = eng.obs_result()
    if world > 1:
        for a in (F, F2, cnt):
            ta = torch.from_numpy(a).to(dev)
            torch.distributed.all_reduce(ta)
            a[...] = ta.cpu().numpy()
    eng.close()
    if rank != 0:
        return
    timed = rows[args.warmup:]
    lc = {"bands_keV": [list(b) for b in EXT25_BANDS],
          "time_bins_with_counts": int(np.count_nonzero(cnt.sum(axis=(1, 2)))),
          "events_binned": float(cnt.sum()),
          "counts_per_band": cnt.sum(axis=(0, 1)).tolist(),
          "first_bins_F_band0..6": F[:8, 0, :].tolist()}
    if args.lc_out:
        out = Path(args.lc_out)
        out.mkdir(parents=True, exist_ok=True)
        binning.outfiles = ["lc07_ev0.dat"]
        observer.write_lc(out, binning, observer.Histogram(F, F2, cnt, obs_ms))
    res = {"workload": "C5-like EC light curve: %dx%d grid, z_max=r_max=1e17 cm, Gamma 25, "
                       "blackbody_G25_4spectra.in on all %d lower rings (EC on t<4e5 s), nst=%d, "
                       "%d rank(s), ext25_lc binning on device" % (nz, nr, nr, nst, world),
           "dt_s": dt, "steps": args.steps, "warmup": args.warmup,
           "packet_steps_per_s": sum(r_["packet_steps"] for r_ in timed) / sum(r_["step_s"] for r_ in timed),
           "obs_kernel_ms_total": obs_ms, "light_curve": lc, "rows": rows}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
