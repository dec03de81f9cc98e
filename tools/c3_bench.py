#!/usr/bin/env python3
"""Coupled MC step on one MI355X: every step runs
on the GPU through the C-ABI

    c2d_volume_em   emission/absorption tables from the electron state
                    (imcgen2d.f:209-333 + volume_em)
    budgets         nsv/ewsv from Eloss_tot (host, as imcgen2d's budget)
    c2d_transport_step  census + volume transport (imcfield2d/imcvol2d)
    c2d_fp_step     FP_calc for every zone with n_field/ecens read from the
                    device tallies (update)

on a 30x9 grid (C3's zone count, Mrk 421 set-up src_20121026/input.dat) of the
inputm.dat medium with FP on (pick-up switch of the FP fixture's constants,
tests/golden/fp_pair.npz, with C3's pair_switch = 1: positrons inert as in the
MPI reference, hazard H6).  Reports per-phase times per step and packet-steps/s.
Synthetic: the medium's tables and electron spectrum are the reference's
(compton2d_amd/data/medium_inputm.npz); no network, no checkpoints.

    python tools/c3_bench.py [--sources 100000000] [--steps 3] [--warmup 1]
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
    ap.add_argument("--sources", type=int, default=100_000_000)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--nz", type=int, default=30)
    ap.add_argument("--nr", type=int, default=9)
    args = ap.parse_args()
    from compton2d_amd import abi, synth
    from compton2d_amd.engine import Engine
    from golden_io import FpGoldenCase

    nz, nr, nsrc = args.nz, args.nr, args.sources
    total = args.warmup + args.steps
    wl = synth.c2_workload(nz=nz, nr=nr, sources=nsrc, comtot_mode=abi.COMTOT_TABLE,
                           census_capacity=int(1.3 * nsrc * (total + 1)) + (1 << 20),
                           event_capacity=int(2 * nsrc) + (1 << 20))
    med = np.load(synth.DATA, allow_pickle=False)
    cells = (nz, nr)
    full = lambda v: np.full(cells, float(v))
    tile = lambda a: np.broadcast_to(a, cells + a.shape).copy()
    _, _, vol, zs = synth.zone_geometry(nz, nr, wl.grid.z[-1], wl.grid.rmin, wl.grid.r[-1])
    state = dict(f_nt=tile(med["f_nt"]), Pnt=tile(med["Pnt"]), tea=full(100.0), n_e=full(med["n_e"]),
                 gmin=full(1e2), gmax=full(1e5), amxwl=full(0.0), p_nth=full(2.3))
    fixed = dict(tna=full(100.0), B_field=full(0.13), f_pair=full(0.0), turb_lev=full(1e-20), vol=vol,
                 zsurf=zs)
    eng = Engine(wl.grid)
    eng.fp_set_config(FpGoldenCase("fp_pair").constants())
    dt = wl.dt
    ec_old = np.zeros(cells)
    rows = []
    for n in range(total):
        t_step = time.perf_counter()
        vin = dict(fixed, tea=state["tea"], n_e=state["n_e"], f_nt=state["f_nt"])
        t0 = time.perf_counter()
        vem = eng.volume_em(dt, vin)
        t_vem = time.perf_counter() - t0
        fas = vem["Eloss_tot"]
        nsv = np.floor(nsrc * fas / fas.sum()).astype(np.int64)
        rem = int(nsrc - nsv.sum())
        np.add.at(nsv.reshape(-1), np.argsort(-fas, axis=None)[:rem], 1)
        ewsv = np.where(nsv > 0, fas / np.maximum(nsv, 1), 0.0)
        si = wl.step0
        si.ncycle, si.time, si.dt = n, n * dt, dt
        si.kappa_tot, si.eps_tot, si.eps_th = vem["kappa_tot"], vem["eps_tot"], vem["eps_th"]
        si.Eloss_tot, si.Eloss_th = fas, vem["Eloss_th"]
        si.f_nt, si.Pnt, si.n_e = state["f_nt"], state["Pnt"], state["n_e"]
        si.nsv, si.ewsv = nsv.astype(np.int32), ewsv
        t0 = time.perf_counter()
        eng.transport_step(si)
        t_tr = time.perf_counter() - t0
        _, tr_ms, _ = eng.last_kernel_ms()
        tal = eng.tallies()
        steps = float(tal["counters"][abi.CNT_STEPS])
        inputs = dict(fixed, tea=state["tea"], n_e=state["n_e"], B_field=vem["B_field"],
                      Eloss_sy=vem["Eloss_sy"], ec_old=ec_old, ecens=None, n_field=None)
        t0 = time.perf_counter()
        state = eng.fp_step(n, n * dt, dt, inputs, state)
        t_fp = time.perf_counter() - t0
        ec_old = tal["ecens"].reshape(cells)
        rows.append(dict(step_s=time.perf_counter() - t_step, vem_s=t_vem, vem_kernel_ms=eng.last_vem_ms(),
                         transport_s=t_tr, transport_kernels_ms=tr_ms, fp_s=t_fp,
                         fp_kernel_ms=eng.last_fp_ms(), packet_steps=steps,
                         mean_Te=float(np.mean(state["tea"]))))
    eng.close()
    timed = rows[args.warmup:]
    avg = {k: float(np.mean([r[k] for r in timed])) for k in timed[0]}
    out = {"workload": "C3-like coupled step: %dx%d grid, %d volume packets/step, FP on (pick-up), "
                       "tables from the electron state each step, inputm.dat medium" % (nz, nr, nsrc),
           "steps": args.steps, "warmup": args.warmup, "per_step": avg,
           "packet_steps_per_s": sum(r["packet_steps"] for r in timed) / sum(r["step_s"] for r in timed),
           "rows": rows}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
