"""The coupled Monte-Carlo step of a T_const = 0 run on one GPU context.

Mirrors the reference's per-step sequence (src/xec2d.f:41-110 master,
:141-193 worker) for the hot path:

    imcgen2d   tables + budgets       Engine.volume_em (c2d_volume_em) +
                                      surface.volume_budget (src/imcgen2d.f:209-456)
    imcfield2d / imcvol2d / imcsurf2d Engine.transport_step (c2d_set_step + c2d_run_step)
    xec_add / cens_add_up             `allreduce` hook (RCCL all-reduce of the fused tallies)
    update                            Engine.fp_step (c2d_fp_step), n_field/ecens read
                                      from the device tallies (src/update2d.f:7-327)

With `device_resident` (the default) the 400-bin emission/absorption tables
and the 200-bin electron spectra never leave the GPU: c2d_volume_em keeps its
tables for c2d_set_step (C2D_DEV_EMISSION) and c2d_fp_step updates the
context's electron state in place (C2D_DEV_ELECTRONS).  Only zone scalars
(270 of each at C3) and the tally buffer's ecens cross the host per step.
"""
from __future__ import annotations

import time as _time
from typing import Callable, Optional

import numpy as np

from . import abi, surface
from .engine import Engine
from .synth import CoupledWorkload


class CoupledRun:
    """Advance a CoupledWorkload one MC step at a time on `eng`."""

    def __init__(self, eng: Engine, wl: CoupledWorkload, device_resident: bool = True,
                 allreduce: Optional[Callable[[], None]] = None, fp_mode: int = abi.FP_AUTO,
                 after_transport: Optional[Callable[[], None]] = None):
        """fp_mode: the FP update's arithmetic (Engine.fp_set_mode); the
        default abi.FP_AUTO picks exact or fast per update, and each step's
        row logs what ran (`fp_mode`).  after_transport: called as soon as a
        step's transport has returned, before the tally exchange and the FP
        update (e.g. the on-device SED binning of the step's escapes, which
        then runs on its own stream beside them)."""
        self.eng, self.wl = eng, wl
        self.after_transport = after_transport
        self.device_resident = device_resident
        self.allreduce = allreduce
        self.state = {k: np.array(v, copy=True) for k, v in wl.state0.items()}
        nz, nr = wl.grid.nz, wl.grid.nr
        self.ecens_prev = np.zeros((nz, nr))
        self.n = 0
        self.last = {}
        self.fp_on = int(wl.deck.get("T_const", 0)) == 0
        eng.fp_set_config(wl.fp_const)
        eng.fp_set_mode(fp_mode)
        self.fp_mode = fp_mode
        L = abi.tally_layout(nz, nr, int(np.asarray(wl.grid.mu).size))
        self._ecens = L["ecens"]
        self._cnt = L["counters"][0]

    def _electrons_on_device(self) -> bool:
        return self.device_resident and self.n > 0

    def step(self) -> dict:
        """One MC step; returns per-phase wall times (s) and counters."""
        eng, wl, st = self.eng, self.wl, self.state
        ncycle, t = wl.clock(self.n)
        dt = wl.dt
        t0 = _time.perf_counter()
        # imcgen2d (src/imcgen2d.f:86-99): ec_old = last step's reduced ecens
        ec_old = self.ecens_prev if ncycle > 0 else np.zeros_like(self.ecens_prev)
        dev_el = self._electrons_on_device()
        vin = dict(wl.fixed, tea=st["tea"], n_e=st["n_e"], f_nt=None if dev_el else st["f_nt"])
        vem = eng.volume_em(dt, vin, tables_to_host=not self.device_resident)
        nsv, ewsv = surface.volume_budget(wl.nst, vem["Eloss_tot"])
        self._last_vem = vem
        t1 = _time.perf_counter()
        nz, nr = wl.grid.nz, wl.grid.nr
        zz, zr = np.zeros(nz), np.zeros(nr)
        izz, izr = np.zeros(nz, np.int32), np.zeros(nr, np.int32)
        tab = (None, None, None) if self.device_resident else (vem["kappa_tot"], vem["eps_tot"],
                                                               vem["eps_th"])
        si = abi.StepInputs(
            ncycle=ncycle, time=t, dt=dt, kappa_tot=tab[0], eps_tot=tab[1], eps_th=tab[2],
            f_nt=None if dev_el else st["f_nt"], Pnt=None if dev_el else st["Pnt"],
            n_e=st["n_e"], Eloss_th=vem["Eloss_th"], Eloss_tot=vem["Eloss_tot"],
            zsurf=wl.fixed["zsurf"], ewsv=ewsv, nsv=nsv, nsurfi=izz, nsurfo=izz, ewsurfi=zz,
            ewsurfo=zz, nsurfu=izr, nsurfl=izr, ewsurfu=zr, ewsurfl=zr, tbbi=zz, tbbo=zz,
            tbbu=zr, tbbl=zr)
        eng.transport_step(si)
        if self.after_transport is not None:
            self.after_transport()
        t2 = _time.perf_counter()
        if self.allreduce is not None:
            self.allreduce()
        t3 = _time.perf_counter()
        # what the step reads back: this step's ecens (the next step's ec_old)
        # and the counters, not the whole tally buffer
        o = self._ecens
        ecens_now = eng.tally_range(o[0], o[1])
        c = eng.tally_range(self._cnt, abi.NCOUNTERS)
        fp_ms = 0.0
        fp_mode = None
        if self.fp_on and ncycle > 0:
            inputs = dict(wl.fixed, tea=st["tea"], n_e=st["n_e"], B_field=vem["B_field"],
                          Eloss_sy=vem["Eloss_sy"], ec_old=ec_old, ecens=None, n_field=None)
            state_in = dict(st)
            if self.device_resident:
                state_in.pop("f_nt", None)
                state_in.pop("Pnt", None)
            new = eng.fp_step(ncycle, t, dt, inputs, state_in)
            for k in ("tea", "n_e", "gmin", "gmax", "amxwl", "p_nth", "Te_new"):
                st[k] = new[k]
            if not self.device_resident:
                st["f_nt"], st["Pnt"] = new["f_nt"], new["Pnt"]
            self.last_fp = new
            fp_ms = eng.last_fp_ms()
            fp_mode = abi.FP_MODE_NAMES.get(eng.last_fp_mode())
        t4 = _time.perf_counter()
        self.ecens_prev = ecens_now.reshape(nz, nr)
        g0_ms, all_ms, _ = eng.last_kernel_ms()
        g0_paths, all_paths = eng.last_path_steps()
        self.last = dict(
            ncycle=ncycle, tables_s=t1 - t0, transport_s=t2 - t1, allreduce_s=t3 - t2, fp_s=t4 - t3,
            step_s=t4 - t0, vem_kernel_ms=eng.last_vem_ms(), transport_gen0_ms=g0_ms,
            transport_all_ms=all_ms, fp_kernel_ms=fp_ms, fp_mode=fp_mode,
            packet_steps=float(c[abi.CNT_STEPS]),
            gen0_steps=float(eng.last_gen0_steps()), gen0_paths=float(g0_paths),
            all_paths=float(all_paths), sources=float(c[abi.CNT_SOURCES]),
            census=float(c[abi.CNT_CENSUS]), escapes=float(c[abi.CNT_ESCAPES]),
            aborted=float(c[abi.CNT_ABORTED]), mean_Te=float(np.mean(st.get("Te_new", st["tea"]))),
            volume_packets=int(nsv.sum()))
        self.n += 1
        return self.last

    def next_step_inputs(self) -> abi.StepInputs:
        """Host-array StepInputs of the NEXT step (tables computed on the GPU
        from the current electron state), e.g. to replay it on the CPU."""
        wl, st = self.wl, self.state
        ncycle, t = wl.clock(self.n)
        f, p = self.electrons()
        vin = dict(wl.fixed, tea=st["tea"], n_e=st["n_e"], f_nt=f)
        vem = self.eng.volume_em(wl.dt, vin, tables_to_host=True)
        nsv, ewsv = surface.volume_budget(wl.nst, vem["Eloss_tot"])
        nz, nr = wl.grid.nz, wl.grid.nr
        zz, zr = np.zeros(nz), np.zeros(nr)
        izz, izr = np.zeros(nz, np.int32), np.zeros(nr, np.int32)
        return abi.StepInputs(
            ncycle=ncycle, time=t, dt=wl.dt, kappa_tot=vem["kappa_tot"], eps_tot=vem["eps_tot"],
            eps_th=vem["eps_th"], f_nt=f, Pnt=p, n_e=st["n_e"], Eloss_th=vem["Eloss_th"],
            Eloss_tot=vem["Eloss_tot"], zsurf=wl.fixed["zsurf"], ewsv=ewsv, nsv=nsv, nsurfi=izz,
            nsurfo=izz, ewsurfi=zz, ewsurfo=zz, nsurfu=izr, nsurfl=izr, ewsurfu=zr, ewsurfl=zr,
            tbbi=zz, tbbo=zz, tbbu=zr, tbbl=zr)

    @staticmethod
    def sample_step(si: abi.StepInputs, frac: float) -> abi.StepInputs:
        """The same step with every zone's volume packet count scaled by frac."""
        import dataclasses
        nsv = np.floor(np.asarray(si.nsv, np.float64) * frac).astype(np.int32)
        return dataclasses.replace(si, nsv=nsv)

    def fp_call_host(self):
        """(ncycle, time, dt, inputs, state) of an FP update from the current
        state and the last step's tallies, as host arrays (CPU replay)."""
        wl, st = self.wl, self.state
        nz, nr = wl.grid.nz, wl.grid.nr
        t = self.eng.tallies()
        f, p = self.electrons()
        ncycle, tm = wl.clock(max(self.n - 1, 1))
        inputs = dict(wl.fixed, tea=st["tea"], n_e=st["n_e"], Eloss_sy=np.zeros((nz, nr)),
                      ec_old=self.ecens_prev, ecens=np.asarray(t["ecens"]).reshape(nz, nr),
                      n_field=np.asarray(t["n_field"]).reshape(nz, nr, abi.NPHFIELD))
        if hasattr(self, "last_fp") and "B_field" in getattr(self, "_last_vem", {}):
            inputs["B_field"] = self._last_vem["B_field"]
            inputs["Eloss_sy"] = self._last_vem["Eloss_sy"]
        state = dict(st, f_nt=f, Pnt=p)
        return ncycle, tm, wl.dt, inputs, state

    def electrons(self):
        """Current f_nt, Pnt [nz, nr, NUM_NT] (downloaded in device-resident mode)."""
        if self._electrons_on_device():
            return self.eng.electron_state()
        return self.state["f_nt"], self.state["Pnt"]
