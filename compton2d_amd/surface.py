"""Host side of imcgen2d's per-step budgets: the EC seed spectrum (`file_sp`),
the surface ring budgets and the volume packet budget handed to the transport.

These produce the `StepInputs` surface fields (`nsurf*`, `ewsurf*`, `tbb*`) and
the `SpectrumTable` that `c2d_set_step` uploads; the sampling itself
(`file_sample`, `planck`, `r_surf_calc`) runs on the GPU.  Reference:

* `file_sp`  src/imcsurf2d_para.f:544-685 — reads `E, L_disk, F_blr, F_ir` per
  record (list-directed: further columns of a record are ignored, so the
  5-column `disk/blackbody_G*_4spectra.in` files read like the 4-column ones),
  normalises the BLR and torus fluxes to Ghisellini & Madau (1996) from the
  disk luminosity, and builds the power-law segment CDF `P_file`.
* time windows  src/imcgen2d.f:111-120 (window t = first with t1(t) > time+dt/2;
  window 1 on ncycle 0) and the EC gate `time + dt/2 >= t0(t)` (`:174`).
* ring budgets  src/imcgen2d.f:155-183 (`erinu`, `erinl`), :436-437 (`nsurfu`,
  `nsurfl`), :476-485 (`ewsurfu`, `ewsurfl`), :499-528 (bias cap); ring areas
  src/setup2d.f:102-113.
* volume budget  src/imcgen2d.f:406-413 (`Emiss_tot`), :446-456 (`nsv`, `ewsv`).

Arithmetic follows the reference's expression order with `math` (glibc) so the
tables equal the reference's bit for bit (tests/test_surface.py pins them
against the golden EC case dumped by the reference itself).
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from pathlib import Path
from typing import Sequence

import numpy as np

from . import abi

PI_REF = 3.1415926536                      # general.pa:25
SIGMA_SB = 1.0267e24                       # imcgen2d.f:13-14: sigma*T^4 with T in keV
NFMAX = abi.NFMAX                          # general.pa:17 (500)
DATA = Path(__file__).resolve().parent / "data" / "ec_seed_spectra.npz"


@dataclass
class EcConstants:
    """reader.f:558,581-586 (`g_bulk`, `R_blr`, `fr_blr`, `R_ir`, `fr_ir`, `R_disk`, `d_jet`)."""
    g_bulk: float = 33.0
    R_blr: float = 2.18e38
    fr_blr: float = 0.1
    R_ir: float = 0.78e19
    fr_ir: float = 0.5
    R_disk: float = 1.0e17
    d_jet: float = 0.5e17


def read_seed_columns(path) -> np.ndarray:
    """The first four values of every record of an EC seed file (E [keV],
    L_disk, F_blr, F_ir), as file_sp's list-directed READ takes them."""
    rows = []
    for line in Path(path).read_text().splitlines():
        f = line.replace("D", "E").replace("d", "e").split()
        if len(f) >= 4:
            rows.append([float(x) for x in f[:4]])
    return np.array(rows, dtype=np.float64).reshape(-1, 4)


def seed_spectrum(name: str) -> np.ndarray:
    """A reference EC seed file shipped as data (compton2d_amd/data/ec_seed_spectra.npz:
    `disk/blackbody_20110929.in`, `disk/blackbody_G25_4spectra.in`, first 4 columns)."""
    with np.load(DATA, allow_pickle=False) as z:
        return z[name].copy()


def file_sp(cols: np.ndarray, c: EcConstants) -> tuple[abi.SpectrumTable, float]:
    """src/imcsurf2d_para.f:544-685.  Returns (table, int_file)."""
    E = [0.0] * (NFMAX + 1)     # 1-based like the COMMON arrays; entries past the file stay 0
    L = [0.0] * (NFMAX + 1)
    Fb = [0.0] * (NFMAX + 1)
    Fi = [0.0] * (NFMAX + 1)
    # read loop 100 (:566-601): read record i; continue while E(i) > 0 and i <= nfmax-1
    i = 0
    n = len(cols)
    while True:
        i += 1
        if i > n:                      # err= branch at end of file
            break
        E[i], L[i], Fb[i], Fi[i] = (float(v) for v in cols[i - 1])
        if not (E[i] > 0.0 and i <= NFMAX - 1):
            break
    nfile = i - 1                      # :602 (the record that ended the loop is not counted)
    if nfile < 2:
        raise ValueError("file_sp: less than 2 lines of input read")   # :641-646 stops
    # totals (:624-633), over nfmax-1 segments as the reference sums them
    Ltot = Fbt = Fit = 0.0
    for k in range(1, NFMAX):
        d = E[k + 1] - E[k]
        Ltot = Ltot + L[k] * d
        Fbt = Fbt + Fb[k] * d
        Fit = Fit + Fi[k] * d
    s = math.sqrt(E[2] / E[1])
    Ltot, Fbt, Fit = Ltot / s, Fbt / s, Fit / s
    g2 = c.g_bulk ** 2
    Fb_norm = 17.0 / 48.0 / PI_REF * g2 * c.fr_blr * Ltot / c.R_blr ** 2
    Fi_norm = 1.0 / 4.0 / PI_REF * g2 * c.fr_ir * Ltot / c.R_ir ** 2
    F = [0.0] * (NFMAX + 1)
    for k in range(1, NFMAX + 1):
        F[k] = Fb[k] / Fbt * Fb_norm + Fi[k] / Fit * Fi_norm
    # loop 150 (:652-666): power-law segments and their running integral
    a1 = np.zeros(nfile - 1)
    I = np.zeros(nfile - 1)
    P = np.zeros(nfile - 1)
    Isum = 0.0
    for k in range(1, nfile):
        alpha = math.log(F[k + 1] / F[k]) / math.log(E[k + 1] / E[k])
        a = alpha + 1.0
        if a > 20.0:
            a = 20.0
        if a < -20.0:
            a = -20.0
        if abs(a) < 1.0e-3:
            Ik = F[k] * E[k] * math.log(E[k + 1] / E[k])
        else:
            Ik = F[k] * E[k] * (math.pow(E[k + 1] / E[k], a) - 1.0) / a
        Isum = Isum + Ik
        a1[k - 1], I[k - 1], P[k - 1] = a, Ik, Isum
    for k in range(nfile - 1):
        P[k] = P[k] / Isum
    tab = abi.SpectrumTable(E_file=np.array(E[1:nfile + 1]), a1=a1, I_file=I,
                            F_file=np.array(F[1:nfile + 1]), P_file=P)
    return tab, Isum


def ring_areas(r: np.ndarray, rmin: float) -> np.ndarray:
    """Asurfl(k) = Asurfu(k) (src/setup2d.f:102-113)."""
    A = np.empty(len(r))
    A[0] = PI_REF * (r[0] ** 2 - rmin ** 2)
    for k in range(1, len(r)):
        A[k] = PI_REF * (r[k] ** 2 - r[k - 1] ** 2)
    return A


def time_window(ncycle: int, time: float, dt: float, t1: Sequence[float]) -> int:
    """0-based window index t (src/imcgen2d.f:111-120)."""
    if ncycle == 0:
        return 0
    t_avg = time + 0.5 * dt
    for t, end in enumerate(t1):
        if end > t_avg:
            return t
    return len(t1)                       # loop ran out: t = ntime+1 (no window)


def ring_budget(r: np.ndarray, rmin: float, nst: int, dt: float, tbb: np.ndarray,
                ec_on: bool, int_file: float):
    """(nsurf, ewsurf, erin) of every upper or lower ring for one window
    (src/imcgen2d.f:155-183 erinu/erinl, :436-437 nsurfu/nsurfl, :476-485
    ewsurfu/ewsurfl; the two sides share the formulas).  `tbb[k] < 0` marks an
    EC file ring; `ec_on` is the `time+dt/2 >= t0` gate.  A ring with tbb > 0
    gets its blackbody energy erin = dt*A*sigma*tbb^4 but no packets: the
    reference sets nsurf only for tbb < 0.  r(0) is taken as rmin (hazard H9:
    the reference reads z(99) there, which is 0 for every grid below 99 zones)."""
    nr = len(r)
    A = ring_areas(r, rmin)
    nsurf = np.zeros(nr, np.int32)
    ewsurf = np.zeros(nr)
    erin = np.zeros(nr)
    for k in range(nr):
        rk0 = rmin if k == 0 else r[k - 1]
        if tbb[k] < 0.0 and ec_on:
            erin[k] = dt * A[k] * int_file
        else:
            erin[k] = dt * A[k] * SIGMA_SB * (tbb[k] ** 4.0)
        if tbb[k] < 0.0:
            nsurf[k] = int(nst * (r[k] ** 2 - rk0 ** 2) / r[-1] ** 2)
        ewsurf[k] = erin[k] / float(nsurf[k]) if nsurf[k] > 0 else 0.0
    return nsurf, ewsurf, erin


def lower_surface_budget(r: np.ndarray, rmin: float, nst: int, dt: float, tbbl: np.ndarray,
                         ec_on: bool, int_file: float):
    """nsurfl, ewsurfl of every lower ring (ring_budget)."""
    n, ew, _ = ring_budget(r, rmin, nst, dt, tbbl, ec_on, int_file)
    return n, ew


def upper_surface_budget(r: np.ndarray, rmin: float, nst: int, dt: float, tbbu: np.ndarray,
                         ec_on: bool, int_file: float):
    """nsurfu, ewsurfu of every upper ring (ring_budget; star_switch = 0)."""
    n, ew, _ = ring_budget(r, rmin, nst, dt, tbbu, ec_on, int_file)
    return n, ew


def volume_budget(nst: int, fas: np.ndarray):
    """nsv, ewsv of every zone (src/imcgen2d.f:406-413, :446-456):
    Emiss_tot sums fas in (j, k) order; nsv = int(0.5*nst*fas/Emiss_tot)
    (Fortran truncation), ewsv = fas/nsv (0 for an empty zone).  Vectorised
    with the same operations: cumsum adds in order (a left fold, as the
    reference's loop), then the same multiply, divide and truncation."""
    fas = np.ascontiguousarray(fas, np.float64)
    nz, nr = fas.shape
    emiss_tot = float(np.cumsum(fas.ravel())[-1]) if fas.size else 0.0
    # the reference casts a NaN budget to an integer (a negative count: the
    # zone's `do i=1,nsv` loop is skipped and the run tracks nothing)
    if not (np.isfinite(fas).all() and np.isfinite(emiss_tot)):
        bad = np.argwhere(~np.isfinite(fas))
        raise FloatingPointError("volume_budget: non-finite emission (Eloss_tot) in %d zone(s), first "
                                 "(j, k) = %s; Emiss_tot = %r" % (len(bad), tuple(int(x) + 1 for x in bad[0])
                                                                  if len(bad) else None, emiss_tot))
    if (fas < 0).any():
        raise ValueError("volume_budget: negative emission in %d zone(s)" % int((fas < 0).sum()))
    if emiss_tot == 0.0:
        return np.zeros((nz, nr), np.int32), np.zeros((nz, nr))
    half = 0.5 * float(nst)
    nsv = np.trunc(half * fas / emiss_tot).astype(np.int32)
    ewsv = np.zeros((nz, nr))
    pos = nsv > 0
    ewsv[pos] = fas[pos] / nsv[pos].astype(np.float64)
    return nsv, ewsv


def apply_bias(nst: int, step: abi.StepInputs) -> float:
    """Cap the packet count at 10*nst (src/imcgen2d.f:499-528).  Returns fbias (1 if unchanged)."""
    n_new = int(np.sum(step.nsurfi) + np.sum(step.nsurfo) + np.sum(step.nsurfu)
                + np.sum(step.nsurfl) + np.sum(step.nsv))
    if n_new <= 10 * nst:
        return 1.0
    fb = float(10 * nst) / float(n_new)
    for nk, ek in (("nsurfi", "ewsurfi"), ("nsurfo", "ewsurfo"), ("nsurfu", "ewsurfu"),
                   ("nsurfl", "ewsurfl"), ("nsv", "ewsv")):
        nv = getattr(step, nk)
        setattr(step, nk, (nv.astype(np.float64) * fb).astype(np.int32))
        setattr(step, ek, getattr(step, ek) / fb)
    return fb
