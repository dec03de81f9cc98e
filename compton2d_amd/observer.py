"""Observer-frame SEDs and light curves from escape events.

The reference turns the escape-event files `p###_evb.dat` (one line per
escaping packet, src/imcleak2d.f:171 format 105) into observables with two
stand-alone C tools:

  * postprocessing/pspt.c  -> time-resolved SED  (`sed30.dat`)
  * postprocessing/plcm.c  -> light curves per angular bin and energy band
                              (`lc07_ev<k>.dat`, `..._aux.dat`, `..._particles.dat`)

Both read an interactive input deck on stdin (e.g. postprocessing/
mrk421_sed.input, mrk421_lc.input), boost every event by the bulk Lorentz
factor, add the light-travel time and histogram it.  Here the same decks are
parsed (`parse_pspt_deck`, `parse_plcm_deck`), the bin edges are built with the
tools' own arithmetic, the per-event loop runs on the GPU (c2d_obs_*,
compton2d_amd/csrc/observe.hip) -- either over event files or directly over
the device event buffer of the last transport step, so no event text needs
to be written at all -- and the output files are written in the tools'
formats (`write_sed`, `write_lc`).

    python -m compton2d_amd.observer pspt < mrk421_sed.input   # in the run dir
    python -m compton2d_amd.observer plcm < mrk421_lc.input
"""
from __future__ import annotations

import ctypes as C
import math
import os
import re
import sys
from dataclasses import dataclass, field
from pathlib import Path
from typing import Iterable, List, Optional, Sequence, Tuple

import numpy as np

from . import abi
from .census_io import fortran_e14_7

PSPT_T_MAX, PSPT_CH_MAX = 90, 200            # pspt.c:8-10 (t_max, ch_max)
PLCM_ST_MAX, PLCM_MU_MAX, PLCM_CH_MAX = 1024, 10, 20   # plcm.c:6-8
# plcm.c:251-266: default energy regions [keV]
PLCM_REGIONS = ((1e-3, 3e-3), (2., 4.), (9., 15.), (15., 20.), (20., 60.), (5e5, 5e7), (1e9, 1e10))
# postprocessing/mrk421_sed.input, the pspt deck of BASELINE configs[2] (C3): input
# series, Gamma, r_max, output file, n_t, t_start, t_end, mu window, 1 log region
# of 100 channels over 1e-7 .. 1e10 keV (an input deck: data, one value a line)
MRK421_SED_DECK = "\n".join(["p001_evb.dat", "33", "1e16", "sed30.dat", "30", "1.6e4", "6e4", "0.99944", "0.99964",
                             "1", "1e-7", "1e10", "100", "0", "n", ""])


# ---------------------------------------------------------------------------
# binning
# ---------------------------------------------------------------------------
@dataclass
class Binning:
    """Bin edges (the tools' arrays) plus what their output headers print."""
    mode: int                       # abi.OBS_SED | abi.OBS_LC
    gam_bulk: float
    rmax: float
    t0: np.ndarray
    t1: np.ndarray
    mu0: np.ndarray
    mu1: np.ndarray
    E0: np.ndarray
    E1: np.ndarray
    dt: float
    t_start: float                  # header values (pspt: t0[0], t1[n_t]; plcm: t_offset, t_max)
    t_end: float
    t_offset: float = 0.0           # LC: subtracted before binning (plcm.c:407)
    t_stop: float = 0.0             # LC: last row printed once t1 > t_stop (plcm.c:234, 548)
    infile: str = "p001_evb.dat"
    outfiles: List[str] = field(default_factory=list)

    @property
    def n_t(self) -> int:
        return len(self.t0)

    @property
    def n_mu(self) -> int:
        return len(self.mu0)

    @property
    def n_e(self) -> int:
        return len(self.E0)

    def to_ctypes(self) -> abi.ObsBins:
        arrs = [np.ascontiguousarray(a, np.float64)
                for a in (self.t0, self.t1, self.mu0, self.mu1, self.E0, self.E1)]
        b = abi.ObsBins(self.mode, self.gam_bulk, self.rmax, self.t_offset,
                        len(arrs[0]), arrs[0].ctypes.data_as(abi.PD), arrs[1].ctypes.data_as(abi.PD),
                        len(arrs[2]), arrs[2].ctypes.data_as(abi.PD), arrs[3].ctypes.data_as(abi.PD),
                        len(arrs[4]), arrs[4].ctypes.data_as(abi.PD), arrs[5].ctypes.data_as(abi.PD))
        b._keep = arrs
        return b


def energy_grid(regions: Sequence[Tuple[float, float, int, bool]]):
    """Energy channels of consecutive regions (E_lower, E_upper, n_r, linear);
    the edge arithmetic of pspt.c:176-195 / plcm.c:280-299 (chained E0*dE)."""
    E0: List[float] = []
    E1: List[float] = []
    for lo, hi, n_r, linear in regions:
        if n_r < 1:
            raise ValueError("energy region needs at least one bin")
        dE = (hi - lo) / float(n_r) if linear else math.exp(math.log(hi / lo) / float(n_r))
        e = lo
        for k in range(n_r):
            E0.append(e)
            e = e + dE if linear else e * dE
            E1.append(e)
    return np.array(E0), np.array(E1)


def sed_binning(gam_bulk=33., rmax=1e16, n_t=30, t_start=1.6e4, t_end=6e4, mu_min=0.99944,
                mu_max=0.99964, regions=((1e-7, 1e10, 100, False),)) -> Binning:
    """pspt.c:131-153 time bins t0[0]+n*dt (+dt), one closed angular window."""
    n_t = min(int(n_t), PSPT_T_MAX)
    dt = (t_end - t_start) / n_t
    t0 = np.array([t_start + n * dt for n in range(n_t)])
    t1 = np.array([t_start + n * dt + dt for n in range(n_t)])
    E0, E1 = energy_grid(regions)
    if len(E0) > PSPT_CH_MAX:
        raise ValueError("pspt: not more than %d energy channels" % PSPT_CH_MAX)
    return Binning(abi.OBS_SED, gam_bulk, rmax, t0, t1, np.array([mu_min]), np.array([mu_max]),
                   E0, E1, dt, t_start, t_end)


def lc_binning(gam_bulk=33., rmax=1e16, mu_bins=((0.99944, 0.99964),), dt=7e2, t_offset=0.,
               t_max=7e4, regions=tuple((lo, hi, 1, False) for lo, hi in PLCM_REGIONS)) -> Binning:
    """plcm.c:236-240 chained time bins t1[k] = t0[k+1] = t0[k] + dt (st_max
    of them), half-open angular bins, possibly overlapping energy bands."""
    t = [0.0]
    for k in range(PLCM_ST_MAX - 1):
        t.append(t[-1] + dt)
    t0 = np.array(t)
    t1 = np.array([x + dt for x in t])
    t1[:-1] = t0[1:]
    E0, E1 = energy_grid(regions)
    if len(E0) > PLCM_CH_MAX:
        raise ValueError("plcm: not more than %d energy channels" % PLCM_CH_MAX)
    mu_bins = list(mu_bins)[:PLCM_MU_MAX]
    return Binning(abi.OBS_LC, gam_bulk, rmax, t0, t1, np.array([m[0] for m in mu_bins]),
                   np.array([m[1] for m in mu_bins]), E0, E1, dt, t_offset, t_max,
                   t_offset=t_offset, t_stop=t_max - t_offset)


# ---------------------------------------------------------------------------
# the tools' input decks (read with gets + atof/atoi, empty line = default)
# ---------------------------------------------------------------------------
_NUM = re.compile(r"\s*[+-]?(\d+\.?\d*|\.\d+)([eE][+-]?\d+)?")
_INT = re.compile(r"\s*[+-]?\d+")


def _atof(s: str) -> float:
    m = _NUM.match(s)
    return float(m.group(0)) if m else 0.0


def _atoi(s: str) -> int:
    m = _INT.match(s)
    return int(m.group(0)) if m else 0


class _Deck:
    def __init__(self, text: str):
        self.lines = text.split("\n")
        self.i = 0

    def line(self) -> str:
        s = self.lines[self.i] if self.i < len(self.lines) else ""
        self.i += 1
        return s

    def d(self, default: float) -> float:            # dinput, pspt.c:53-61
        s = self.line()
        return _atof(s) if len(s) else default

    def n(self, default: int) -> int:                # iinput, pspt.c:64-72
        s = self.line()
        return _atoi(s) if len(s) else default


def _add_dat(s: str) -> str:                         # add_dat, pspt.c:38-50
    return s if len(s) >= 4 and s[-4] == "." else s + ".dat"


def _infile(a: str, default="p001_evb.dat") -> str:  # pspt.c:107-116
    if not a:
        return default
    if a[0].isdigit():
        return _add_dat(default[:2] + a)
    return _add_dat(a)


def parse_pspt_deck(text: str) -> Binning:
    """The stdin dialogue of pspt.c:105-205 (e.g. postprocessing/mrk421_sed.input)."""
    D = _Deck(text)
    infile = _infile(D.line())
    gam_bulk = D.d(33.)
    rmax = D.d(1e16)
    a = D.line()
    outfile = _add_dat(a) if a else "seds_30.dat"
    n_t = D.n(30)
    t_start = D.d(1.6e4)
    t_end = D.d(6e4)
    mu0 = D.d(0.99944)
    mu1 = D.d(0.99964)
    regions = D.n(1)
    E_lower, E_upper, n_r = 1e-7, 1e10, 100
    regs = []
    for _ in range(regions):
        E_lower = D.d(E_lower)
        E_upper = D.d(E_upper)
        n_r = D.n(n_r)
        a = D.line()
        regs.append((E_lower, E_upper, n_r, a[:1] == "1"))
        E_lower = E_upper                            # pspt.c:194
    b = sed_binning(gam_bulk, rmax, n_t, t_start, t_end, mu0, mu1, regs)
    b.infile, b.outfiles = infile, [outfile]
    return b


def mrk421_sed_binning() -> Binning:
    """The SED binning of C3's named output (postprocessing/mrk421_sed.input
    through pspt.c:105-205)."""
    return parse_pspt_deck(MRK421_SED_DECK)


def parse_plcm_deck(text: str) -> Binning:
    """The stdin dialogue of plcm.c:97-302 (e.g. postprocessing/mrk421_lc.input).
    Output names: lc file per angular bin, its `_aux` file and one `_particles`
    file (plcm.c:120-141, 175-214)."""
    D = _Deck(text)
    infile = _infile(D.line())
    gam_bulk = D.d(33.)
    rmax = D.d(1e16)
    name0 = "lc" + infile[2] + "7" + infile[4:len(infile) - 5] + "0" + infile[len(infile) - 4:]
    a = D.line()
    name0 = _add_dat(a if a else name0)
    n_mu = min(D.n(1), PLCM_MU_MAX)
    lo, hi = 0.99944, 0.99964
    names, mus = [], []
    for k in range(n_mu):
        dflt = name0 if k == 0 else name0[:len(name0) - 5] + chr(48 + k) + name0[len(name0) - 4:]
        a = D.line()
        names.append(_add_dat(a if a else dflt))
        lo = D.d(lo)
        hi = D.d(hi)
        mus.append((lo, hi))
        lo = hi                                      # plcm.c:215: mu0[k+1] = mu1[k+1] = mu1[k]
    dt = D.d(7e2)
    t_offset = D.d(0.)
    t_max = D.d(7e4)
    regions = D.n(7)
    E_lower, E_upper, n_r = 1e-3, 3e-3, 1
    regs = []
    for reg in range(regions):
        if reg < len(PLCM_REGIONS):
            E_lower, E_upper = PLCM_REGIONS[reg]
        else:
            E_lower = E_upper
        E_lower = D.d(E_lower)
        E_upper = D.d(E_upper)
        n_r = D.n(n_r)
        a = D.line()
        regs.append((E_lower, E_upper, n_r, a[:1] == "1"))
    b = lc_binning(gam_bulk, rmax, mus, dt, t_offset, t_max, regs)
    b.infile, b.outfiles = infile, names
    return b


# ---------------------------------------------------------------------------
# event files (imcleak2d.f:181 format 6(e14.7,1x),e14.7)
# ---------------------------------------------------------------------------
def write_events(path, ev: np.ndarray) -> None:
    ev = np.asarray(ev, np.float64).reshape(-1, abi.EVENT_WORDS)
    with open(path, "w") as f:
        for row in ev:
            f.write(" ".join(fortran_e14_7(v) for v in row) + "\n")


def read_events(path) -> np.ndarray:
    """fscanf("%lf" x 7) over the whole file, pspt.c:240-245."""
    with open(path) as f:
        vals = np.array(f.read().split(), dtype=np.float64)
    return vals[: len(vals) // 7 * 7].reshape(-1, 7)


def event_files(infile: str = "p001_evb.dat", directory=".") -> Tuple[List[Path], int]:
    """The input-file walk of pspt.c:222-238 / 303-318: p001_evb.dat,
    p002_evb.dat, ... then the next letter series (evc, evd, ... < 'l');
    `factor` counts series that did not restart at p001."""
    d = Path(directory)
    name = list(infile)
    files, factor, n_file = [], 0, 1
    while n_file <= 1000:
        if not (d / "".join(name)).exists():
            while True:
                if name[1] != "0" or name[2] != "0" or name[3] != "1":
                    factor += 1
                name[7] = chr(ord(name[7]) + 1)
                name[1:4] = ["0", "0", "1"]
                if (d / "".join(name)).exists() or not name[7] < "l":
                    break
            if name[7] >= "l":
                break
        files.append(d / "".join(name))
        if name[3] == "9":
            if name[2] == "9":
                name[1] = chr(ord(name[1]) + 1)
                name[2] = "0"
            else:
                name[2] = chr(ord(name[2]) + 1)
            name[3] = "0"
        else:
            name[3] = chr(ord(name[3]) + 1)
        n_file += 1
    return files, factor


# ---------------------------------------------------------------------------
# device binning
# ---------------------------------------------------------------------------
@dataclass
class Histogram:
    """Raw sums per [n_t, n_mu, n_e] bin: F = sum ew, F2 = sum ew^2, count."""
    F: np.ndarray
    F2: np.ndarray
    count: np.ndarray
    kernel_ms: float = 0.0


def bin_events(engine, binning: Binning, events: Iterable[Optional[np.ndarray]]) -> Histogram:
    """Histogram event batches on the engine's GPU (None = the device event
    buffer of the last transport step)."""
    engine.obs_begin(binning)
    for ev in events:
        engine.obs_accumulate(ev)
    F, F2, cnt, ms = engine.obs_result()
    return Histogram(F, F2, cnt, ms)


# ---------------------------------------------------------------------------
# normalisation and output (the tools' formats)
# ---------------------------------------------------------------------------
def _e(x: float) -> str:
    """C printf %e, including glibc's "-nan" for a negative-signed NaN."""
    if x != x:
        return "-nan" if math.copysign(1.0, x) < 0 else "nan"
    return "%e" % x


def cmax(x: float, y: float) -> float:               # max(), pspt.c:15-20 (NaN -> y)
    return x if x > y else y


def sed_flux(b: Binning, h: Histogram) -> np.ndarray:
    """pspt.c:323-328: F[n][k] / (dt (E1-E0) (mu1-mu0) / 2), shape [n_t, n_e]."""
    F = h.F[:, 0, :].copy()
    for k in range(b.n_e):
        den = b.dt * (b.E1[k] - b.E0[k]) * (b.mu1[0] - b.mu0[0]) / 2.
        F[:, k] = F[:, k] / den
    return F


def write_sed(path, b: Binning, h: Histogram, factor: int = 0) -> None:
    """The seds file of pspt.c:330-353."""
    F = sed_flux(b, h)
    cnt = h.count[:, 0, :]
    out = ["#time(s): %e %e dt(s): %e\n" % (b.t_start, b.t_end, b.dt),
           "#angle: %f %f\n" % (b.mu0[0], b.mu1[0]),
           "#factor: %i\n" % factor,
           "#Energy(keV)   Luminosity(erg/s/keV)\n"]
    for k in range(b.n_e):
        row = [_e(cmax(1e-20, math.sqrt(b.E0[k] * b.E1[k]))) + " "]
        for n in range(b.n_t - 1):
            row.append(_e(cmax(1e-20, F[n, k])) + " ")
        n = b.n_t - 1
        row.append("%s %i\n" % (_e(cmax(1e-20, F[n, k])), int(cnt[n, k])))
        out.append("".join(row))
    Path(path).write_text("".join(out))


def lc_moments(b: Binning, h: Histogram):
    """plcm.c:466-490: luminosity F/(dt (mu1-mu0)/2), mean <ew>, <ew^2> and
    the spread sF = sqrt(<ew^2> - <ew>^2) per [n_t, n_mu, n_e] bin."""
    den = np.array([b.dt * (b.mu1[n] - b.mu0[n]) / 2. for n in range(b.n_mu)])
    L = h.F / den[None, :, None]
    cnt = h.count
    with np.errstate(invalid="ignore", divide="ignore"):
        F1 = np.where(cnt > 0, h.F / np.where(cnt > 0, cnt, 1.0), 1e-20)
        F2 = np.where(cnt > 0, h.F2 / np.where(cnt > 0, cnt, 1.0), 1e-20)
        sF = np.where(cnt > 0, np.sqrt(F2 - F1 * F1), 1e-20)
    sF = np.where(cnt == 1, 0.0, sF)
    return L, F1, F2, sF


_LC_HDR1 = ("#   time      +----------------------------- luminosity ----------------------------+ "
            "+--------------------------- particle_sum ---------------------+ "
            "+---------------------------- var(ew)/<ew> -------------------------+\n")
_LC_HDR2 = ("#             |    1         2         3         4         5         6         7    | "
            "|       1        2        3        4        5        6        7| "
            "|    1         2         3         4         5         6         7  |\n")


def aux_name(lc_name: str) -> str:
    """plcm.c:139-141: '<stem>_aux.dat'."""
    return lc_name[:-4] + "_aux.dat"


def particles_name(lc_name: str) -> str:
    """plcm.c:142-144: '<stem>_particles.dat' (from the angular bin 0 name)."""
    return lc_name[:-4] + "_particles.dat"


def write_lc(directory, b: Binning, h: Histogram, factor: int = 0) -> List[Path]:
    """The light-curve files of plcm.c:377-388 and 506-552: per angular bin
    `<name>` (luminosity, counts, sF/<ew>) and `<name>_aux` (<ew>, <ew^2>, sF),
    plus the `_particles` header file.  Rows run until t1 > t_max - t_offset."""
    d = Path(directory)
    L, F1, F2, sF = lc_moments(b, h)
    eh = "".join("#energy range%i: %e %e (keV)\n" % (l + 1, b.E0[l], b.E1[l]) for l in range(b.n_e))
    head = ("#time: %e %e %e\n" % (b.t_start, b.t_end, b.dt) +
            "#angle: %f %f\n" % (b.mu0[0], b.mu1[0]) + "#factor: %i\n" % factor)
    names = b.outfiles or ["lc07_ev%d.dat" % n for n in range(b.n_mu)]
    written = []
    part = [("# energy range %i : %e %e (keV)\n" % (l + 1, b.E0[l], b.E1[l])) for l in range(b.n_e)]
    part += ["# time   : %e %e %e\n" % (b.t_start, b.t_end, b.dt),
             "# mu     : %f %f\n" % (b.mu0[0], b.mu1[0]), "#\n",
             "# time, E, ew, mu, r, z, k(time), n(mu), l(energy)\n", "#\n"]
    p = d / particles_name(names[0])
    p.write_text("".join(part))
    written.append(p)
    for n in range(b.n_mu):
        o1, o2 = [eh, head, _LC_HDR1, _LC_HDR2], [eh, head]
        for k in range(b.n_t):
            mid = _e(cmax(1e-20, (b.t0[k] + b.t1[k]) / 2.))
            r1 = [mid] + [" " + _e(cmax(1e-20, L[k, n, l])) for l in range(b.n_e)]
            r1 += [" %d" % int(h.count[k, n, l]) for l in range(b.n_e)]
            with np.errstate(invalid="ignore", divide="ignore"):
                r1 += [" " + _e(sF[k, n, l] / F1[k, n, l]) for l in range(b.n_e)]
            o1.append("".join(r1) + "\n")
            r2 = [mid] + [" " + _e(F1[k, n, l]) for l in range(b.n_e)]
            r2 += [" " + _e(F2[k, n, l]) for l in range(b.n_e)]
            r2 += [" " + _e(sF[k, n, l]) for l in range(b.n_e)]
            o2.append("".join(r2) + "\n")
            if b.t1[k] > b.t_stop:
                break
        for nm, body in ((names[n], o1), (aux_name(names[n]), o2)):
            (d / nm).write_text("".join(body))
            written.append(d / nm)
    return written


# ---------------------------------------------------------------------------
# command line: the tools' drop-in
# ---------------------------------------------------------------------------
def run_tool(tool: str, deck: str, directory=".", device: int = 0) -> List[Path]:
    """Run the pspt / plcm dialogue `deck` over the event files in `directory`
    with the binning on GPU `device`; write the tool's output files."""
    from .engine import obs_engine
    b = parse_pspt_deck(deck) if tool == "pspt" else parse_plcm_deck(deck)
    files, factor = event_files(b.infile, directory)
    eng = obs_engine(device)
    try:
        h = bin_events(eng, b, (read_events(f) for f in files))
    finally:
        eng.close()
    d = Path(directory)
    if tool == "pspt":
        write_sed(d / b.outfiles[0], b, h, factor)
        return [d / b.outfiles[0]]
    return write_lc(d, b, h, factor)


def main(argv=None) -> int:
    argv = sys.argv[1:] if argv is None else argv
    if not argv or argv[0] not in ("pspt", "plcm"):
        print("usage: python -m compton2d_amd.observer {pspt|plcm} < deck", file=sys.stderr)
        return 2
    for p in run_tool(argv[0], sys.stdin.read()):
        print(p)
    return 0


if __name__ == "__main__":
    sys.exit(main())
