"""ctypes mirror of include/compton2d.h and numpy builders for its structs.

The C-ABI takes every per-zone table as (pointer, strides); the builders
here keep dense numpy arrays in the layouts the reference COMMON blocks
would hand over (src/commonblock.f:53-70) and describe them with strides,
so the same structs drive the HIP library and the test oracle.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass, field
from typing import List, Optional

import numpy as np

N_VOL = 400
NUM_NT = 200
NPHFIELD = 400
NPHOMAX = 128
NPHLCMAX = 10
NMUMAX = 32
NFMAX = 500
MAXZONE = 99
EVENT_WORDS = 7
NCOUNTERS = 16
TR_PROF_WORDS = 32                 # C2D_TR_PROF_WORDS (c2d_transport_prof)

COMTOT_EXACT = 0
COMTOT_TABLE = 1
TRK_SRC = 0           # c2d_config.trk_variant: src/imctrk2d.f (default)
TRK_2012_11 = 1       # src_20121113/imctrk2d.f (hazard H1 fixed)

CNT_STEPS, CNT_ESCAPES, CNT_CENSUS, CNT_COLLIDE, CNT_KILLED, CNT_SOURCES, \
    CNT_COMPB, CNT_EVENTS, CNT_GENS, CNT_ABORTED = range(10)
CNT_ESC_SCAT = 11          # escapes of Compton-scattered packets (imctrk2d(1) copies)

FP_EXACT, FP_FAST, FP_AUTO = 0, 1, 2   # c2d_fp_set_mode
FP_MODE_NAMES = {FP_EXACT: "exact", FP_FAST: "fast", FP_AUTO: "auto"}

ERRORS = {
    0: "C2D_OK", -1: "C2D_E_ARG", -2: "C2D_E_HIP", -3: "C2D_E_CENSUS_OVERFLOW",
    -4: "C2D_E_EVENT_OVERFLOW", -5: "C2D_E_QUEUE_OVERFLOW", -6: "C2D_E_NOMEM",
    -7: "C2D_E_STATE", -8: "C2D_E_FP", -9: "C2D_E_RCCL", -10: "C2D_E_IO",
    -11: "C2D_E_NONFINITE",
}

PD = C.POINTER(C.c_double)
PI32 = C.POINTER(C.c_int32)


class Array3(C.Structure):
    _fields_ = [("data", PD), ("s_i", C.c_int64), ("s_j", C.c_int64), ("s_k", C.c_int64)]


class Array2(C.Structure):
    _fields_ = [("data", PD), ("s_j", C.c_int64), ("s_k", C.c_int64)]


class IArray2(C.Structure):
    _fields_ = [("data", PI32), ("s_j", C.c_int64), ("s_k", C.c_int64)]


class Spectrum(C.Structure):
    _fields_ = [("nfile", C.c_int32), ("E_file", PD), ("a1", PD), ("I_file", PD),
                ("F_file", PD), ("P_file", PD)]


class Config(C.Structure):
    _fields_ = [
        ("nz", C.c_int32), ("nr", C.c_int32), ("rmin", C.c_double), ("zmin", C.c_double),
        ("z", PD), ("r", PD), ("E_ph", PD), ("E_field", PD), ("gnt", PD),
        ("nphtotal", C.c_int32), ("hu", PD), ("nph_lc", C.c_int32), ("Elcmin", PD),
        ("Elcmax", PD), ("nmu", C.c_int32), ("mu", PD),
        ("split1", C.c_int32), ("split2", C.c_int32), ("split3", C.c_int32),
        ("spl3_trg", C.c_int32), ("spec_switch", C.c_int32), ("cr_sent", C.c_int32),
        ("pair_switch", C.c_int32), ("kappa_lag", C.c_int32), ("comtot_mode", C.c_int32),
        ("device", C.c_int32), ("seed", C.c_uint64), ("rank", C.c_int32), ("world", C.c_int32),
        ("census_capacity", C.c_int64), ("event_capacity", C.c_int64),
        ("queue_capacity", C.c_int64), ("census_inplace", C.c_int32),
        ("trk_variant", C.c_int32),
    ]


class StepIn(C.Structure):
    _fields_ = [
        ("ncycle", C.c_int32), ("time", C.c_double), ("dt", C.c_double),
        ("kappa_tot", Array3), ("eps_tot", Array3), ("eps_th", Array3),
        ("f_nt", Array3), ("Pnt", Array3),
        ("n_e", Array2), ("Eloss_th", Array2), ("Eloss_tot", Array2), ("zsurf", Array2),
        ("ewsv", Array2), ("nsv", IArray2),
        ("nsurfi", PI32), ("nsurfo", PI32), ("ewsurfi", PD), ("ewsurfo", PD),
        ("nsurfu", PI32), ("nsurfl", PI32), ("ewsurfu", PD), ("ewsurfl", PD),
        ("tbbi", PD), ("tbbo", PD), ("tbbu", PD), ("tbbl", PD),
        ("spec_i", PI32), ("spec_o", PI32), ("spec_u", PI32), ("spec_l", PI32),
        ("n_spectra", C.c_int32), ("spectra", C.POINTER(Spectrum)),
        ("device_tables", C.c_int32),
    ]

COMM_ID_BYTES = 128          # C2D_COMM_ID_BYTES
CENSUS_REC_WORDS = 8         # C2D_CENSUS_REC_WORDS
# c2d_step_in.device_tables (include/compton2d.h)
DEV_EMISSION, DEV_ELECTRONS = 1, 2


class TallyLayout(C.Structure):
    _fields_ = [(n, C.c_int64) for n in (
        "edep", "prdep", "ecens", "npcen", "n_field", "E_IC", "nelectron", "fout", "edout",
        "erlki", "erlko", "erlku", "erlkl", "Ed_in", "counters", "total")]


class FpIn(C.Structure):
    _fields_ = [("ncell", C.c_int32), ("a", PD), ("b", PD), ("c", PD), ("r", PD),
                ("nt", C.c_int32)]


def tally_layout(nz: int, nr: int, nmu: int) -> dict:
    """Python restatement of c2d_tally_layout_for (include/compton2d.h)."""
    nc = nz * nr
    sizes = [("edep", nc), ("prdep", nc), ("ecens", nc), ("npcen", nc),
             ("n_field", nc * NPHFIELD), ("E_IC", NUM_NT + 2), ("nelectron", NUM_NT + 2),
             ("fout", nmu * NPHOMAX), ("edout", nmu * NPHLCMAX), ("erlki", nz), ("erlko", nz),
             ("erlku", nr), ("erlkl", nr), ("Ed_in", nr), ("counters", NCOUNTERS)]
    out, o = {}, 0
    for name, n in sizes:
        out[name] = (o, n)
        o += n
    out["total"] = (o, 0)
    return out


def split_tallies(buf: np.ndarray, nz: int, nr: int, nmu: int) -> dict:
    """View a fused tally buffer as named arrays (reference shapes, 0-based)."""
    L = tally_layout(nz, nr, nmu)
    t = {}
    for name, (o, n) in L.items():
        if name == "total":
            continue
        t[name] = buf[o:o + n]
    t["edep"] = t["edep"].reshape(nz, nr)
    t["prdep"] = t["prdep"].reshape(nz, nr)
    t["ecens"] = t["ecens"].reshape(nz, nr)
    t["npcen"] = t["npcen"].reshape(nz, nr)
    t["n_field"] = t["n_field"].reshape(nz, nr, NPHFIELD)
    t["fout"] = t["fout"].reshape(nmu, NPHOMAX)
    t["edout"] = t["edout"].reshape(nmu, NPHLCMAX)
    return t


def _pd(a: np.ndarray):
    return a.ctypes.data_as(PD)


def _pi(a: np.ndarray):
    return a.ctypes.data_as(PI32)


@dataclass
class GridConfig:
    """Run-constant set-up: what src/setup2d.f leaves in COMMON."""
    nz: int
    nr: int
    rmin: float
    zmin: float
    z: np.ndarray            # [nz]
    r: np.ndarray            # [nr]
    E_ph: np.ndarray         # [N_VOL]
    E_field: np.ndarray      # [NPHFIELD]
    gnt: np.ndarray          # [NUM_NT]
    hu: np.ndarray           # [nphtotal+1]
    Elcmin: np.ndarray
    Elcmax: np.ndarray
    mu: np.ndarray
    split1: int = 10
    split2: int = 10
    split3: int = 3
    spl3_trg: int = 10
    spec_switch: int = 0
    cr_sent: int = 0
    pair_switch: int = 0
    kappa_lag: int = 1
    comtot_mode: int = COMTOT_EXACT
    device: int = 0
    seed: int = 0x5EEDC2D
    rank: int = 0
    world: int = 1
    census_capacity: int = 1 << 20
    event_capacity: int = 1 << 20
    queue_capacity: int = 1 << 18
    census_inplace: int = 0
    trk_variant: int = 0          # TRK_SRC | TRK_2012_11 (include/compton2d.h)

    def to_ctypes(self) -> Config:
        self._keep = [np.ascontiguousarray(a, dtype=np.float64) for a in (
            self.z, self.r, self.E_ph, self.E_field, self.gnt, self.hu, self.Elcmin,
            self.Elcmax, self.mu)]
        z, r, eph, efield, gnt, hu, elmin, elmax, mu = self._keep
        assert eph.size == N_VOL and efield.size == NPHFIELD and gnt.size == NUM_NT
        return Config(
            nz=self.nz, nr=self.nr, rmin=self.rmin, zmin=self.zmin, z=_pd(z), r=_pd(r),
            E_ph=_pd(eph), E_field=_pd(efield), gnt=_pd(gnt), nphtotal=hu.size - 1, hu=_pd(hu),
            nph_lc=elmin.size, Elcmin=_pd(elmin), Elcmax=_pd(elmax), nmu=mu.size, mu=_pd(mu),
            split1=self.split1, split2=self.split2, split3=self.split3, spl3_trg=self.spl3_trg,
            spec_switch=self.spec_switch, cr_sent=self.cr_sent, pair_switch=self.pair_switch,
            kappa_lag=self.kappa_lag, comtot_mode=self.comtot_mode, device=self.device,
            seed=self.seed, rank=self.rank, world=self.world,
            census_capacity=self.census_capacity, event_capacity=self.event_capacity,
            queue_capacity=self.queue_capacity, census_inplace=self.census_inplace,
            trk_variant=self.trk_variant)


@dataclass
class SpectrumTable:
    """file_sp output (src/imcsurf2d_para.f:544-685)."""
    E_file: np.ndarray
    a1: np.ndarray
    I_file: np.ndarray
    F_file: np.ndarray
    P_file: np.ndarray


@dataclass
class StepInputs:
    """Per-step transport inputs (what imcgen2d/volume_em/file_sp leave in COMMON).

    Dense C-order layouts: kappa_tot/eps_tot/eps_th [nz,nr,N_VOL],
    f_nt/Pnt [nz,nr,NUM_NT], zone scalars [nz,nr], z-surface arrays [nz],
    r-surface arrays [nr].  kappa_tot/eps_tot/eps_th = None: the tables of
    the context's last volume_em (C2D_DEV_EMISSION); f_nt/Pnt = None: the
    context's device electron state (C2D_DEV_ELECTRONS).
    """
    ncycle: int
    time: float
    dt: float
    kappa_tot: Optional[np.ndarray]
    eps_tot: Optional[np.ndarray]
    eps_th: Optional[np.ndarray]
    f_nt: Optional[np.ndarray]
    Pnt: Optional[np.ndarray]
    n_e: np.ndarray
    Eloss_th: np.ndarray
    Eloss_tot: np.ndarray
    zsurf: np.ndarray
    ewsv: np.ndarray
    nsv: np.ndarray
    nsurfi: np.ndarray
    nsurfo: np.ndarray
    ewsurfi: np.ndarray
    ewsurfo: np.ndarray
    nsurfu: np.ndarray
    nsurfl: np.ndarray
    ewsurfu: np.ndarray
    ewsurfl: np.ndarray
    tbbi: np.ndarray
    tbbo: np.ndarray
    tbbu: np.ndarray
    tbbl: np.ndarray
    spectra: List[SpectrumTable] = field(default_factory=list)
    spec_i: Optional[np.ndarray] = None
    spec_o: Optional[np.ndarray] = None
    spec_u: Optional[np.ndarray] = None
    spec_l: Optional[np.ndarray] = None

    def to_ctypes(self) -> StepIn:
        nz, nr = self.n_e.shape
        keep = []

        def d(a):
            a = np.ascontiguousarray(a, dtype=np.float64)
            keep.append(a)
            return a

        def i(a):
            a = np.ascontiguousarray(a, dtype=np.int32)
            keep.append(a)
            return a

        def a3(a, n):
            a = d(a)
            assert a.shape == (nz, nr, n), (a.shape, (nz, nr, n))
            return Array3(_pd(a), 1, nr * n, n)

        def a2(a):
            a = d(a)
            assert a.shape == (nz, nr)
            return Array2(_pd(a), nr, 1)

        nsv = i(self.nsv)
        s = StepIn()
        s.ncycle = int(self.ncycle)
        s.time = float(self.time)
        s.dt = float(self.dt)
        dev = 0
        em = (self.kappa_tot, self.eps_tot, self.eps_th)
        if all(x is None for x in em):
            dev |= DEV_EMISSION
            s.kappa_tot = s.eps_tot = s.eps_th = Array3(None, 0, 0, 0)
        else:
            s.kappa_tot = a3(self.kappa_tot, N_VOL)
            s.eps_tot = a3(self.eps_tot, N_VOL)
            s.eps_th = a3(self.eps_th, N_VOL)
        if self.f_nt is None and self.Pnt is None:
            dev |= DEV_ELECTRONS
            s.f_nt = s.Pnt = Array3(None, 0, 0, 0)
        else:
            s.f_nt = a3(self.f_nt, NUM_NT)
            s.Pnt = a3(self.Pnt, NUM_NT)
        s.device_tables = dev
        s.n_e = a2(self.n_e)
        s.Eloss_th = a2(self.Eloss_th)
        s.Eloss_tot = a2(self.Eloss_tot)
        s.zsurf = a2(self.zsurf)
        s.ewsv = a2(self.ewsv)
        s.nsv = IArray2(_pi(nsv), nr, 1)
        s.nsurfi, s.nsurfo = _pi(i(self.nsurfi)), _pi(i(self.nsurfo))
        s.ewsurfi, s.ewsurfo = _pd(d(self.ewsurfi)), _pd(d(self.ewsurfo))
        s.nsurfu, s.nsurfl = _pi(i(self.nsurfu)), _pi(i(self.nsurfl))
        s.ewsurfu, s.ewsurfl = _pd(d(self.ewsurfu)), _pd(d(self.ewsurfl))
        s.tbbi, s.tbbo = _pd(d(self.tbbi)), _pd(d(self.tbbo))
        s.tbbu, s.tbbl = _pd(d(self.tbbu)), _pd(d(self.tbbl))
        spec_default_z = np.zeros(nz, np.int32) if self.spectra else np.full(nz, -1, np.int32)
        spec_default_r = np.zeros(nr, np.int32) if self.spectra else np.full(nr, -1, np.int32)
        s.spec_i = _pi(i(self.spec_i if self.spec_i is not None else spec_default_z))
        s.spec_o = _pi(i(self.spec_o if self.spec_o is not None else spec_default_z))
        s.spec_u = _pi(i(self.spec_u if self.spec_u is not None else spec_default_r))
        s.spec_l = _pi(i(self.spec_l if self.spec_l is not None else spec_default_r))
        nsp = len(self.spectra)
        arr = (Spectrum * max(nsp, 1))()
        for m, sp in enumerate(self.spectra):
            e, a1, ii, f, p = (d(x) for x in (sp.E_file, sp.a1, sp.I_file, sp.F_file, sp.P_file))
            arr[m] = Spectrum(e.size, _pd(e), _pd(a1), _pd(ii), _pd(f), _pd(p))
        keep.append(arr)
        s.n_spectra = nsp
        s.spectra = C.cast(arr, C.POINTER(Spectrum))
        s._keep = keep
        return s


# ---------------------------------------------------------------------------
# Fokker-Planck electron update (c2d_fp_config / c2d_fp_step_in / _out)
# ---------------------------------------------------------------------------
C2D_E_FP = -8
C2D_E_NONFINITE = -11
ERRORS[C2D_E_FP] = "C2D_E_FP"
FP_E_OLD, FP_E_NEW, FP_HR, FP_HR_ST, FP_DELTA_T, FP_STEPS, FP_SKIPPED = range(7)
FP_NDIAG = 8

_d, _i32, _i64 = C.c_double, C.c_int32, C.c_int64


class MArray2(C.Structure):
    _fields_ = [("data", PD), ("s_j", _i64), ("s_k", _i64)]


class MArray3(C.Structure):
    _fields_ = [("data", PD), ("s_i", _i64), ("s_j", _i64), ("s_k", _i64)]


class FpConfig(C.Structure):
    _fields_ = [
        ("pair_switch", _i32), ("df_implicit", _d), ("df_T", _d), ("r_esc", _d), ("r_acc", _d),
        ("cf_sentinel", _i32), ("r_flare", _d), ("z_flare", _d), ("t_flare", _d),
        ("sigma_r", _d), ("sigma_z", _d), ("sigma_t", _d), ("flare_amp", _d),
        ("inj_switch", _i32), ("inj_dis", _i32), ("g2var_switch", _i32), ("pick_sw", _i32),
        ("inj_g1", _d), ("inj_g2", _d), ("inj_p", _d), ("inj_t", _d), ("inj_L", _d),
        ("pick_rate", _d), ("inj_gg", _d), ("inj_sigma", _d), ("inj_v", _d),
        ("F_IC", PD), ("F_IC_s_i", _i64), ("F_IC_s_ph", _i64),
    ]


class FpStepIn(C.Structure):
    _fields_ = [
        ("ncycle", _i32), ("time", _d), ("dt", _d),
        ("tea", Array2), ("tna", Array2), ("n_e", Array2), ("B_field", Array2),
        ("Eloss_sy", Array2), ("ec_old", Array2), ("turb_lev", Array2), ("vol", Array2),
        ("f_pair", Array2), ("ecens", Array2), ("n_field", Array3),
    ]


class FpStepOut(C.Structure):
    _fields_ = [
        ("f_nt", MArray3), ("Pnt", MArray3), ("Te_new", MArray2), ("tea", MArray2),
        ("n_e", MArray2), ("gmin", MArray2), ("gmax", MArray2), ("amxwl", MArray2),
        ("p_nth", MArray2), ("zone_diag", PD),
        ("E_tot_old", _d), ("E_tot_new", _d), ("hr_total", _d), ("hr_st_total", _d),
        ("dT_max", _d),
    ]


@dataclass
class FpConstants:
    """FP_calc run constants (src/reader.f:512-559, general.pa:27-28)."""
    F_IC: np.ndarray                 # [NUM_NT, NPHFIELD] (icloss2d.f)
    pair_switch: int = 0
    df_implicit: float = 1.0e-2
    df_T: float = 2.5e-1
    r_esc: float = 0.3
    r_acc: float = 1.0
    cf_sentinel: int = 0
    r_flare: float = 0.0
    z_flare: float = 0.0
    t_flare: float = 1.0e6
    sigma_r: float = 1.0e6
    sigma_z: float = 1.0e6
    sigma_t: float = 1.0e6
    flare_amp: float = 0.0
    inj_switch: int = 0
    inj_dis: int = 2
    g2var_switch: int = 0
    pick_sw: int = 0
    inj_g1: float = 1.0e2
    inj_g2: float = 3.0e4
    inj_p: float = 1.0
    inj_t: float = 1.2e6
    inj_L: float = 5.0e40
    pick_rate: float = 0.8e-3
    inj_gg: float = 1.0e2
    inj_sigma: float = 1.0e1
    g_bulk: float = 33.0

    @property
    def inj_v(self) -> float:
        return float(np.sqrt(1.0 - 1.0 / self.g_bulk ** 2) * 2.9979245620e10)   # reader.f:559

    def to_ctypes(self) -> FpConfig:
        f = np.ascontiguousarray(self.F_IC, dtype=np.float64)
        assert f.shape == (NUM_NT, NPHFIELD)
        self._keep = f
        c = FpConfig()
        for name, _ in FpConfig._fields_:
            if name in ("F_IC", "F_IC_s_i", "F_IC_s_ph", "inj_v"):
                continue
            setattr(c, name, getattr(self, name))
        c.inj_v = self.inj_v
        c.F_IC = _pd(f)
        c.F_IC_s_i, c.F_IC_s_ph = NPHFIELD, 1
        return c


FP_STATE_KEYS = ("tea", "n_e", "gmin", "gmax", "amxwl", "p_nth")
FP_INPUT_KEYS = ("tna", "B_field", "Eloss_sy", "ec_old", "turb_lev", "vol", "f_pair", "ecens")


class FpCall:
    """ctypes structs for one c2d_fp_step / c2o_fp_step call.

    `inputs`: zone arrays [nz,nr] for FP_INPUT_KEYS (+ 'n_field' [nz,nr,NPHFIELD];
    'ecens'/'n_field' may be None = the device tally buffer), plus 'tea' and 'n_e'.
    `state`: f_nt/Pnt [nz,nr,NUM_NT] and FP_STATE_KEYS zone arrays; copied, the
    copies are updated in place by the call and returned by result().
    """

    def __init__(self, ncycle: int, time: float, dt: float, inputs: dict, state: dict):
        nz, nr = np.asarray(state["tea"]).shape
        self.nz, self.nr = nz, nr
        keep = []

        def a2(a):
            if a is None:
                return Array2(None, 0, 0)
            a = np.ascontiguousarray(a, dtype=np.float64)
            assert a.shape == (nz, nr)
            keep.append(a)
            return Array2(_pd(a), nr, 1)

        s = FpStepIn()
        s.ncycle, s.time, s.dt = int(ncycle), float(time), float(dt)
        s.tea, s.n_e = a2(state["tea"]), a2(state["n_e"])
        for k in FP_INPUT_KEYS:
            setattr(s, k, a2(inputs.get(k)))
        nf = inputs.get("n_field")
        if nf is None:
            s.n_field = Array3(None, 0, 0, 0)
        else:
            nf = np.ascontiguousarray(nf, dtype=np.float64)
            assert nf.shape == (nz, nr, NPHFIELD)
            keep.append(nf)
            s.n_field = Array3(_pd(nf), 1, nr * NPHFIELD, NPHFIELD)
        # f_nt/Pnt absent or None: the context's device electron state (C2D_DEV_ELECTRONS)
        self.device_electrons = state.get("f_nt") is None and state.get("Pnt") is None
        el = () if self.device_electrons else ("f_nt", "Pnt")
        self.st = {k: np.array(state[k], dtype=np.float64, copy=True) for k in el + FP_STATE_KEYS}
        self.st["Te_new"] = np.zeros((nz, nr))
        self.diag = np.zeros((nz, nr, FP_NDIAG))
        o = FpStepOut()
        for k in ("f_nt", "Pnt"):
            setattr(o, k, MArray3(_pd(self.st[k]), 1, nr * NUM_NT, NUM_NT) if k in self.st
                    else MArray3(None, 0, 0, 0))
        for k in FP_STATE_KEYS + ("Te_new",):
            setattr(o, k, MArray2(_pd(self.st[k]), nr, 1))
        o.zone_diag = _pd(self.diag)
        self.sin, self.sout, self._keep = s, o, keep

    def result(self) -> dict:
        r = dict(self.st)
        r["zone_diag"] = self.diag
        for k in ("E_tot_old", "E_tot_new", "hr_total", "hr_st_total", "dT_max"):
            r[k] = getattr(self.sout, k)
        return r


# ---------------------------------------------------------------------------
# Observer-frame binning (c2d_obs_bins; postprocessing/pspt.c, plcm.c)
# ---------------------------------------------------------------------------
OBS_SED, OBS_LC = 0, 1
OBS_MAX_T, OBS_MAX_MU, OBS_MAX_E = 1024, 32, 256


class ObsBins(C.Structure):
    _fields_ = [
        ("mode", _i32), ("gam_bulk", _d), ("rmax", _d), ("t_offset", _d),
        ("n_t", _i32), ("t0", PD), ("t1", PD),
        ("n_mu", _i32), ("mu0", PD), ("mu1", PD),
        ("n_e", _i32), ("E0", PD), ("E1", PD),
    ]


# ---------------------------------------------------------------------------
# Per-step emission / absorption tables (c2d_vem_in / c2d_vem_out)
# ---------------------------------------------------------------------------
class VemIn(C.Structure):
    _fields_ = [("dt", _d), ("tea", Array2), ("tna", Array2), ("n_e", Array2), ("B_field", Array2),
                ("f_pair", Array2), ("zsurf", Array2), ("vol", Array2), ("ep_switch", IArray2),
                ("f_nt", Array3)]


class VemOut(C.Structure):
    _fields_ = [("kappa_tot", MArray3), ("eps_tot", MArray3), ("eps_th", MArray3),
                ("B_field", MArray2), ("Eloss_sy", MArray2), ("Eloss_cy", MArray2),
                ("Eloss_th", MArray2), ("Eloss_tot", MArray2), ("E_ph", PD)]


VEM_STATE_KEYS = ("tea", "tna", "n_e", "B_field", "f_pair", "zsurf", "vol")


class VemCall:
    """Builds c2d_vem_in/out over dense numpy arrays: per-cell state [nz, nr],
    f_nt [nz, nr, NUM_NT], ep_switch [nz, nr] (int, optional); outputs
    kappa_tot/eps_tot/eps_th [nz, nr, N_VOL] and the per-cell scalars."""

    def __init__(self, dt: float, state: dict, tables_to_host: bool = True):
        """state['f_nt'] = None reads the context's device electron state;
        tables_to_host = False leaves kappa_tot/eps_tot/eps_th on the device
        only (for a following set_step with C2D_DEV_EMISSION)."""
        f = state.get("f_nt")
        f = None if f is None else np.ascontiguousarray(f, np.float64)
        nz, nr = np.asarray(state["tea"]).shape
        self.keep = []

        def a2(key, dflt=0.0):
            v = state.get(key)
            arr = np.ascontiguousarray(np.full((nz, nr), dflt) if v is None else v, np.float64)
            self.keep.append(arr)
            return Array2(arr.ctypes.data_as(PD), nr, 1)

        ep = state.get("ep_switch")
        ep = np.ascontiguousarray(np.zeros((nz, nr)) if ep is None else ep, np.int32)
        self.keep += [f, ep]
        fv = (Array3(None, 0, 0, 0) if f is None else
              Array3(f.ctypes.data_as(PD), 1, nr * NUM_NT, NUM_NT))
        self.sin = VemIn(float(dt), *(a2(k) for k in VEM_STATE_KEYS),
                         IArray2(ep.ctypes.data_as(PI32), nr, 1), fv)
        tabs = ("kappa_tot", "eps_tot", "eps_th")
        self.res = {k: np.zeros((nz, nr, N_VOL)) for k in tabs} if tables_to_host else {}
        for k in ("B_field", "Eloss_sy", "Eloss_cy", "Eloss_th", "Eloss_tot"):
            self.res[k] = np.zeros((nz, nr))
        self.res["E_ph"] = np.zeros(N_VOL)
        r = self.res
        m3 = [MArray3(r[k].ctypes.data_as(PD), 1, nr * N_VOL, N_VOL) if k in r else MArray3(None, 0, 0, 0)
              for k in tabs]
        m2 = [MArray2(r[k].ctypes.data_as(PD), nr, 1) for k in ("B_field", "Eloss_sy", "Eloss_cy", "Eloss_th", "Eloss_tot")]
        self.sout = VemOut(*m3, *m2, r["E_ph"].ctypes.data_as(PD))
