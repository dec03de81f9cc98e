"""Synthetic workloads shaped like the reference's configurations.

`c2_workload` builds BASELINE config C2: a 32x32 (r,z)
cylinder with the src_20121026/inputm.dat medium in every zone (n_e = 80
cm^-3, B = 0.13 G, power-law electrons gmin=1e2, gmax=1e5, p=2.3),
z_max = 1e16 cm, r_max = 7.5e15 cm, Gamma = 33, T_const = 1 (no FP),
no surface sources, and N volume packets per step distributed over the zones
in proportion to their emitted energy as imcgen2d does (src/imcgen2d.f:446-456).

The per-zone tables (kappa_tot, eps_tot, eps_th, f_nt, Pnt) are the ones the
reference's volume_em/P_nontherm compute for that medium
(compton2d_amd/data/medium_inputm.npz, made by tests/golden/make_golden.py).
Grids follow src/setup2d.f:47-222.
"""
from __future__ import annotations

import math
from pathlib import Path

import numpy as np

from . import abi

DATA = Path(__file__).resolve().parent / "data" / "medium_inputm.npz"
IC_LOSS = Path(__file__).resolve().parent / "data" / "ic_loss.npz"
C_LIGHT = 2.9979245620e10
PI_REF = 3.1415926536

# BASELINE config C3: the Mrk 421 SSC deck, src_20121026/input.dat (line
# numbers below) with src_20121026/inputm.dat in every zone.  Two deliberate
# deviations, both stated wherever C3 numbers are reported:
#   * splits 10/10/3/10 instead of the deck's 1000/1000/300/10 (:113-116), the
#     throughput setting of SURVEY.md §8(d) for every config;
#   * the lineage Philox RNG on the GPU; the reference-side goldens run the
#     deck with rand_switch = 1 (lagged Fibonacci, per-zone reseeding), not
#     the deck's rand_switch = 2 (:78, ran1 seeded per MPI rank, whose
#     streams depend on the master/worker schedule).
C3_DECK = dict(
    nz=30, nr=9,                                    # :1-2
    zmax=1.0e16, rmin=0.0, rmax=0.75e16,            # :3-5
    tstop=5.0e6, mcdt=1.0,                          # :7-8
    t0=1.0, t1=1.0,                                 # :9-11 (ntime = 1)
    tbbu=0.0, tbbl=0.0, spec_file="blackbody.in",   # :12-47 (no boundary sources)
    spec_switch=0,                                  # :48
    regions=((1.0e-7, 1.0e-3, 10), (1.0e-3, 1.0e2, 49), (1.0e2, 1.0e11, 69)),   # :49-58
    nmu=1,                                          # :59
    lc=((1e-7, 1e-3), (1e-3, 1e0), (1e0, 1e2), (1e2, 1e5), (1e5, 1e9)),         # :60-70
    nst=800000, rseed=9857,                         # :76-77
    rand_switch=1,                                  # deck :78 says 2 (see above)
    cr_sent=0, pair_switch=1, T_const=0,            # :79, :82-83
    cf_sentinel=0, r_flare=0.0, z_flare=0.0, t_flare=1.0e6, sigma_r=1.0e15,
    sigma_z=1.0e15, sigma_t=1.0e6, flare_amp=10.0,  # :84-91
    r_esc=0.3, r_acc=1.0, inj_switch=1, inj_dis=2, g2var_switch=0, pick_sw=1,   # :92-97
    inj_g1=1.0e2, inj_g2=3.0e4, inj_p=1.0, inj_t=1.2e6, inj_L=5.0e40,
    pick_rate=0.8e-3, inj_gg=1.0e2, inj_sigma=1.0e1, g_bulk=33.0,              # :98-106
    split1=10, split2=10, split3=3, spl3_trg=10,    # deck :113-116: 1000/1000/300/10
    # inputm.dat:1-11 (per zone)
    tea=100.0, tna=100.0, n_e=80.0, B=0.13, amxwl=0.0, gmin=1.0e2, gmax=1.0e5,
    p_nth=2.3, q_turb=1.666667, turb_lev=1.0e-20,
)
FP_CONST_KEYS = ("cf_sentinel", "r_flare", "z_flare", "t_flare", "sigma_r", "sigma_z", "sigma_t",
                 "flare_amp", "r_esc", "r_acc", "inj_switch", "inj_dis", "g2var_switch", "pick_sw",
                 "inj_g1", "inj_g2", "inj_p", "inj_t", "inj_L", "pick_rate", "inj_gg", "inj_sigma",
                 "g_bulk")


def c3_refcase(nst: int = 800000) -> dict:
    """The C3 deck as a reference input-deck description (tests/refcase.py)."""
    d = dict(C3_DECK)
    d["nst"] = int(nst)
    return d


def ic_loss() -> np.ndarray:
    """F_IC [NUM_NT, NPHFIELD] of the reference setup (src/icloss2d.f:1-64)."""
    with np.load(IC_LOSS, allow_pickle=False) as z:
        return z["F_IC"].copy()


def fp_constants(deck: dict = C3_DECK) -> abi.FpConstants:
    """FP_calc run constants of a deck (reader.f:512-559)."""
    return abi.FpConstants(F_IC=ic_loss(), pair_switch=int(deck["pair_switch"]),
                           **{k: deck[k] for k in FP_CONST_KEYS})


def mc_dt(zmax: float, rmax: float, nz: int, nr: int, mcdt: float, g_bulk: float) -> float:
    """dt(1) = mcdt * min(r(nr)/nr, z(nz)/nz) / inj_v (src/setup2d.f:49-51),
    evaluated before setup rebuilds z()/r() by accumulation, i.e. on the
    deck's z(nz), r(nr); inj_v from src/reader.f:559."""
    inj_v = math.sqrt(1.0 - 1.0 / g_bulk ** 2) * C_LIGHT
    return mcdt * min(rmax / nr, zmax / nz) / inj_v


def photon_grid(regions=((1e-7, 1e-3, 10), (1e-3, 1e2, 49), (1e2, 1e11, 69))) -> np.ndarray:
    """hu(1..nphtotal+1) as src/setup2d.f:162-173 builds it (glibc log/exp via
    `math`, as the Fortran intrinsics)."""
    hu = [0.0] * (1 + sum(r[2] for r in regions))
    i = 0
    for lo, hi, nb in regions:
        dE = math.exp(math.log(hi / lo) / float(nb))
        hu[i] = lo
        for _ in range(nb):
            i += 1
            hu[i] = hu[i - 1] * dE
    return np.array(hu)


def field_grid() -> np.ndarray:
    """E_field (src/setup2d.f:215-222)."""
    dE = math.exp(math.log(1.0e20) / float(abi.NPHFIELD))
    e = np.empty(abi.NPHFIELD)
    e[0] = 1.0e-10
    for i in range(1, abi.NPHFIELD):
        e[i] = e[i - 1] * dE
    return e


def zone_geometry(nz, nr, zmax, rmin, rmax):
    """z, r, vol, zsurf (src/setup2d.f:60-100)."""
    delj = zmax / nz
    delk = (rmax - rmin) / nr
    z = np.empty(nz)
    r = np.empty(nr)
    z[0] = delj
    r[0] = rmin + delk
    for j in range(nz - 1):
        z[j + 1] = z[j] + delj
    for k in range(nr - 1):
        r[k + 1] = r[k] + delk
    vol = np.empty((nz, nr))
    zs = np.empty((nz, nr))
    for j in range(nz):
        dz = z[0] if j == 0 else z[j] - z[j - 1]
        for k in range(nr):
            rl = rmin if k == 0 else r[k - 1]
            vol[j, k] = PI_REF * (r[k] ** 2 - rl ** 2) * dz
            zs[j, k] = 2.0 * PI_REF * ((r[k] + rl) * dz + (r[k] ** 2 - rl ** 2))
    return z, r, vol, zs


class Workload:
    def __init__(self, grid: abi.GridConfig, step: abi.StepInputs, dt: float, description: str):
        self.grid = grid
        self.step0 = step
        self.dt = dt
        self.description = description

    def clock(self, n: int):
        """(ncycle, time) of step n (src/xec2d.f:100-107: time advances from ncycle 1)."""
        return n, max(n - 1, 0) * self.dt


def c2_workload(nz: int = 32, nr: int = 32, sources: int = 10_000_000, splits=(10, 10, 3, 10),
                comtot_mode: int = abi.COMTOT_TABLE, rank: int = 0, world: int = 1,
                device: int = 0, seed: int = 0x5EEDC2D, census_capacity: int | None = None,
                event_capacity: int | None = None) -> Workload:
    med = np.load(DATA, allow_pickle=False)
    zmax, rmin, rmax, g_bulk, mcdt = 1.0e16, 0.0, 7.5e15, 33.0, 1.0
    z, r, vol, zs = zone_geometry(nz, nr, zmax, rmin, rmax)
    dt = mc_dt(zmax, rmax, nz, nr, mcdt, g_bulk)
    fas = med["emiss_per_vol_per_s"] * vol * dt
    nsv = np.floor(sources * fas / fas.sum()).astype(np.int64)
    # hand the rounding remainder to the largest zones so the total is exact
    rem = int(sources - nsv.sum())
    order = np.argsort(-fas, axis=None)[:rem]
    np.add.at(nsv.reshape(-1), order, 1)
    ewsv = np.where(nsv > 0, fas / np.maximum(nsv, 1), 0.0)
    cells = (nz, nr)
    tile3 = lambda a: np.broadcast_to(a, cells + a.shape).copy()
    hu = photon_grid()
    lc = np.array([(1e-7, 1e-3), (1e-3, 1e0), (1e0, 1e2), (1e2, 1e5), (1e5, 1e9)])
    per_gpu = int(np.ceil(sources / world))
    grid = abi.GridConfig(
        nz=nz, nr=nr, rmin=rmin, zmin=0.0, z=z, r=r, E_ph=med["E_ph"], E_field=field_grid(),
        gnt=med["gnt"], hu=hu, Elcmin=lc[:, 0], Elcmax=lc[:, 1], mu=np.array([1.0]),
        split1=splits[0], split2=splits[1], split3=splits[2], spl3_trg=splits[3],
        comtot_mode=comtot_mode, device=device, seed=seed, rank=rank, world=world,
        census_capacity=census_capacity or max(1 << 20, 8 * per_gpu),
        event_capacity=event_capacity or max(1 << 20, 2 * per_gpu),
        queue_capacity=1 << 20)
    zeros_z, zeros_r = np.zeros(nz), np.zeros(nr)
    izeros_z, izeros_r = np.zeros(nz, np.int32), np.zeros(nr, np.int32)
    step = abi.StepInputs(
        ncycle=0, time=0.0, dt=dt,
        kappa_tot=tile3(med["kappa_tot"]), eps_tot=tile3(med["eps_tot"]),
        eps_th=tile3(med["eps_th"]), f_nt=tile3(med["f_nt"]), Pnt=tile3(med["Pnt"]),
        n_e=np.full(cells, float(med["n_e"])),
        Eloss_th=fas * float(med["Eloss_th_frac"]), Eloss_tot=fas, zsurf=zs, ewsv=ewsv,
        nsv=nsv.astype(np.int32), nsurfi=izeros_z, nsurfo=izeros_z, ewsurfi=zeros_z,
        ewsurfo=zeros_z, nsurfu=izeros_r, nsurfl=izeros_r, ewsurfu=zeros_r, ewsurfl=zeros_r,
        tbbi=zeros_z, tbbo=zeros_z, tbbu=zeros_r, tbbl=zeros_r)
    desc = ("C2: %dx%d (r,z) grid, %d volume packets/step, splits %s, inputm.dat medium, "
            "T_const=1 (FP off), no surface sources" % (nz, nr, sources, "/".join(map(str, splits))))
    return Workload(grid, step, dt, desc)


class CoupledWorkload:
    """A T_const = 0 run: grid, deck, the initial zone state and what stays
    fixed per zone (the imcgen2d / update inputs of src/xec2d.f:67-87)."""

    def __init__(self, grid: abi.GridConfig, deck: dict, nst: int, dt: float, state0: dict,
                 fixed: dict, fp_const: abi.FpConstants, description: str):
        self.grid, self.deck, self.nst, self.dt = grid, deck, nst, dt
        self.state0, self.fixed, self.fp_const = state0, fixed, fp_const
        self.description = description

    def clock(self, n: int):
        return n, max(n - 1, 0) * self.dt


def c3_workload(sources: int = 100_000_000, comtot_mode: int = abi.COMTOT_TABLE, rank: int = 0,
                world: int = 1, device: int = 0, seed: int = 0x5EEDC2D,
                census_capacity: int | None = None, event_capacity: int | None = None,
                deck: dict = C3_DECK) -> CoupledWorkload:
    """BASELINE config C3: the Mrk 421 SSC deck (C3_DECK)
    with nst = 2*sources (imcgen2d hands 0.5*nst volume packets per step,
    src/imcgen2d.f:448), FP on.  The initial electron state is the
    reference's P_nontherm of the inputm.dat medium in every zone
    (compton2d_amd/data/medium_inputm.npz); tables, budgets and electrons
    then evolve on the device every step (compton2d_amd/coupled.py)."""
    med = np.load(DATA, allow_pickle=False)
    nz, nr = deck["nz"], deck["nr"]
    if deck["nmu"] != 1:
        raise ValueError("c3_workload: one angular bin (input.dat:59)")
    z, r, vol, zs = zone_geometry(nz, nr, deck["zmax"], deck["rmin"], deck["rmax"])
    dt = mc_dt(deck["zmax"], deck["rmax"], nz, nr, deck["mcdt"], deck["g_bulk"])
    lc = np.array(deck["lc"])
    per_gpu = int(np.ceil(sources / world))
    grid = abi.GridConfig(
        nz=nz, nr=nr, rmin=deck["rmin"], zmin=0.0, z=z, r=r, E_ph=med["E_ph"], E_field=field_grid(),
        gnt=med["gnt"], hu=photon_grid(deck["regions"]), Elcmin=lc[:, 0], Elcmax=lc[:, 1],
        mu=np.array([1.0]),
        split1=deck["split1"], split2=deck["split2"], split3=deck["split3"], spl3_trg=deck["spl3_trg"],
        spec_switch=deck["spec_switch"], cr_sent=deck["cr_sent"], pair_switch=deck["pair_switch"],
        comtot_mode=comtot_mode, device=device, seed=seed, rank=rank, world=world,
        census_capacity=census_capacity or max(1 << 20, 8 * per_gpu),
        event_capacity=event_capacity or max(1 << 20, 2 * per_gpu),
        queue_capacity=1 << 20)
    cells = (nz, nr)
    full = lambda v: np.full(cells, float(v))
    tile = lambda a: np.broadcast_to(a, cells + a.shape).copy()
    state0 = dict(f_nt=tile(med["f_nt"]), Pnt=tile(med["Pnt"]), tea=full(deck["tea"]),
                  n_e=full(deck["n_e"]), gmin=full(deck["gmin"]), gmax=full(deck["gmax"]),
                  amxwl=full(deck["amxwl"]), p_nth=full(deck["p_nth"]))
    fixed = dict(tna=full(deck["tna"]), B_field=full(deck["B"]), f_pair=full(0.0),
                 turb_lev=full(deck["turb_lev"]), vol=vol, zsurf=zs)
    desc = ("C3: Mrk 421 SSC deck (src_20121026/input.dat + inputm.dat), %dx%d (z,r) grid, "
            "%d volume packets/step, FP on (pick-up + injection, pair_switch=1 inert), splits %s"
            % (nz, nr, sources, "/".join(str(deck[k]) for k in ("split1", "split2", "split3",
                                                               "spl3_trg"))))
    return CoupledWorkload(grid, deck, 2 * int(sources), dt, state0, fixed, fp_constants(deck), desc)
