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

from pathlib import Path

import numpy as np

from . import abi

DATA = Path(__file__).resolve().parent / "data" / "medium_inputm.npz"
C_LIGHT = 2.9979245620e10
PI_REF = 3.1415926536


def photon_grid(regions=((1e-7, 1e-3, 10), (1e-3, 1e2, 49), (1e2, 1e11, 69))) -> np.ndarray:
    """hu(1..nphtotal+1) as src/setup2d.f:163-173 builds it."""
    hu = [0.0] * (1 + sum(r[2] for r in regions))
    i = 0
    for lo, hi, nb in regions:
        dE = np.exp(np.log(hi / lo) / nb)
        hu[i] = lo
        for _ in range(nb):
            i += 1
            hu[i] = hu[i - 1] * dE
    return np.array(hu)


def field_grid() -> np.ndarray:
    """E_field (src/setup2d.f:217-222)."""
    dE = np.exp(np.log(1.0e20) / abi.NPHFIELD)
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
    inj_v = np.sqrt(1.0 - 1.0 / g_bulk ** 2) * C_LIGHT
    dt = mcdt * min(r[-1] / nr, z[-1] / nz) / inj_v
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
