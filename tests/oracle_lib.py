"""ctypes front-end of the C oracle (oracle/c2d_oracle.c) — TEST INFRASTRUCTURE.

Builds oracle/_build/liboracle_{ref,det}.so on demand (gcc is available here
and on the GPU box) and wraps them.  Used only by tests/, __graft_entry__.smoke()
and bench.py's cpu_baseline leg.
"""
from __future__ import annotations

import ctypes as C
import subprocess
from pathlib import Path

import numpy as np

from compton2d_amd import abi

ROOT = Path(__file__).resolve().parents[1]
ORACLE_DIR = ROOT / "oracle"

RNG_FIB, RNG_RAN1, RNG_LINEAGE = 1, 2, 3

_libs = {}


def build() -> None:
    subprocess.run(["make", "-s", "-C", str(ORACLE_DIR)], check=True)


def load(flavor: str = "ref") -> C.CDLL:
    """flavor 'ref' = glibc libm (reference parity); 'det' = c2d_math (GPU parity)."""
    if flavor in _libs:
        return _libs[flavor]
    path = ORACLE_DIR / "_build" / ("liboracle_%s.so" % flavor)
    srcs = (ORACLE_DIR / "c2d_oracle.c", ORACLE_DIR / "c2d_fp_oracle.c",
            ORACLE_DIR / "c2d_obs_oracle.c")
    if not path.exists() or any(path.stat().st_mtime < s.stat().st_mtime for s in srcs):
        build()
    lib = C.CDLL(str(path))
    lib.c2o_create.restype = C.c_void_p
    lib.c2o_create.argtypes = [C.POINTER(abi.Config), C.c_int, C.c_int, C.c_int32, C.c_int]
    lib.c2o_destroy.argtypes = [C.c_void_p]
    lib.c2o_step.restype = C.c_int
    lib.c2o_step.argtypes = [C.c_void_p, C.POINTER(abi.StepIn)]
    lib.c2o_tallies.restype = C.POINTER(C.c_double)
    lib.c2o_tallies.argtypes = [C.c_void_p, C.POINTER(C.c_int64)]
    lib.c2o_event_count.restype = C.c_int64
    lib.c2o_event_count.argtypes = [C.c_void_p]
    lib.c2o_events.restype = C.c_int64
    lib.c2o_events.argtypes = [C.c_void_p, C.POINTER(C.c_double), C.c_int64]
    lib.c2o_census_count.restype = C.c_int64
    lib.c2o_census_count.argtypes = [C.c_void_p]
    lib.c2o_census_export.restype = C.c_int64
    lib.c2o_census_export.argtypes = [C.c_void_p, C.POINTER(C.c_double), C.POINTER(C.c_int32),
                                      C.POINTER(C.c_uint64), C.c_int64]
    lib.c2o_census_import.restype = C.c_int
    lib.c2o_census_import.argtypes = [C.c_void_p, C.POINTER(C.c_double), C.POINTER(C.c_int32),
                                      C.POINTER(C.c_uint64), C.c_int64]
    lib.c2o_rseed.restype = C.c_int32
    lib.c2o_rseed.argtypes = [C.c_void_p]
    lib.c2o_unit_fib_init.argtypes = [C.c_int32]
    lib.c2o_unit_fib_draw.argtypes = [C.c_int64, C.POINTER(C.c_double)]
    lib.c2o_unit_seed_zone.argtypes = [C.POINTER(C.c_int32), C.c_int, C.c_int,
                                       C.POINTER(C.c_int32), C.POINTER(C.c_int32),
                                       C.POINTER(C.c_int32)]
    lib.c2o_unit_ran1.argtypes = [C.POINTER(C.c_int32), C.c_int64, C.POINTER(C.c_double)]
    lib.c2o_unit_dilog.restype = C.c_double
    lib.c2o_unit_dilog.argtypes = [C.c_double]
    lib.c2o_unit_intg_v.restype = C.c_double
    lib.c2o_unit_intg_v.argtypes = [C.c_double]
    lib.c2o_unit_comtot.restype = C.c_double
    lib.c2o_unit_comtot.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_double]
    lib.c2o_unit_set_tables.argtypes = [C.c_void_p, C.POINTER(abi.StepIn)]
    lib.c2o_unit_compb2d.restype = C.c_int
    lib.c2o_unit_compb2d.argtypes = [C.c_void_p, C.POINTER(C.c_double), C.POINTER(C.c_int32),
                                     C.c_int, C.c_uint64, C.POINTER(C.c_uint32)]
    lib.c2o_unit_planck.restype = C.c_double
    lib.c2o_unit_planck.argtypes = [C.c_void_p, C.c_double, C.c_double, C.POINTER(C.c_int32)]
    lib.c2o_unit_philox_draw.restype = C.c_double
    lib.c2o_unit_philox_draw.argtypes = [C.c_uint64, C.c_uint32]
    lib.c2o_unit_philox_draw_s.restype = C.c_double
    lib.c2o_unit_philox_draw_s.argtypes = [C.c_uint64, C.c_uint32, C.c_uint32]
    lib.c2o_unit_derive_s.restype = C.c_uint64
    lib.c2o_unit_derive_s.argtypes = [C.c_uint64, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32]
    lib.c2o_unit_derive.restype = C.c_uint64
    lib.c2o_unit_derive.argtypes = [C.c_uint64, C.c_uint32, C.c_uint32, C.c_uint32]
    lib.c2o_is_detmath.restype = C.c_int
    lib.c2o_fp_step.restype = C.c_int
    lib.c2o_fp_step.argtypes = [C.POINTER(abi.Config), C.POINTER(abi.FpConfig),
                                C.POINTER(abi.FpStepIn), C.POINTER(abi.FpStepOut)]
    lib.c2o_fp_step_zones.restype = C.c_int
    lib.c2o_fp_step_zones.argtypes = [C.POINTER(abi.Config), C.POINTER(abi.FpConfig),
                                      C.POINTER(abi.FpStepIn), C.POINTER(abi.FpStepOut),
                                      C.POINTER(C.c_int32), C.c_int]
    lib.c2o_gamma_bar.restype = C.c_double
    lib.c2o_gamma_bar.argtypes = [C.c_double]
    _libs[flavor] = lib
    return lib


class Oracle:
    """One oracle context = the reference's worker state for one run."""

    def __init__(self, grid: abi.GridConfig, rng_mode: int = RNG_LINEAGE, flavor: str = "det",
                 rand_switch: int = 1, rseed: int = 9857, h4_stale: int = 0):
        self.lib = load(flavor)
        self.grid = grid
        self._cfg = grid.to_ctypes()
        self.ctx = self.lib.c2o_create(C.byref(self._cfg), rng_mode, rand_switch, rseed, h4_stale)
        if not self.ctx:
            raise ValueError("c2o_create rejected the configuration")
        self.nz, self.nr, self.nmu = grid.nz, grid.nr, grid.mu.size

    def close(self):
        if self.ctx:
            self.lib.c2o_destroy(self.ctx)
            self.ctx = None

    __del__ = close

    def step(self, si: abi.StepInputs) -> int:
        self._si = si.to_ctypes()
        return self.lib.c2o_step(self.ctx, C.byref(self._si))

    def tallies(self) -> np.ndarray:
        n = C.c_int64()
        p = self.lib.c2o_tallies(self.ctx, C.byref(n))
        return np.ctypeslib.as_array(p, shape=(n.value,)).copy()

    def split(self) -> dict:
        return abi.split_tallies(self.tallies(), self.nz, self.nr, self.nmu)

    def events(self) -> np.ndarray:
        n = self.lib.c2o_event_count(self.ctx)
        out = np.zeros((max(n, 1), abi.EVENT_WORDS))
        self.lib.c2o_events(self.ctx, out.ctypes.data_as(C.POINTER(C.c_double)), n)
        return out[:n]

    def census(self):
        n = self.lib.c2o_census_count(self.ctx)
        d6 = np.zeros((max(n, 1), 6))
        i5 = np.zeros((max(n, 1), 5), np.int32)
        keys = np.zeros(max(n, 1), np.uint64)
        self.lib.c2o_census_export(self.ctx, d6.ctypes.data_as(C.POINTER(C.c_double)),
                                   i5.ctypes.data_as(C.POINTER(C.c_int32)),
                                   keys.ctypes.data_as(C.POINTER(C.c_uint64)), n)
        return d6[:n], i5[:n], keys[:n]

    def import_census(self, d6, i5, keys) -> int:
        d6 = np.ascontiguousarray(d6, np.float64)
        i5 = np.ascontiguousarray(i5, np.int32)
        keys = np.ascontiguousarray(keys, np.uint64)
        return self.lib.c2o_census_import(self.ctx, d6.ctypes.data_as(C.POINTER(C.c_double)),
                                          i5.ctypes.data_as(C.POINTER(C.c_int32)),
                                          keys.ctypes.data_as(C.POINTER(C.c_uint64)), len(keys))


def fp_step(grid: abi.GridConfig, const: abi.FpConstants, ncycle: int, time: float, dt: float,
            inputs: dict, state: dict, flavor: str = "det", cells=None) -> dict:
    """The oracle's `update` (oracle/c2d_fp_oracle.c): returns the new state.
    `cells` (ascending j*nr+k): solve only those zones (the others keep their
    input state; the E_add_up sums cover the listed zones)."""
    lib = load(flavor)
    g, fc = grid.to_ctypes(), const.to_ctypes()
    call = abi.FpCall(ncycle, time, dt, inputs, state)
    if cells is not None:
        sel = np.ascontiguousarray(sorted(int(x) for x in cells), np.int32)
        rc = lib.c2o_fp_step_zones(C.byref(g), C.byref(fc), C.byref(call.sin), C.byref(call.sout),
                                   sel.ctypes.data_as(C.POINTER(C.c_int32)), len(sel))
    else:
        rc = lib.c2o_fp_step(C.byref(g), C.byref(fc), C.byref(call.sin), C.byref(call.sout))
    if rc != 0:
        raise RuntimeError("c2o_fp_step failed: %d" % rc)
    return call.result()


def obs_bin(binning, events: np.ndarray, flavor: str = "ref"):
    """The tools' per-event loop (oracle/c2d_obs_oracle.c) in event order:
    (F, F2, count) each [n_t, n_mu, n_e]."""
    lib = load(flavor)
    lib.c2o_obs_bin.restype = C.c_int
    lib.c2o_obs_bin.argtypes = [C.POINTER(abi.ObsBins), C.POINTER(C.c_double), C.c_int64] + \
        [C.POINTER(C.c_double)] * 3
    b = binning.to_ctypes()
    ev = np.ascontiguousarray(events, np.float64).reshape(-1, abi.EVENT_WORDS)
    shape = (binning.n_t, binning.n_mu, binning.n_e)
    F, F2, cnt = (np.zeros(shape) for _ in range(3))
    rc = lib.c2o_obs_bin(C.byref(b), ev.ctypes.data_as(abi.PD), len(ev), F.ctypes.data_as(abi.PD),
                         F2.ctypes.data_as(abi.PD), cnt.ctypes.data_as(abi.PD))
    if rc != 0:
        raise RuntimeError("c2o_obs_bin failed: %d" % rc)
    return F, F2, cnt


def volume_em(gnt, f_nt, T_keV, ne, B, l_min, flavor: str = "ref"):
    """One cell of volume_em (oracle/c2d_vem_oracle.c): kappa, eps_tot,
    eps_th [400], Eloss_cy, Eloss_th (raw sums)."""
    lib = load(flavor)
    P = C.POINTER(C.c_double)
    lib.c2o_volume_em.restype = None
    lib.c2o_volume_em.argtypes = [P, P] + [C.c_double] * 4 + [P] * 5
    g = np.ascontiguousarray(gnt, np.float64)
    f = np.ascontiguousarray(f_nt, np.float64)
    kap, et, eh = (np.zeros(abi.N_VOL) for _ in range(3))
    ecy, eth = C.c_double(), C.c_double()
    lib.c2o_volume_em(g.ctypes.data_as(P), f.ctypes.data_as(P), T_keV, ne, B, l_min,
                      kap.ctypes.data_as(P), et.ctypes.data_as(P), eh.ctypes.data_as(P),
                      C.byref(ecy), C.byref(eth))
    return kap, et, eh, ecy.value, eth.value


def vem_grid(flavor: str = "ref") -> np.ndarray:
    lib = load(flavor)
    e = np.zeros(abi.N_VOL)
    lib.c2o_vem_grid.argtypes = [C.POINTER(C.c_double)]
    lib.c2o_vem_grid(e.ctypes.data_as(C.POINTER(C.c_double)))
    return e


def vem_step(grid: abi.GridConfig, dt: float, state: dict, flavor: str = "det") -> dict:
    """imcgen2d's per-cell loop (oracle c2o_vem_step) over dense state arrays."""
    lib = load(flavor)
    lib.c2o_vem_step.restype = C.c_int
    lib.c2o_vem_step.argtypes = [C.POINTER(abi.Config), C.POINTER(abi.VemIn), C.POINTER(abi.VemOut)]
    g = grid.to_ctypes()
    call = abi.VemCall(dt, state)
    rc = lib.c2o_vem_step(C.byref(g), C.byref(call.sin), C.byref(call.sout))
    if rc != 0:
        raise RuntimeError("c2o_vem_step failed: %d" % rc)
    return call.res
