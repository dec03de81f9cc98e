"""Host-side mirror of the reference's per-step transport interface.

The reference runs, each Monte-Carlo time step (src/xec2d.f:67-87):

    imcgen2d   -> budgets + tables          (host side here: StepInputs)
    imcfield2d -> census transport          \\
    imcvol2d   -> volume-source transport    > Engine.transport_step()
    imcsurf2d  -> surface-source transport  /   (one C-ABI call, c2d_transport_step)
    imcredist  -> census rebalance          (not needed: census stays on its GPU)
    xec_add / graphics_collect / cens_add_up -> Engine.allreduce_tallies()

`Engine` owns one c2d context (one GPU).  Errors raise `C2DError` carrying
the library's message (the reference `stop`s instead).  The HIP library is
required: there is no CPU fallback on the product path.
"""
from __future__ import annotations

import ctypes as C
from pathlib import Path
from typing import Optional

import numpy as np

from . import abi

import os

# C2D_LIBRARY selects an alternative build of the same library (tuning sweeps)
LIB_PATH = Path(os.environ.get("C2D_LIBRARY") or
                Path(__file__).resolve().parent / "libcompton2d.so")
_lib = None


class C2DError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__("%s (%d): %s" % (abi.ERRORS.get(code, "C2D_E_?"), code, msg))
        self.code = code


def load_library(path: Optional[Path] = None) -> C.CDLL:
    """Load libcompton2d.so (built by `make -C compton2d_amd/csrc`); raise if absent."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = Path(path) if path else LIB_PATH
    if not p.exists():
        raise RuntimeError(
            "compton2d_amd: HIP library %s is missing; build it with "
            "`make -C compton2d_amd/csrc` (hipcc --offload-arch=gfx950)" % p)
    lib = C.CDLL(str(p))
    vp = C.c_void_p
    lib.c2d_version.restype = C.c_char_p
    lib.c2d_init.restype = C.c_int
    lib.c2d_init.argtypes = [C.POINTER(abi.Config), C.POINTER(vp)]
    lib.c2d_finalize.argtypes = [vp]
    lib.c2d_last_error.restype = C.c_char_p
    lib.c2d_last_error.argtypes = [vp]
    for fn in ("c2d_transport_step", "c2d_set_step"):
        getattr(lib, fn).restype = C.c_int
        getattr(lib, fn).argtypes = [vp, C.POINTER(abi.StepIn)]
    lib.c2d_set_clock.restype = C.c_int
    lib.c2d_set_clock.argtypes = [vp, C.c_int32, C.c_double, C.c_double]
    lib.c2d_run_step.restype = C.c_int
    lib.c2d_run_step.argtypes = [vp]
    lib.c2d_set_tally_buffer.restype = C.c_int
    lib.c2d_set_tally_buffer.argtypes = [vp, C.c_void_p]
    lib.c2d_tally_layout_get.restype = C.c_int
    lib.c2d_tally_layout_get.argtypes = [vp, C.POINTER(abi.TallyLayout)]
    lib.c2d_tally_device_ptr.restype = C.c_void_p
    lib.c2d_tally_device_ptr.argtypes = [vp]
    lib.c2d_tally_download.restype = C.c_int
    lib.c2d_tally_download.argtypes = [vp, C.POINTER(C.c_double), C.c_int64]
    lib.c2d_tally_download_range.restype = C.c_int
    lib.c2d_tally_download_range.argtypes = [vp, C.POINTER(C.c_double), C.c_int64, C.c_int64]
    lib.c2d_events.restype = C.c_int
    lib.c2d_events.argtypes = [vp, C.POINTER(C.c_double), C.c_int64, C.POINTER(C.c_int64)]
    lib.c2d_census_count.restype = C.c_int
    lib.c2d_census_count.argtypes = [vp, C.POINTER(C.c_int64)]
    lib.c2d_census_export.restype = C.c_int
    lib.c2d_census_export.argtypes = [vp, C.POINTER(C.c_double), C.POINTER(C.c_int32),
                                      C.POINTER(C.c_uint64), C.c_int64, C.POINTER(C.c_int64)]
    lib.c2d_census_export_range.restype = C.c_int
    lib.c2d_census_export_range.argtypes = [vp, C.c_int64, C.c_int64, C.POINTER(C.c_double),
                                            C.POINTER(C.c_int32), C.POINTER(C.c_uint64), C.c_int64,
                                            C.POINTER(C.c_int64)]
    lib.c2d_census_pack.restype = C.c_int
    lib.c2d_census_pack.argtypes = [vp, C.c_int64, C.c_int64, C.c_void_p]
    lib.c2d_census_append.restype = C.c_int
    lib.c2d_census_append.argtypes = [vp, C.c_void_p, C.c_int64]
    lib.c2d_census_truncate.restype = C.c_int
    lib.c2d_census_truncate.argtypes = [vp, C.c_int64]
    lib.c2d_census_import.restype = C.c_int
    lib.c2d_census_import.argtypes = [vp, C.POINTER(C.c_double), C.POINTER(C.c_int32),
                                      C.POINTER(C.c_uint64), C.c_int64]
    lib.c2d_fp_tridag.restype = C.c_int
    lib.c2d_fp_tridag.argtypes = [vp, C.POINTER(abi.FpIn), C.POINTER(C.c_double)]
    lib.c2d_selftest_math.restype = C.c_int
    lib.c2d_selftest_math.argtypes = [C.c_int, C.c_int, C.POINTER(C.c_double),
                                      C.POINTER(C.c_double), C.c_int64]
    lib.c2d_selftest_geom.restype = C.c_int
    lib.c2d_selftest_geom.argtypes = [C.c_int, C.c_int, C.POINTER(C.c_double),
                                      C.POINTER(C.c_double), C.c_int64]
    lib.c2d_last_gen0_steps.restype = C.c_int
    lib.c2d_last_gen0_steps.argtypes = [vp, C.POINTER(C.c_int64)]
    lib.c2d_last_path_steps.restype = C.c_int
    lib.c2d_last_path_steps.argtypes = [vp, C.POINTER(C.c_int64), C.POINTER(C.c_int64)]
    lib.c2d_last_compaction.restype = C.c_int
    lib.c2d_last_compaction.argtypes = [vp, C.POINTER(C.c_int32), C.POINTER(C.c_int64),
                                        C.POINTER(C.c_int64)]
    lib.c2d_last_census_chunks.restype = C.c_int
    lib.c2d_last_census_chunks.argtypes = [vp] + [C.POINTER(C.c_int64)] * 4
    lib.c2d_last_kernel_ms.restype = C.c_int
    lib.c2d_last_kernel_ms.argtypes = [vp, C.POINTER(C.c_double), C.POINTER(C.c_double),
                                       C.POINTER(C.c_int32)]
    lib.c2d_transport_prof.restype = C.c_int
    lib.c2d_transport_prof.argtypes = [vp, C.POINTER(C.c_uint64), C.c_int32]
    lib.c2d_fp_set_config.restype = C.c_int
    lib.c2d_fp_set_config.argtypes = [vp, C.POINTER(abi.FpConfig)]
    lib.c2d_fp_step.restype = C.c_int
    lib.c2d_fp_step.argtypes = [vp, C.POINTER(abi.FpStepIn), C.POINTER(abi.FpStepOut)]
    lib.c2d_fp_set_mode.restype = C.c_int
    lib.c2d_fp_set_mode.argtypes = [vp, C.c_int32]
    lib.c2d_last_fp_mode.restype = C.c_int
    lib.c2d_last_fp_mode.argtypes = [vp, C.POINTER(C.c_int32)]
    lib.c2d_last_fp_ms.restype = C.c_int
    lib.c2d_last_fp_ms.argtypes = [vp, C.POINTER(C.c_double)]
    lib.c2d_volume_em.restype = C.c_int
    lib.c2d_volume_em.argtypes = [vp, C.POINTER(abi.VemIn), C.POINTER(abi.VemOut)]
    lib.c2d_last_vem_ms.restype = C.c_int
    lib.c2d_last_vem_ms.argtypes = [vp, C.POINTER(C.c_double)]
    lib.c2d_obs_begin.restype = C.c_int
    lib.c2d_obs_begin.argtypes = [vp, C.POINTER(abi.ObsBins)]
    lib.c2d_obs_accumulate.restype = C.c_int
    lib.c2d_obs_accumulate.argtypes = [vp, C.POINTER(C.c_double), C.c_int64]
    lib.c2d_obs_accumulate_device.restype = C.c_int
    lib.c2d_obs_accumulate_device.argtypes = [vp, C.c_void_p, C.c_int64]
    lib.c2d_obs_result.restype = C.c_int
    lib.c2d_obs_result.argtypes = [vp] + [C.POINTER(C.c_double)] * 4
    lib.c2d_obs_begin_pspt.restype = C.c_int
    lib.c2d_obs_begin_pspt.argtypes = [vp, C.c_char_p]
    lib.c2d_obs_write_pspt.restype = C.c_int
    lib.c2d_obs_write_pspt.argtypes = [vp, C.c_char_p, C.c_int32, C.c_int32]
    lib.c2d_electron_state.restype = C.c_int
    lib.c2d_electron_state.argtypes = [vp, abi.MArray3, abi.MArray3]
    lib.c2d_comm_unique_id.restype = C.c_int
    lib.c2d_comm_unique_id.argtypes = [C.c_void_p, C.c_int64]
    lib.c2d_comm_init.restype = C.c_int
    lib.c2d_comm_init.argtypes = [vp, C.c_void_p, C.c_int32, C.c_int32]
    lib.c2d_allreduce_tallies.restype = C.c_int
    lib.c2d_allreduce_tallies.argtypes = [vp]
    if path is None:
        _lib = lib
    return lib


class Engine:
    """One GPU's transport context (c2d_ctx)."""

    def __init__(self, grid: abi.GridConfig, lib_path: Optional[Path] = None):
        self.lib = load_library(lib_path)
        self.grid = grid
        self._cfg = grid.to_ctypes()
        ctx = C.c_void_p()
        rc = self.lib.c2d_init(C.byref(self._cfg), C.byref(ctx))
        self.ctx = ctx
        if rc != 0:
            msg = self.lib.c2d_last_error(ctx).decode() if ctx.value else "c2d_init rejected config"
            if ctx.value:
                self.lib.c2d_finalize(ctx)
            self.ctx = None
            raise C2DError(rc, msg)
        L = abi.TallyLayout()
        self._check(self.lib.c2d_tally_layout_get(self.ctx, C.byref(L)))
        self.layout = L
        self.nz, self.nr, self.nmu = grid.nz, grid.nr, int(np.asarray(grid.mu).size)
        self._tally_tensor = None

    # -- lifecycle -------------------------------------------------------
    def close(self) -> None:
        if getattr(self, "ctx", None):
            self.lib.c2d_finalize(self.ctx)
            self.ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def _check(self, rc: int) -> None:
        if rc != 0:
            raise C2DError(rc, self.lib.c2d_last_error(self.ctx).decode())

    # -- the step ------------------------------------------------------------
    def set_step(self, si: abi.StepInputs) -> None:
        self._si = si.to_ctypes()
        self._check(self.lib.c2d_set_step(self.ctx, C.byref(self._si)))

    def set_clock(self, ncycle: int, time: float, dt: float) -> None:
        self._check(self.lib.c2d_set_clock(self.ctx, int(ncycle), float(time), float(dt)))

    def run_step(self) -> None:
        self._check(self.lib.c2d_run_step(self.ctx))

    def transport_step(self, si: abi.StepInputs) -> None:
        """imcfield2d + imcvol2d + imcsurf2d of one time step."""
        self.set_step(si)
        self.run_step()

    # -- tallies -------------------------------------------------------------
    def use_tally_tensor(self, tensor) -> None:
        """Write tallies into a caller-owned device tensor (float64, >= layout.total)."""
        assert tensor.dtype.itemsize == 8 and tensor.numel() >= self.layout.total
        self._tally_tensor = tensor
        self._check(self.lib.c2d_set_tally_buffer(self.ctx, C.c_void_p(tensor.data_ptr())))

    def tallies_raw(self) -> np.ndarray:
        out = np.zeros(self.layout.total, np.float64)
        self._check(self.lib.c2d_tally_download(
            self.ctx, out.ctypes.data_as(C.POINTER(C.c_double)), out.size))
        return out

    def tally_range(self, offset: int, n: int) -> np.ndarray:
        """Tally words [offset, offset + n) of the fused buffer (c2d_tally_download_range)."""
        out = np.zeros(n, np.float64)
        self._check(self.lib.c2d_tally_download_range(
            self.ctx, out.ctypes.data_as(C.POINTER(C.c_double)), int(offset), int(n)))
        return out

    def tallies(self) -> dict:
        return abi.split_tallies(self.tallies_raw(), self.nz, self.nr, self.nmu)

    def last_event_count(self) -> int:
        """Escape events the last transport step wrote (c2d_events with no buffer)."""
        n = C.c_int64()
        self._check(self.lib.c2d_events(self.ctx, None, 0, C.byref(n)))
        return n.value

    def events(self) -> np.ndarray:
        n = C.c_int64()
        self._check(self.lib.c2d_events(self.ctx, None, 0, C.byref(n)))
        out = np.zeros((max(n.value, 1), abi.EVENT_WORDS))
        self._check(self.lib.c2d_events(self.ctx, out.ctypes.data_as(C.POINTER(C.c_double)),
                                        n.value, C.byref(n)))
        return out[:n.value]

    def census_count(self) -> int:
        n = C.c_int64()
        self._check(self.lib.c2d_census_count(self.ctx, C.byref(n)))
        return n.value

    def census(self):
        n = self.census_count()
        d6 = np.zeros((max(n, 1), 6))
        i5 = np.zeros((max(n, 1), 5), np.int32)
        keys = np.zeros(max(n, 1), np.uint64)
        m = C.c_int64()
        self._check(self.lib.c2d_census_export(
            self.ctx, d6.ctypes.data_as(C.POINTER(C.c_double)),
            i5.ctypes.data_as(C.POINTER(C.c_int32)), keys.ctypes.data_as(C.POINTER(C.c_uint64)),
            n, C.byref(m)))
        return d6[:n], i5[:n], keys[:n]

    def census_sample(self, first: int, stride: int, cap: int):
        """Census records first, first+stride, ... (at most cap)."""
        n = C.c_int64()
        self._check(self.lib.c2d_census_export_range(self.ctx, first, stride, None, None, None, 0,
                                                     C.byref(n)))
        m = min(cap, n.value)
        d6 = np.zeros((max(m, 1), 6))
        i5 = np.zeros((max(m, 1), 5), np.int32)
        keys = np.zeros(max(m, 1), np.uint64)
        self._check(self.lib.c2d_census_export_range(
            self.ctx, first, stride, d6.ctypes.data_as(C.POINTER(C.c_double)),
            i5.ctypes.data_as(C.POINTER(C.c_int32)), keys.ctypes.data_as(C.POINTER(C.c_uint64)),
            m, C.byref(n)))
        return d6[:m], i5[:m], keys[:m]

    # -- device-resident census records (C2D_CENSUS_REC_WORDS u64 each) ------
    def census_pack(self, first: int, n: int, d_ptr: int) -> None:
        """Pack records [first, first+n) into device memory at d_ptr."""
        self._check(self.lib.c2d_census_pack(self.ctx, int(first), int(n), C.c_void_p(d_ptr)))

    def census_append(self, d_ptr: int, n: int) -> None:
        """Append n packed records from device memory at d_ptr."""
        self._check(self.lib.c2d_census_append(self.ctx, C.c_void_p(d_ptr), int(n)))

    def census_truncate(self, n: int) -> None:
        self._check(self.lib.c2d_census_truncate(self.ctx, int(n)))

    def import_census(self, d6, i5, keys) -> None:
        d6 = np.ascontiguousarray(d6, np.float64)
        i5 = np.ascontiguousarray(i5, np.int32)
        keys = np.ascontiguousarray(keys, np.uint64)
        self._check(self.lib.c2d_census_import(
            self.ctx, d6.ctypes.data_as(C.POINTER(C.c_double)),
            i5.ctypes.data_as(C.POINTER(C.c_int32)), keys.ctypes.data_as(C.POINTER(C.c_uint64)),
            len(keys)))

    def save_census(self, path) -> int:
        """Checkpoint the device census as a reference record file
        (write_cens, src/census2d.f:1-36) + `<path>.keys`; returns the count."""
        from . import census_io
        d6, i5, keys = self.census()
        census_io.write_census(path, d6, i5, keys)
        return len(keys)

    def load_census(self, path) -> int:
        """Restart from a census record file (read_cens, src/census2d.f:40-76)."""
        from . import census_io
        d6, i5, keys = census_io.read_census(path)
        self.import_census(d6, i5, keys)
        return len(keys)

    def last_kernel_ms(self):
        """(generation-0 kernel ms, all launches ms, launches) of the last step (HIP events)."""
        g0, al, nl = C.c_double(), C.c_double(), C.c_int32()
        self._check(self.lib.c2d_last_kernel_ms(self.ctx, C.byref(g0), C.byref(al), C.byref(nl)))
        return g0.value, al.value, nl.value

    def transport_prof(self) -> np.ndarray:
        """Section counters of the last step's transport launches (zeros unless
        the library was built with -DC2D_TR_PROF; tools/tr_prof.py)."""
        out = (C.c_uint64 * abi.TR_PROF_WORDS)()
        self._check(self.lib.c2d_transport_prof(self.ctx, out, abi.TR_PROF_WORDS))
        return np.array(out[:], dtype=np.uint64)

    def last_gen0_steps(self) -> int:
        n = C.c_int64()
        self._check(self.lib.c2d_last_gen0_steps(self.ctx, C.byref(n)))
        return n.value

    def last_path_steps(self) -> tuple[int, int]:
        """(generation-0, all launches) lane path-steps of the last step: a
        probe bundle's shared step counts once for all its copies."""
        g0, al = C.c_int64(), C.c_int64()
        self._check(self.lib.c2d_last_path_steps(self.ctx, C.byref(g0), C.byref(al)))
        return g0.value, al.value

    def last_compaction(self) -> tuple[int, int, int]:
        """(rounds, records moved, physical slots) of the last step's census
        close: the dead-tail compaction (double-buffered) or the packing of
        the partly filled chunks (chunked) (c2d_last_compaction)."""
        r, m, ph = C.c_int32(), C.c_int64(), C.c_int64()
        self._check(self.lib.c2d_last_compaction(self.ctx, C.byref(r), C.byref(m), C.byref(ph)))
        return r.value, m.value, ph.value

    def last_census_chunks(self) -> tuple[int, int, int, int]:
        """Chunked census: (chunks in the census, chunks recycled within the
        last step, census chunks not counted down, chunks held)
        (c2d_last_census_chunks); zeros when double-buffered."""
        v = [C.c_int64() for _ in range(4)]
        self._check(self.lib.c2d_last_census_chunks(self.ctx, *[C.byref(x) for x in v]))
        return tuple(x.value for x in v)

    # -- Fokker-Planck -------------------------------------------------------
    def fp_set_config(self, const: abi.FpConstants) -> None:
        """FP_calc run constants + F_IC (replaces setup_bcast / FP_bcast)."""
        self._fpc = const.to_ctypes()
        self._check(self.lib.c2d_fp_set_config(self.ctx, C.byref(self._fpc)))

    def fp_set_mode(self, mode: int) -> None:
        """abi.FP_EXACT (bit for bit the reference order, default),
        abi.FP_FAST (block-parallel sums, PCR tridag, tree-summed McDonald
        series: equal within rounding) or abi.FP_AUTO (per update: exact while
        every zone sits on the tea clamp within a few sub-steps, fast
        otherwise); include/compton2d.h c2d_fp_set_mode."""
        self._check(self.lib.c2d_fp_set_mode(self.ctx, int(mode)))

    def last_fp_mode(self) -> int:
        """abi.FP_EXACT or abi.FP_FAST: what the last fp_step ran (-1: none yet)."""
        m = C.c_int32()
        self._check(self.lib.c2d_last_fp_mode(self.ctx, C.byref(m)))
        return m.value

    def fp_step(self, ncycle: int, time: float, dt: float, inputs: dict, state: dict) -> dict:
        """One `update` (src/update2d.f:7-327) on the GPU; returns the new state.

        inputs['n_field'] / inputs['ecens'] set to None read the context's
        (all-reduced) tally buffer on the device instead of host arrays."""
        call = abi.FpCall(ncycle, time, dt, inputs, state)
        self._check(self.lib.c2d_fp_step(self.ctx, C.byref(call.sin), C.byref(call.sout)))
        return call.result()

    def last_fp_ms(self) -> float:
        ms = C.c_double()
        self._check(self.lib.c2d_last_fp_ms(self.ctx, C.byref(ms)))
        return ms.value

    def electron_state(self):
        """The context's device electron state (f_nt, Pnt), each [nz, nr, NUM_NT]."""
        f = np.zeros((self.nz, self.nr, abi.NUM_NT))
        p = np.zeros_like(f)
        mv = lambda a: abi.MArray3(a.ctypes.data_as(abi.PD), 1, self.nr * abi.NUM_NT, abi.NUM_NT)
        self._check(self.lib.c2d_electron_state(self.ctx, mv(f), mv(p)))
        return f, p

    # -- RCCL tally all-reduce (xec_add / cens_add_up over xGMI) --------------
    @staticmethod
    def comm_unique_id() -> bytes:
        lib = load_library()
        buf = C.create_string_buffer(abi.COMM_ID_BYTES)
        rc = lib.c2d_comm_unique_id(buf, abi.COMM_ID_BYTES)
        if rc != 0:
            raise C2DError(rc, "c2d_comm_unique_id failed")
        return buf.raw

    def comm_init(self, uid: bytes, rank: int, world: int) -> None:
        buf = C.create_string_buffer(bytes(uid), abi.COMM_ID_BYTES)
        self._check(self.lib.c2d_comm_init(self.ctx, buf, int(rank), int(world)))

    def allreduce_tallies(self) -> None:
        """One in-place RCCL all-reduce of the fused tally buffer."""
        self._check(self.lib.c2d_allreduce_tallies(self.ctx))

    # -- emission / absorption tables (imcgen2d.f:209-333, volume_em) ---------
    def volume_em(self, dt: float, state: dict, tables_to_host: bool = True) -> dict:
        """kappa_tot, eps_tot, eps_th [nz, nr, 400], B_field, Eloss_sy/cy/th/tot
        [nz, nr] and E_ph [400] for the cell state (tea, tna, n_e, B_field,
        f_pair, zsurf, vol [nz, nr], f_nt [nz, nr, 200], ep_switch).
        f_nt None: the device electron state; tables_to_host False: the three
        tables stay on the device for set_step(kappa_tot=None, ...)."""
        call = abi.VemCall(dt, state, tables_to_host)
        self._check(self.lib.c2d_volume_em(self.ctx, C.byref(call.sin), C.byref(call.sout)))
        return call.res

    def last_vem_ms(self) -> float:
        ms = C.c_double()
        self._check(self.lib.c2d_last_vem_ms(self.ctx, C.byref(ms)))
        return ms.value

    # -- observer-frame binning (postprocessing/pspt.c, plcm.c) ---------------
    def obs_begin(self, binning) -> None:
        """Zero a device histogram for `binning` (observer.Binning)."""
        self._obs = binning
        self._obs_c = binning.to_ctypes()
        self._check(self.lib.c2d_obs_begin(self.ctx, C.byref(self._obs_c)))

    def obs_accumulate(self, events=None) -> None:
        """Bin host events [n, 7] (t_bound, xnu, ew, rpre, zpre, wmu, phi), or
        with None the last transport step's device event buffer."""
        if events is None:
            self._check(self.lib.c2d_obs_accumulate(self.ctx, None, 0))
            return
        ev = np.ascontiguousarray(events, np.float64).reshape(-1, abi.EVENT_WORDS)
        self._check(self.lib.c2d_obs_accumulate(self.ctx, ev.ctypes.data_as(abi.PD), len(ev)))

    def obs_accumulate_device(self, ptr: int, n: int) -> None:
        """Bin n events at device address `ptr` (e.g. tensor.data_ptr() of a
        cuda float64 [n, 7] tensor on this context's GPU)."""
        self._check(self.lib.c2d_obs_accumulate_device(self.ctx, C.c_void_p(ptr), n))

    def obs_result(self):
        """Raw sums (F = sum ew, F2 = sum ew^2, count), each [n_t, n_mu, n_e],
        and the device milliseconds of the binning launches so far."""
        b = self._obs
        shape = (b.n_t, b.n_mu, b.n_e)
        F, F2, cnt = (np.zeros(shape) for _ in range(3))
        ms = C.c_double()
        self._check(self.lib.c2d_obs_result(self.ctx, F.ctypes.data_as(abi.PD),
                                            F2.ctypes.data_as(abi.PD),
                                            cnt.ctypes.data_as(abi.PD), C.byref(ms)))
        return F, F2, cnt, ms.value

    def obs_begin_pspt(self, deck: str = "") -> None:
        """The SED binning of pspt's input dialogue `deck` (c2d_obs_begin_pspt)."""
        from . import observer
        self._check(self.lib.c2d_obs_begin_pspt(self.ctx, deck.encode()))
        self._obs = observer.parse_pspt_deck(deck)

    def obs_write_pspt(self, path: str = "", factor: int = 0, world_sum: bool = False) -> None:
        """Write pspt's output file from the histogram so far (c2d_obs_write_pspt)."""
        self._check(self.lib.c2d_obs_write_pspt(self.ctx, str(path).encode(), int(factor), int(world_sum)))

    def fp_tridag(self, a, b, c, r, x0=None) -> np.ndarray:
        """Batched tridag (src/update2d.f:2476-2518); arrays [ncell, nt]."""
        a, b, c, r = (np.ascontiguousarray(x, np.float64) for x in (a, b, c, r))
        ncell, nt = a.shape
        x = np.zeros_like(a) if x0 is None else np.array(x0, np.float64, copy=True)
        fin = abi.FpIn(ncell, a.ctypes.data_as(abi.PD), b.ctypes.data_as(abi.PD),
                       c.ctypes.data_as(abi.PD), r.ctypes.data_as(abi.PD), nt)
        self._check(self.lib.c2d_fp_tridag(self.ctx, C.byref(fin), x.ctypes.data_as(abi.PD)))
        return x


def obs_engine(device: int = 0) -> Engine:
    """A context for observer-frame binning only (no transport tables used)."""
    from . import synth
    g = synth.c2_workload(nz=1, nr=1, sources=1, device=device, census_capacity=1024,
                          event_capacity=1024).grid
    g.queue_capacity = 1024
    return Engine(g)


def device_mcdonald(z: np.ndarray, device: int = 0):
    """K2(z), K3(z) by the GPU's wave-level McDonald series and the shader
    cycles of each evaluation (c2d_selftest_mcdonald)."""
    lib = load_library()
    lib.c2d_selftest_mcdonald.restype = C.c_int
    lib.c2d_selftest_mcdonald.argtypes = [C.c_int, C.POINTER(C.c_double), C.c_int, C.POINTER(C.c_double)]
    z = np.ascontiguousarray(z, np.float64)
    out = np.zeros((len(z), 3))
    rc = lib.c2d_selftest_mcdonald(device, z.ctypes.data_as(abi.PD), len(z), out.ctypes.data_as(abi.PD))
    if rc != 0:
        raise C2DError(rc, "c2d_selftest_mcdonald failed")
    return out[:, 0], out[:, 1], out[:, 2]


def device_mcd_fast(z: np.ndarray, device: int = 0) -> np.ndarray:
    """The fast FP kernel's McDonald pair at z from its moment table and from
    its term-by-term series (c2d_selftest_mcd_fast): rows (K2, K3 table, K2,
    K3 series, table answered, cycles of the table's gamma_bar, cycles of the
    series, gamma_bar from the table as the fast kernel forms it)."""
    lib = load_library()
    lib.c2d_selftest_mcd_fast.restype = C.c_int
    lib.c2d_selftest_mcd_fast.argtypes = [C.c_int, C.POINTER(C.c_double), C.c_int, C.POINTER(C.c_double)]
    z = np.ascontiguousarray(z, np.float64)
    out = np.zeros((len(z), 8))
    rc = lib.c2d_selftest_mcd_fast(device, z.ctypes.data_as(abi.PD), len(z), out.ctypes.data_as(abi.PD))
    if rc != 0:
        raise C2DError(rc, "c2d_selftest_mcd_fast failed")
    return out


def device_geom(nr: int, rays: np.ndarray, device: int = 0) -> np.ndarray:
    """(disbr, trldb) of the flight step's r-boundary distance for rays
    (rpre, Eta, wmu, rbnd) on the GPU, with the fast build's sqrt / reciprocal
    after `nr` Newton steps, or IEEE (nr = 0) (c2d_selftest_geom)."""
    lib = load_library()
    rays = np.ascontiguousarray(rays, np.float64).reshape(-1, 4)
    out = np.zeros((rays.shape[0], 2))
    rc = lib.c2d_selftest_geom(device, nr, rays.ctypes.data_as(abi.PD), out.ctypes.data_as(abi.PD),
                               rays.shape[0])
    if rc != 0:
        raise C2DError(rc, "c2d_selftest_geom failed")
    return out


def device_math(fn: int, x: np.ndarray, device: int = 0) -> np.ndarray:
    """Evaluate c2d_math function `fn` on the GPU (c2d_selftest_math)."""
    lib = load_library()
    x = np.ascontiguousarray(x, np.float64)
    y = np.zeros_like(x)
    rc = lib.c2d_selftest_math(device, fn, x.ctypes.data_as(abi.PD), y.ctypes.data_as(abi.PD),
                               x.size)
    if rc != 0:
        raise C2DError(rc, "c2d_selftest_math failed")
    return y
